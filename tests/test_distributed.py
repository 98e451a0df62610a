"""Multi-process film sharding (the N>1 path of bench.py) on CPU with gloo, world_size 2:
each rank renders its row stripes, one sum-reduce of the film, result == single process.
Weak scaling (bench.py's default for N > 1) renders the job at spp x N; strong at spp."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, SCENES


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, scaling):
    import sys
    sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import pbrt_amd as pa
    import pyoracle
    from pbrt_amd.tiles import job_spp, reduce_film, rows_for_rank
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=40, yresolution=36, spp=job_spp(2, world, scaling))
    i = sc.info
    film = pyoracle.render(sc, rows=rows_for_rank(i.py0, i.py1, rank, world, block=4), threads=2)
    t = torch.from_numpy(film.reshape(-1).copy())
    reduce_film(t, dst=0)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_gloo_two_ranks_match_single(tmp_path, pa, oracle, scaling):
    out = tmp_path / "film.npy"
    mp.spawn(_worker, args=(2, _free_port(), str(out), scaling), nprocs=2, join=True)
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=40, yresolution=36, spp=4 if scaling == "weak" else 2)
    single = oracle.render(sc, threads=4).reshape(-1)
    np.testing.assert_array_equal(np.load(out), single)


def test_rows_partition_is_exact_cover():
    from pbrt_amd.tiles import rows_for_rank
    for world in (1, 2, 3, 8):
        got = np.sort(np.concatenate([rows_for_rank(5, 733, r, world) for r in range(world)]))
        np.testing.assert_array_equal(got, np.arange(5, 733))


def test_job_spp():
    from pbrt_amd.tiles import job_spp
    assert job_spp(64, 8) == 512 and job_spp(64, 8, "strong") == 64 and job_spp(64, 1) == 64
    with pytest.raises(ValueError):
        job_spp(64, 2, "both")
