"""Multi-process film sharding (the N>1 path of bench.py) on CPU with gloo, world_size 2:
each rank renders its row stripes, one sum-reduce of the film, result == single process.
Strong scaling (bench.py's default for N > 1) renders the job at spp; weak at spp x N.  The
bench line's metric / config must name the job the ranks actually rendered."""
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


def _bench_worker(rank, world, port, out_path, scaling):
    """bench.py's N > 1 job on the CPU: bench.job_spec decides the job, the ranks render it
    (oracle in place of the GPU library) and reduce the film; rank 0 records the line's fields."""
    import json
    import sys
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import bench
    import pbrt_amd as pa
    import pyoracle
    from pbrt_amd.tiles import reduce_film, rows_for_rank
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    argv = ["--gpus", str(world), "--xres", "32", "--yres", "24", "--spp", "2"]
    if scaling:
        argv += ["--scaling", scaling]
    args = bench.parse(argv)
    job = bench.job_spec(args, world, args.scaling if world > 1 else "weak")
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=args.xres, yresolution=args.yres, spp=job["spp"])
    i = sc.info
    rows = rows_for_rank(i.py0, i.py1, rank, world, block=1)
    film = pyoracle.render(sc, rows=rows, threads=2)
    t = torch.from_numpy(film.reshape(-1).copy())
    reduce_film(t, dst=0)
    n_rows = torch.tensor([len(rows)])
    dist.all_reduce(n_rows)
    if rank == 0:
        np.save(out_path + ".npy", t.numpy())
        rec = dict(job, rendered_spp=i.spp, rendered_rows=int(n_rows.item()), xres=i.xres, yres=i.yres)
        open(out_path + ".json", "w").write(json.dumps(rec))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scaling", [None, "weak"])
def test_bench_line_names_the_rendered_job(tmp_path, pa, oracle, scaling):
    import json
    out = str(tmp_path / "job")
    mp.spawn(_bench_worker, args=(2, _free_port(), out, scaling), nprocs=2, join=True)
    rec = json.loads(open(out + ".json").read())
    spp = 2 if scaling is None else 4  # default for N > 1 is strong scaling
    assert rec["scaling"] == ("strong" if scaling is None else "weak")
    assert rec["spp"] == rec["rendered_spp"] == spp
    assert rec["metric"] == f"Msamples/sec (paths x spp / s) at 32x24x{spp}spp"
    assert rec["rendered_rows"] == rec["yres"] == 24
    assert f"32x24x{spp}spp" in rec["sharding"]
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=32, yresolution=24, spp=spp)
    np.testing.assert_array_equal(np.load(out + ".npy"), oracle.render(sc, threads=4).reshape(-1))


def test_closest_bytes_from_queue_counts():
    import sys
    sys.path.insert(0, str(ROOT))
    import bench
    # columns: rays, diffuse, shadow, escaped, emissive, dielectric, conductor; maxdepth 1
    q = np.array([[100, 60, 0, 30, 5, 4, 1], [65, 0, 0, 20, 3, 0, 0]])
    total, rays = bench.closest_bytes(q, 1)
    # depth 0: 24*100 + 20*65 hits + 4*(65 + 5 + 30); depth 1: 24*65 + 20*3 emissive + 4*(0 + 3 + 20)
    assert rays == 165
    assert total == (2400 + 1300 + 400) + (1560 + 60 + 92)


def _gpu_worker(rank, world, port, out_path):
    """bench.py's N > 1 data path with the product: this rank renders its single-row interleave
    (rows_for_rank(block=1)) with libpbrt_amd on device 0, wraps the device film with
    film_tensor_from_device_ptr, and sum-reduces it (gloo, via the host) onto rank 0."""
    import sys
    sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
    import pbrt_amd as pa
    from pbrt_amd.tiles import film_tensor_from_device_ptr, reduce_film, rows_for_rank
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=96, yresolution=72, spp=8)
    i = sc.info
    integ = pa.WavefrontPathIntegrator(sc, device=0, max_paths=1 << 18)
    integ.film_clear()
    integ.render(rows=rows_for_rank(i.py0, i.py1, rank, world, block=1), first_sample=0, n_samples=i.spp)
    integ.synchronize()
    ptr, n = integ.film_device_ptr()
    t = film_tensor_from_device_ptr(ptr, n, 0).cpu()
    reduce_film(t, dst=0)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_product_film_equals_single_gpu(tmp_path, pa):
    """The product's multi-rank path once on the GPU: two ranks, each rendering every other film
    row with libpbrt_amd on device 0, their device films reduced -- the same bits as one
    process rendering the whole image (non-owned pixels are exact zeros)."""
    out = tmp_path / "film.npy"
    mp.spawn(_gpu_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=96, yresolution=72, spp=8)
    integ = pa.WavefrontPathIntegrator(sc, device=0, max_paths=1 << 18)
    integ.render()
    integ.synchronize()
    single = integ.film_raw().reshape(-1)
    got = np.load(out)
    assert np.abs(single).sum() > 0
    np.testing.assert_array_equal(got, single)
