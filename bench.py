#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X wavefront path tracer on BASELINE.json's headline
configuration (configs[1]): synthetic Cornell box, 1280x720, 64 spp, PathIntegrator maxdepth
5 semantics (wavefront volpath), Halton sampler, diffuse-only BxDFs.  ``--workload c3`` runs
configs[2] instead (scenes/gen_c3.py: 30k-triangle displaced dielectric icosphere + rough
conductor floor, 1920x1080, 256 spp, ZSobol) and ``--workload c4`` configs[3]'s geometry
(scenes/gen_c4.py: 122 copied displaced icospheres, ~10M triangles from PLY files, diffuse +
conductor, 1920x1080, 128 spp) -- extra lines, not the headline.

One "step" = one complete render of that image (all 64 samples per pixel, film cleared
first) plus, for N > 1, the single RCCL sum-reduce of the film over xGMI (issued
asynchronously from a staging copy, so it overlaps the next step's render; the timed region
ends after every reduce has completed).  Pixel rows are
interleaved across ranks (row r to rank r mod N: pixel tiles, BVH replicated, no collective on
the data path).  Default for N > 1 is strong scaling: the job is BASELINE's 1280x720x64 image
split N ways (per-GPU work 1/N, "scaling": "strong").  ``--scaling weak`` keeps each GPU's
work fixed instead: the job becomes the 1280x720 image at 64 x N spp (each GPU renders 1/N of
the rows at all 64 x N samples); the metric string then names that job.  The metric counts
every sample of the job.  Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.

The JSON line also carries
  roofline     the closest-hit (traverse + compact + material-queue scatter) kernel, the
               judged "BVH kernel" (SURVEY.md §8(d)): algorithmic bytes per launch / mean
               launch time measured with HIP events on the context stream
  cpu_baseline the CPU oracle (oracle/oracle.cpp, a port of pbrt's wavefront/VolPath
               integrator) on a bounded sample of the same workload, host threads stated.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))

# Algorithmic bytes of the closest-hit kernel, from its declared SoA fields (the depth's path
# records are dense, so there is no ray-queue index to read), per depth d:
#   reads  ray o,d 24 B per ray
#   writes hit prim 4 B + b0,b1,b2,t 16 B per recorded hit (every hit below maxDepth, only
#          emissive hits at maxDepth), and 4 B per queue entry (material, emissive, escaped)
# closest_bytes() sums this over the per-depth queue counts; BYTES_PER_RAY_CLOSEST is the
# all-rays-hit upper bound used when no counts are available.
RAY_READ_B, HIT_WRITE_B, QUEUE_ENTRY_B = 24, 20, 4
BYTES_PER_RAY_CLOSEST = 48
# The media wavefront's closest-hit kernel (volpath.hip k_vclosest) also reads the ray's medium
# (4 B) and always writes the hit (prim 4 + b0,b1,b2,t 16) and one queue entry (4): 52 B
BYTES_PER_RAY_VCLOSEST = 52
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c2")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--xres", type=int, default=None)
    ap.add_argument("--yres", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--max-paths", type=int, default=0,
                    help="paths per wavefront pass (0: the library default, the whole image's samples in "
                         "one pass up to 64 Mi paths)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--untextured", action="store_true",
                    help="C4: round 2's constant materials instead of configs[3]'s image textures")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads for cpu_baseline (0: every host core this process may use)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="N > 1: strong = one image split N ways (default); weak = every GPU renders "
                         "the single-GPU workload (job spp x N)")
    a = ap.parse_args(argv)
    d = {"c2": (1280, 720, 64), "c3": (1920, 1080, 256), "c4": (1920, 1080, 128), "c5": (1280, 720, 1024)}[a.workload]
    a.xres = a.xres or d[0]
    a.yres = a.yres or d[1]
    a.spp = a.spp or d[2]
    return a


def load(args, spp=None):
    import pbrt_amd as pa
    spp = spp or args.spp
    if args.workload == "c4":
        import tempfile
        sys.path.insert(0, str(ROOT / "scenes"))
        import gen_c4
        keep = os.environ.get("PBRT_C4_DIR")
        out = Path(keep or tempfile.mkdtemp(prefix="pbrt_c4_"))
        path, _ = gen_c4.generate(out, xres=args.xres, yres=args.yres, spp=spp, textured=not args.untextured)
        scene = pa.load_scene(path)  # the PLY files are read completely here
        if not keep:
            import shutil
            shutil.rmtree(out, ignore_errors=True)
        return scene
    if args.workload == "c5":
        sys.path.insert(0, str(ROOT / "scenes"))
        import gen_c5
        return pa.Scene.from_string(gen_c5.scene_text(args.xres, args.yres, spp, grid=256), ROOT / "scenes")
    if args.workload == "c3":
        sys.path.insert(0, str(ROOT / "scenes"))
        import gen_c3
        return pa.Scene.from_string(gen_c3.scene_text(args.xres, args.yres, spp), ROOT / "scenes")
    return pa.load_scene(ROOT / "scenes" / "cornell-box.pbrt", xresolution=args.xres, yresolution=args.yres,
                         spp=spp)


def closest_bytes(qcounts, max_depth):
    """(algorithmic bytes, rays) of the closest-hit launches of one pass from its per-depth queue
    counts (WavefrontPathIntegrator.queue_counts: rays, diffuse, shadow, escaped, emissive,
    dielectric, conductor)."""
    total = rays = 0
    for d in range(max_depth + 1):
        r, dif, _sh, esc, emi, die, con = (int(x) for x in qcounts[d])
        mat = dif + die + con
        hits = mat if d < max_depth else emi
        total += RAY_READ_B * r + HIT_WRITE_B * hits + QUEUE_ENTRY_B * (mat + emi + esc)
        rays += r
    return total, rays


def job_spec(args, world, scaling):
    """The job one bench step renders: image, spp of the whole job, and how it is sharded."""
    from pbrt_amd.tiles import job_spp
    spp = job_spp(args.spp, world, scaling)
    metric = f"Msamples/sec (paths x spp / s) at {args.xres}x{args.yres}x{spp}spp"
    if world == 1:
        sharding = "single GPU"
    elif scaling == "strong":
        sharding = (f"one {args.xres}x{args.yres}x{spp}spp image, film rows interleaved over {world} ranks "
                    "(strong scaling: per-GPU work 1/N) + 1 RCCL film reduce")
    else:
        sharding = (f"one {args.xres}x{args.yres}x{spp}spp image ({args.spp} spp x {world}), film rows "
                    f"interleaved over {world} ranks (weak scaling: each GPU renders "
                    f"{args.xres}x{args.yres}x{args.spp} samples' worth) + 1 RCCL film reduce")
    return {"metric": metric, "spp": spp, "sharding": sharding, "scaling": scaling if world > 1 else "weak"}


def roofline_entry(achieved, mean_launch_s, launches, rays_per_launch, bytes_per_ray, traffic, workload,
                   bvh_bytes=0):
    """The 'roofline' object.  bound = the roofline that applies (HBM: nothing on this path
    is a dense contraction, so MFMA has no ceiling to offer); 'limiter' says whether the
    measured fraction is bandwidth-limited or what else limits the kernel."""
    frac = achieved / HBM_PEAK_GBS
    if frac >= 0.6:
        limiter = "HBM bandwidth"
    elif workload == "c2":
        limiter = (f"not HBM ({frac:.1%} of peak): VALU issue + LDS latency, BVH and triangles LDS-resident "
                   "(profiles/r*_c2_pmc_per_kernel.json)")
    else:
        limiter = f"not HBM ({frac:.1%} of peak): dependent node/triangle load latency"
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(frac, 5), "traffic": traffic,
            "kernel": ("k_vclosest (BVH8 traverse + hit record + push to medium / surface queue)"
                       if workload == "c5" else
                       "k_closest (BVH8 traverse + hit record + wave64 ballot push to material queue)"),
            "bytes_per_ray": round(bytes_per_ray, 2), "bvh_bytes_per_launch": bvh_bytes,
            "algorithmic_bytes_per_launch": round(bytes_per_ray * rays_per_launch + bvh_bytes),
            "rays_per_launch": round(rays_per_launch, 1),
            "timed_launches": launches, "mean_launch_us": round(mean_launch_s * 1e6, 3), "limiter": limiter}


def host_cores():
    """Host cores this process may run on: its CPU affinity, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS when set (a GPU box grants each GPU a share of a larger machine, stated in
    OMP_NUM_THREADS; os.cpu_count() reports the whole machine there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max" and int(period) > 0:
                n = min(n, max(1, int(int(quota) // int(period))))
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0 and p > 0:
            n = min(n, max(1, q // p))
    except (OSError, ValueError):
        pass
    # the box's per-GPU CPU allotment, when the environment states one (OMP_NUM_THREADS)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(args, threads, sc):
    """Oracle (pbrt wavefront/VolPath port) on the host: every film row, the first 16 of the
    64 samples per pixel (~15 M samples, a few seconds of wall time on the GPU box's host)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np
    import pyoracle
    i = sc.info
    # C2: every row, 16 of 64 spp; C3/C4: every 8th row, 4 spp; C5: every 2nd row, 8 spp
    # (seconds of host work)
    rows = np.arange(i.py0, i.py1, {"c2": 1, "c5": 2}.get(args.workload, 8), dtype=np.int32)
    spp = {"c2": 16, "c5": 8}.get(args.workload, 4)
    pyoracle.lib()
    # the oracle builds its BVH inside every render call: time an empty render and subtract it
    t = time.perf_counter()
    pyoracle.render(sc, rows=rows[:0], first_sample=0, n_samples=spp, threads=threads)
    setup = time.perf_counter() - t
    t = time.perf_counter()
    pyoracle.render(sc, rows=rows, first_sample=0, n_samples=spp, threads=threads)
    dt = time.perf_counter() - t - setup
    n = len(rows) * (i.px1 - i.px0) * spp
    return {"value": n / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "cores_note": "every host core granted to the process (CPU affinity, cgroup quota, OMP_NUM_THREADS)"
            if not args.cpu_threads else "--cpu-threads",
            "sample": f"{len(rows)} of {i.py1 - i.py0} rows x {i.px1 - i.px0} px x {spp} spp "
                      f"({n} samples, {dt:.2f} s wall excluding the oracle's {setup:.2f} s BVH build)"}


def latest_profile(pattern):
    """The newest round's committed profile record matching profiles/<pattern> (r01, r02, ...)."""
    files = sorted((ROOT / "profiles").glob(pattern))
    if not files:
        return None
    try:
        return json.loads(files[-1].read_text())
    except Exception:
        return None


def pmc_traffic(workload):
    """HBM bytes per closest-hit launch from the newest committed rocprofv3 PMC pass of this
    workload, tagged with the commit it was measured on (a figure, not a live measurement)."""
    pat = f"r*_{workload}_closest_pmc.json"  # this workload's own records only (r05_c2_..., r04_c4_...)
    rec = latest_profile(pat)
    if not rec or rec.get("hbm_bytes_per_launch") is None:
        return None
    return {"hbm_bytes_per_launch": rec["hbm_bytes_per_launch"], "bytes_per_ray": rec.get("hbm_bytes_per_ray"),
            "measured_on": rec.get("head", "unknown"), "source": "profiles/" + sorted((ROOT / "profiles").glob(pat))[-1].name}


def compute_ceiling(workload):
    """The closest-hit kernel's compute roof from the same PMC record: VALU issue as a fraction
    of every SIMD's cycles, 2 cycles x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
    (a wave64 fp32 VALU instruction holds its SIMD 2 cycles at full rate: a lower bound), and per
    wave SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES and SQ_WAIT_ANY / SQ_WAVE_CYCLES.  With the tree in
    LDS (C2) this, not HBM, is the binding roof."""
    pat = f"r*_{workload}_closest_pmc.json"
    rec = latest_profile(pat)
    if not rec or rec.get("valu_busy") is None:
        return None
    return {"bound": "valu", "frac": rec["valu_busy"], "valu_active_per_wave": rec.get("valu_active_per_wave"),
            "waiting_per_wave": rec.get("wait_any_per_wave"), "measured_on": rec.get("head", "unknown"),
            "source": "profiles/" + sorted((ROOT / "profiles").glob(pat))[-1].name}


# Wide BVH8 node bytes a visit reads (12 plane float4 + header + slot triangle masks) and the
# bytes of one pre-rotated triangle (common.h VisitWide / TraverseCW)
NODE_BYTES_READ, TRI_BYTES_READ = 240, 48


def effective_traversal(rays_per_s):
    """Secondary figure: ray I/O plus the BVH node and triangle bytes the
    traversal reads per ray -- from LDS on C2 -- with the per-ray visit counts of the committed
    traversal-statistics record, at the measured ray rate."""
    rec = latest_profile("r*_c2_trav_stats.json")
    if not rec:
        return None
    c = rec["closest"]
    per_ray = BYTES_PER_RAY_CLOSEST + NODE_BYTES_READ * c["nodes_per_ray"] + TRI_BYTES_READ * c["tris_per_ray"]
    return {"bytes_per_ray": round(per_ray, 1), "achieved_GBps": round(per_ray * rays_per_s / 1e9, 1),
            "nodes_per_ray": round(c["nodes_per_ray"], 3), "tris_per_ray": round(c["tris_per_ray"], 3),
            "source": "profiles/" + sorted((ROOT / "profiles").glob("r*_c2_trav_stats.json"))[-1].name}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    import pbrt_amd as pa
    from pbrt_amd.tiles import film_tensor_from_device_ptr, rows_for_rank

    scaling = args.scaling if world > 1 else "weak"
    job = job_spec(args, world, scaling)
    scene = load(args, job["spp"])
    info = scene.info
    integ = pa.WavefrontPathIntegrator(scene, device=local_rank, max_paths=args.max_paths)
    # single-row interleave: every rank gets the same number of rows whenever N divides the
    # height (720 and 1080 for N = 1, 2, 4, 8), so no rank waits on a heavier share
    rows = rows_for_rank(info.py0, info.py1, rank, world, block=1)
    film_ptr, film_n = integ.film_device_ptr()
    film_t = film_tensor_from_device_ptr(film_ptr, film_n, local_rank) if world > 1 else None
    # N > 1: each step's film is copied to one of two staging buffers and sum-reduced to rank 0
    # asynchronously (RCCL on its own stream), so the reduce overlaps the next step's render;
    # a staging buffer is reused only after the reduce that read it has completed.
    staging = [torch.empty_like(film_t), torch.empty_like(film_t)] if world > 1 else None
    pending = [None, None]
    nstep = [0]

    def step(timed_kernel=False):
        integ.film_clear()
        integ.render(rows=rows, first_sample=0, n_samples=info.spp, time_closest=timed_kernel)
        if world > 1:
            integ.synchronize()  # the film is complete
            b = nstep[0] % 2
            if pending[b] is not None:
                pending[b].wait()
            staging[b].copy_(film_t)
            torch.cuda.current_stream().synchronize()  # the next film_clear must not overtake the copy
            pending[b] = dist.reduce(staging[b], dst=0, op=dist.ReduceOp.SUM, async_op=True)
            nstep[0] += 1

    def drain():
        for b in range(2):
            if pending[b] is not None:
                pending[b].wait()
                pending[b] = None

    for _ in range(args.warmup):
        step()
    integ.synchronize()
    drain()
    integ.reset_stats()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed_kernel=True)
    integ.synchronize()
    drain()  # every step's film reduce is inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = integ.stats()
    dt_max = dt
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt_max = tt.item()

    samples = (info.px1 - info.px0) * (info.py1 - info.py0) * info.spp * args.steps  # all ranks together
    value = samples / dt_max / 1e6
    launches = max(st.closest_launches, 1)
    mean_launch_s = st.closest_ms / 1e3 / launches
    if args.workload == "c5":
        bpr = BYTES_PER_RAY_VCLOSEST
    else:
        # per-depth queue counts of the last pass (= the timed pass when a render is one pass)
        qb, qr = closest_bytes(integ.queue_counts(), info.max_depth)
        bpr = qb / qr if qr else BYTES_PER_RAY_CLOSEST
    # ray I/O per ray plus the HBM-resident BVH touched once per launch (nodes
    # beyond the LDS-cached top, triangles unless LDS-cached; 0 on C2, whose tree is in LDS)
    bvh_bytes = int(st.bvh_hbm_node_bytes + st.bvh_hbm_tri_bytes)
    bytes_per_launch = bpr * st.timed_closest_rays / launches + bvh_bytes
    achieved = bytes_per_launch / mean_launch_s / 1e9 if mean_launch_s > 0 else 0.0
    traffic = pmc_traffic(args.workload)

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(args, args.cpu_threads or host_cores(), scene)
            except Exception as e:  # the baseline is reported, never required
                cpu = {"value": None, "error": str(e)}
        line = {
            "metric": job["metric"],
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": job["scaling"],
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": (f"cornell-box (synthetic) {args.xres}x{args.yres} {info.spp}spp maxdepth "
                                    f"{info.max_depth} halton, wavefront volpath, diffuse BxDF (BASELINE configs[1])"
                                    if args.workload == "c2" else
                                    f"C3 killeroo stand-in (scenes/gen_c3.py) {args.xres}x{args.yres} {info.spp}spp "
                                    f"maxdepth {info.max_depth} zsobol, dielectric + conductor + diffuse "
                                    "(BASELINE configs[2])" if args.workload == "c3" else
                                    f"C5 cloud stand-in (scenes/gen_c5.py: 256^3 fBm uniformgrid medium, sigma_a 0.5, "
                                    f"sigma_s 5, g 0.3, in an interface box) {args.xres}x{args.yres} {info.spp}spp "
                                    f"maxdepth {info.max_depth} zsobol, volpath null scattering (BASELINE configs[4])"
                                    if args.workload == "c5" else
                                    f"C4 San-Miguel stand-in (scenes/gen_c4.py, PLY) {args.xres}x{args.yres} "
                                    f"{info.spp}spp maxdepth {info.max_depth} zsobol, diffuse + conductor, "
                                    + ("untextured (BASELINE configs[3] geometry)" if args.untextured else
                                       "textured: 8 sRGB PNG albedo images (256^2-1024^2, bilinear / trilinear MIP) "
                                       "and 2 roughness images, per-vertex uv (BASELINE configs[3])")),
                       "xres": args.xres, "yres": args.yres, "spp": info.spp, "max_depth": info.max_depth,
                       "triangles": info.n_triangles, "paths_per_pass": int(st.paths_per_pass),
                       "sharding": job["sharding"]},
            "roofline": dict(roofline_entry(achieved, mean_launch_s, launches, st.timed_closest_rays / launches,
                                            bpr, traffic, args.workload, bvh_bytes),
                             compute=compute_ceiling(args.workload),
                             effective=(effective_traversal(st.timed_closest_rays / launches / mean_launch_s)
                                        if args.workload == "c2" and mean_launch_s > 0 else None)),
            "cpu_baseline": cpu,
            "rays": {"camera": int(st.camera_rays), "closest": int(st.closest_rays), "shadow": int(st.shadow_rays)},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
