"""Pixel-tile sharding of the film across GPUs.

Every path depends only on (pixel, sample index, dimension) (wavefront/samples.cpp:39-46,
camera.cpp:50-51), and RGBFilm::AddSample touches only its own pixel (film.h:251-257), so
disjoint row stripes rendered on different GPUs and summed equal the single-GPU film
exactly (non-owned pixels are exact zeros; x + 0 == x).  Rows are dealt in blocks of
``block`` round-robin so that every rank gets a similar mix of cheap (sky) and expensive
rows; the only collective is one sum-reduce of the film buffer at the end."""
from __future__ import annotations

import numpy as np


def rows_for_rank(py0: int, py1: int, rank: int, world: int, block: int = 16) -> np.ndarray:
    rows = np.arange(py0, py1, dtype=np.int32)
    if world <= 1:
        return rows
    blk = (rows - py0) // block
    return rows[(blk % world) == rank]


def job_spp(spp_per_gpu: int, world: int, scaling: str = "weak") -> int:
    """Samples per pixel of the whole job.  Strong scaling (bench.py's default for N > 1): the
    same W x H x spp image split N ways.  Weak scaling: every GPU keeps the single-GPU workload
    (W x H x spp samples), so the job is one W x H image at spp x N samples per pixel whose row
    stripes are dealt over the N GPUs (each renders 1/N of the rows at all spp x N samples)."""
    if scaling not in ("weak", "strong"):
        raise ValueError(f"scaling must be 'weak' or 'strong', not {scaling!r}")
    return spp_per_gpu * world if scaling == "weak" else spp_per_gpu


def reduce_film(film_tensor, dst: int = 0, group=None):
    """Sum-reduce the RGBFilm buffer ([4][yres*xres] float64: rgbSum[3], weightSum) onto
    rank ``dst`` with torch.distributed (RCCL over xGMI for device tensors, gloo on CPU)."""
    import torch.distributed as dist
    dist.reduce(film_tensor, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return film_tensor


def film_tensor_from_device_ptr(ptr: int, n_doubles: int, device: int):
    """Wrap the context's device film buffer as a torch tensor without copying."""
    import torch

    class _CAI:
        def __init__(self, p, n):
            self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (p, False), "version": 3}

    return torch.as_tensor(_CAI(ptr, n_doubles), device=f"cuda:{device}")
