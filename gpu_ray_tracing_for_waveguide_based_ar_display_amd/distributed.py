"""Multi-GPU sharding of the bounce kernel: one process per GPU, FoV x wavelength blocks.

Rays are independent and every ray's random stream is keyed by its GLOBAL index
(RNG seed ``0x9E3779B9 * (gid + 1)``, MAIN:158; zero-state fix-up, GRTF:28-29), so a
contiguous, R-aligned range of global ray ids -- a set of whole FoV x wavelength
blocks (layout ``gid = ((ii * NY + jj) * L + l) * R + r``, MAIN:82-115) -- can be traced
on any GPU with ``gid_offset`` and gives bit-identical results.  Each shard writes only
the eyebox slabs ``EB[l, n, m]`` of its own blocks, and eyebox values are integer
counts, so one sum-reduce of ``matrix_EB`` to rank 0 (RCCL over xGMI on MI355X, gloo in
the CPU tests) reproduces the single-GPU grid exactly.  That reduce is the only
collective on the path.

The tracer is pluggable (``trace_fn``) so the same sharding / reduction code runs with
the HIP kernel in production and with the CPU oracle in the multi-process CPU tests.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def block_range(n_blocks: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block range of ``rank`` (sizes differ by at most one block)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return rank * n_blocks // world, (rank + 1) * n_blocks // world


@dataclass
class Shard:
    rank: int
    world: int
    block_lo: int
    block_hi: int
    rays_per_block: int

    @property
    def gid_offset(self) -> int:
        return self.block_lo * self.rays_per_block

    @property
    def n_rays(self) -> int:
        return (self.block_hi - self.block_lo) * self.rays_per_block


def make_shard(num_fov_x: int, num_fov_y: int, n_lambda: int, rays_per_fov: int, world: int,
               rank: int) -> Shard:
    lo, hi = block_range(num_fov_x * num_fov_y * n_lambda, world, rank)
    return Shard(rank, world, lo, hi, rays_per_fov)


def reduce_eyebox(eb, group=None, dst: int = 0):
    """Sum-reduce the eyebox grid to ``dst`` (exact: integer counts in float32 < 2**24)."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.reduce(eb, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return eb


def trace_job(shard: Shard, build_rays_fn, trace_fn, new_eb, num_iter: int = 4, group=None):
    """Run the reference's job (``num_iter`` chained launches, MAIN:169-177) on this rank's
    shard and reduce the eyebox grid to rank 0.

    build_rays_fn(block_lo, block_hi) -> (rays, rng) for the shard (rng seeded with the
    global ids); trace_fn(rays, rng, eb, gid_offset) performs one launch in place;
    new_eb() -> zeroed eyebox grid (numpy array or torch tensor).
    Returns (eb, rng): eb holds the full-job grid on rank 0 (this rank's partial elsewhere).
    """
    rays, rng = build_rays_fn(shard.block_lo, shard.block_hi)
    eb = new_eb()
    for _ in range(num_iter):
        if shard.n_rays:
            trace_fn(rays, rng, eb, shard.gid_offset)
    return reduce_eyebox(eb, group), rng


def hip_tracer(scene, variant: int = 0):
    """trace_fn for ``trace_job`` using the HIP kernel (torch device tensors)."""
    from .engine import trace_fullcolor

    def fn(rays, rng, eb, gid_offset):
        trace_fullcolor(scene, rays, rng, eb, gid_offset=gid_offset, variant=variant)
    return fn


def shard_rays_host(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, block_lo, block_hi):
    """Host SoA columns + seeds of one shard (rays.build_rays restricted to the blocks)."""
    from .rays import build_rays, rng_seeds
    rays = build_rays(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, blocks=(block_lo, block_hi))
    return rays, rng_seeds(rays["x"].shape[0], block_lo * rays_per_fov)


__all__ = ["block_range", "Shard", "make_shard", "reduce_eyebox", "trace_job", "hip_tracer",
           "shard_rays_host"]
