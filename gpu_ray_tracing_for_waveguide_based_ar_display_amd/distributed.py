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

The tracer is pluggable (``trace_fn(rays, rng, eb, gid_offset, num_iter)``) so the same
sharding / stepping / reduction code runs with the HIP kernel in production (``bench.py``,
the reference-flow driver) and with the CPU oracle in the multi-process CPU tests.
"""
from __future__ import annotations

from dataclasses import dataclass

MAX_TRACES_PER_CALL = 255   # wgrt_launch_opts.num_iter


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


def split_calls(steps: int, per_call: int = 1) -> list[int]:
    """``steps`` chained traces as calls of at most ``per_call`` traces each (0: as few calls as
    possible), each call at most ``MAX_TRACES_PER_CALL``."""
    if steps < 0:
        raise ValueError("steps must be >= 0")
    f = min(MAX_TRACES_PER_CALL, steps if per_call <= 0 else per_call) or 1
    out = []
    while steps > 0:
        out.append(min(f, steps))
        steps -= out[-1]
    return out


def run_steps(trace_fn, rays, rng, eb, gid_offset: int, steps: int, per_call: int = 1, hook=None) -> list[int]:
    """The reference's loop of chained launches (MAIN:169-177) over one shard: ``steps`` traces
    of every ray, each starting from the RNG states the previous one left, issued as calls of
    at most ``per_call`` traces (``trace_fn(..., num_iter=k)``; a fused call gives the results
    of k separate ones).  ``hook(j, "start" | "end")`` brackets call j (HIP events in bench.py).
    Returns the traces per call."""
    calls = split_calls(steps, per_call)
    for j, k in enumerate(calls):
        if hook is not None:
            hook(j, "start")
        trace_fn(rays, rng, eb, gid_offset, k)
        if hook is not None:
            hook(j, "end")
    return calls


def reduce_eyebox(eb, group=None, dst: int = 0):
    """Sum-reduce the eyebox grid to ``dst`` (exact: integer counts in float32 < 2**24)."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        if getattr(eb, "is_cuda", False) and dist.get_backend(group) == "gloo":
            # gloo reduces device tensors only as an all-reduce (the bench's one-GPU rehearsal)
            dist.all_reduce(eb, op=dist.ReduceOp.SUM, group=group)
        else:
            dist.reduce(eb, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return eb


def trace_job(shard: Shard, build_rays_fn, trace_fn, new_eb, num_iter: int = 4, per_call: int = 1, group=None):
    """Run the reference's job (``num_iter`` chained launches, MAIN:169-177) on this rank's
    shard and reduce the eyebox grid to rank 0.

    build_rays_fn(block_lo, block_hi) -> (rays, rng) for the shard (rng seeded with the
    global ids); trace_fn(rays, rng, eb, gid_offset, num_iter) performs num_iter chained
    traces in place; new_eb() -> zeroed eyebox grid (numpy array or torch tensor).
    Returns (eb, rng): eb holds the full-job grid on rank 0 (this rank's partial elsewhere).
    """
    rays, rng = build_rays_fn(shard.block_lo, shard.block_hi)
    eb = new_eb()
    if shard.n_rays:
        run_steps(trace_fn, rays, rng, eb, shard.gid_offset, num_iter, per_call)
    return reduce_eyebox(eb, group), rng


def timed_run(trace_fn, rays, rng, eb, gid_offset: int, steps: int, per_call: int, stats, sync=None, hook=None,
              group=None):
    """bench.py's timed region on one rank: barrier + ``sync()``, ``steps`` chained traces of the
    shard (``run_steps``), the eyebox reduce to rank 0, ``sync()`` + barrier.  ``stats[0]`` (the
    device bounce counter, zeroed here) is what the tracer adds to.  Returns ``(elapsed, bounces,
    bounces_local)``: the wall time MAX over ranks, the bounce total SUM over ranks, this rank's
    own bounces.  The two small all-reduces run on ``stats``'s device (RCCL on the GPU box, gloo
    in the CPU tests)."""
    import time

    import torch
    import torch.distributed as dist
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    sync = sync or (lambda: None)
    stats.zero_()
    if multi:
        dist.barrier(group)
    sync()
    t0 = time.perf_counter()
    if steps and (rng.numel() if hasattr(rng, "numel") else len(rng)):
        run_steps(trace_fn, rays, rng, eb, gid_offset, steps, per_call, hook)
    reduce_eyebox(eb, group)
    sync()
    if multi:
        dist.barrier(group)
    elapsed = time.perf_counter() - t0
    local = int(stats[0].item())
    t = torch.tensor([elapsed], dtype=torch.float64, device=stats.device)
    b = torch.tensor([local], dtype=torch.int64, device=stats.device)
    if multi:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(b, op=dist.ReduceOp.SUM, group=group)
    return float(t.item()), int(b.item()), local


def hip_tracer(scene, variant: int = 0, stats=None):
    """trace_fn for ``run_steps`` / ``trace_job`` using the HIP kernel (torch device tensors);
    ``stats`` (int64[4] device tensor) is added to by every call."""
    from .engine import trace_fullcolor

    def fn(rays, rng, eb, gid_offset, num_iter=1):
        trace_fullcolor(scene, rays, rng, eb, gid_offset=gid_offset, stats=stats, variant=variant,
                        num_iter=num_iter)
    return fn


def hip_shard_builder(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, device):
    """build_rays_fn for ``trace_job`` that lays the shard out on the device (``wgrt_rays_init``,
    MAIN:59-158 without host arrays): only the eight columns the kernel reads."""
    from .engine import init_rays

    def build(block_lo, block_hi):
        return init_rays(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, blocks=(block_lo, block_hi),
                         device=device, all_columns=False)
    return build


def shard_rays_host(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, block_lo, block_hi):
    """Host SoA columns + seeds of one shard (rays.build_rays restricted to the blocks)."""
    from .rays import build_rays, rng_seeds
    rays = build_rays(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, blocks=(block_lo, block_hi))
    return rays, rng_seeds(rays["x"].shape[0], block_lo * rays_per_fov)


__all__ = ["block_range", "Shard", "make_shard", "split_calls", "run_steps", "reduce_eyebox", "trace_job", "timed_run",
           "hip_tracer", "hip_shard_builder", "shard_rays_host", "MAX_TRACES_PER_CALL"]
