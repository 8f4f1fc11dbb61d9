"""Multi-GPU sharding of the bounce kernel: one process per GPU, FoV x wavelength blocks.

Rays are independent and every ray's random stream is keyed by its GLOBAL index
(RNG seed ``0x9E3779B9 * (gid + 1)``, MAIN:158; zero-state fix-up, GRTF:28-29), so any set
of whole FoV x wavelength blocks (layout ``gid = ((ii * NY + jj) * L + l) * R + r``,
MAIN:82-115) can be traced on any GPU and gives bit-identical results, provided each local
ray knows its global id (``GidMap``).

Assignment.  Ray lifetimes differ by FoV and wavelength, so contiguous block ranges load the
ranks unevenly (the same effect measured across the dies of one GPU).  The
default assignment is therefore *interleaved*: block ``b = fov * L + k`` goes to rank
``(fov + k) mod N`` (``rank_blocks``) -- every N-th FoV, with the wavelength rotating, so each rank
gets a representative mix of FoVs and wavelengths whatever N and L are; ``contiguous`` remains
available.

Replicas (weak scaling).  ``replica_shard`` gives rank r the WHOLE batch again as replica r: the
same FoV x wavelength blocks and ray columns, with global ids ``r * N + i`` (N rays per replica),
so its random streams are its own.  N ranks then trace the reference's kernel over the batch's
columns tiled N times (RNG seeded by global index, MAIN:158) -- per-GPU work fixed as N grows, the
shape bench.py measures at N > 1 -- and every rank writes every slab, so the collective is the
sum-reduce of the grid (the north star's single RCCL reduce of the eyebox over xGMI).

Collective.  Each rank writes only the eyebox slabs ``EB[l, n, m]`` of its own blocks, plus --
through the compiled-numba flat-offset aliasing of an out-coupling exactly on the eyebox edge
(GRTF:154-165) -- the first ``SPILL`` floats of the slab after one of its own.
``collect_eyebox`` gathers exactly those bytes to rank 0 (``gather``: each rank sends
``nb x (9600 + SPILL)`` floats, 1/N of the grid, over its own xGMI link) and rank 0 assembles the
grid; ``reduce`` is the plain sum-reduce of the whole grid (50.8 MB at 21x21).  Eyebox values are
integer counts, so both reproduce the single-GPU grid exactly.  That is the only collective on
the path.

The tracer is pluggable (``trace_fn(rays, rng, eb, gid, num_iter)``, ``gid`` a ``GidMap``) so the
same sharding / stepping / collection code runs with the HIP kernel in production (``bench.py``,
the reference-flow driver) and with the CPU oracle in the multi-process CPU tests.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

MAX_TRACES_PER_CALL = 255   # wgrt_launch_opts.num_iter
EB_SLAB = 80 * 120          # one (wavelength, FoV) slab of matrix_EB (MAIN:37)
SPILL = 121                 # floats of the next slab an edge out-coupling can alias into (ix <= 120 at iy 80)


def block_range(n_blocks: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block range of ``rank`` (sizes differ by at most one block)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return rank * n_blocks // world, (rank + 1) * n_blocks // world


def rank_blocks(n_blocks: int, world: int, rank: int, assign: str = "interleaved", n_lambda: int = 1) -> np.ndarray:
    """Global block ids of ``rank`` (ascending): ``interleaved`` -- block ``fov * n_lambda + k`` to
    rank ``(fov + k) % world`` -- or ``contiguous`` (block_range)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    if assign == "interleaved":
        b = np.arange(n_blocks, dtype=np.int64)
        return b[(b // n_lambda + b % n_lambda) % world == rank]
    if assign == "contiguous":
        lo, hi = block_range(n_blocks, world, rank)
        return np.arange(lo, hi, dtype=np.int64)
    raise ValueError(f"unknown assignment {assign!r}")


@dataclass
class GidMap:
    """Global id of local ray i: ``block_gid[i // rays_per_block] + i % rays_per_block``."""
    block_gid: np.ndarray
    rays_per_block: int

    @property
    def offset(self) -> int | None:
        """The single ``gid_offset`` when the blocks are consecutive, else None."""
        b, R = self.block_gid, self.rays_per_block
        if len(b) == 0:
            return 0
        return int(b[0]) if np.array_equal(b, b[0] + R * np.arange(len(b))) else None

    def device_blocks(self, device):
        """``block_gid`` as an int64 tensor on ``device`` (wgrt_launch_opts.gid_blocks), uploaded on first
        use and cached on this map."""
        import torch
        cache = self.__dict__.setdefault("_dev", {})
        key = str(device)
        if key not in cache:
            cache[key] = torch.as_tensor(self.block_gid, dtype=torch.int64, device=device)
        return cache[key]

    def runs(self):
        """Consecutive stretches: ``(local_ray_lo, local_ray_hi, global_gid_lo)``."""
        b, R = self.block_gid, self.rays_per_block
        i = 0
        while i < len(b):
            j = i + 1
            while j < len(b) and b[j] == b[j - 1] + R:
                j += 1
            yield i * R, j * R, int(b[i])
            i = j


@dataclass
class Shard:
    rank: int
    world: int
    blocks: np.ndarray            # global block ids, ascending
    rays_per_block: int
    assign: str = "interleaved"
    gid_base: int = 0             # global id of the first ray of block 0 (replica r: r * rays of the batch)
    _gid: GidMap | None = field(default=None, repr=False)

    @property
    def n_rays(self) -> int:
        return len(self.blocks) * self.rays_per_block

    @property
    def gid(self) -> GidMap:
        if self._gid is None:
            self._gid = GidMap(self.gid_base + self.blocks * self.rays_per_block, self.rays_per_block)
        return self._gid

    @property
    def gid_offset(self) -> int | None:
        return self.gid.offset


def make_shard(num_fov_x: int, num_fov_y: int, n_lambda: int, rays_per_fov: int, world: int,
               rank: int, assign: str = "interleaved") -> Shard:
    return Shard(rank, world, rank_blocks(num_fov_x * num_fov_y * n_lambda, world, rank, assign, n_lambda),
                 rays_per_fov, assign)


def replica_shard(num_fov_x: int, num_fov_y: int, n_lambda: int, rays_per_fov: int, world: int,
                  rank: int) -> Shard:
    """Replica ``rank`` of the whole batch (weak scaling): every block, global ids offset by
    ``rank`` times the batch's ray count."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    nb = num_fov_x * num_fov_y * n_lambda
    return Shard(rank, world, np.arange(nb, dtype=np.int64), rays_per_fov, "replica",
                 gid_base=rank * nb * rays_per_fov)


def seeds_like(rng, gid: "GidMap"):
    """RNG seeds ``0x9E3779B9 * (gid + 1)`` (MAIN:158) of a shard's rays, written into ``rng``
    (a torch int32 view of the uint32 states, or a numpy uint32 array)."""
    R = gid.rays_per_block
    if hasattr(rng, "is_cuda"):
        import torch
        b = torch.as_tensor(gid.block_gid, dtype=torch.int64, device=rng.device)
        g = (b[:, None] + torch.arange(R, dtype=torch.int64, device=rng.device)[None, :]).reshape(-1)
        v = ((g + 1) * 0x9E3779B9) & 0xFFFFFFFF
        rng.copy_(torch.where(v >= 2 ** 31, v - 2 ** 32, v).to(torch.int32))
        return rng
    g = (np.asarray(gid.block_gid, dtype=np.uint64)[:, None] + np.arange(R, dtype=np.uint64)[None, :]).reshape(-1)
    rng[:] = ((g + np.uint64(1)) * np.uint64(0x9E3779B9) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    return rng


def slab_ids(blocks, num_fov_x: int, num_fov_y: int, lambdas) -> np.ndarray:
    """Flat slab index ``(lambda * NY + n) * NX + m`` of matrix_EB for each global block
    ``((m * NY + n) * L + k) * R`` (MAIN:82-115; lambda = lambdas[k])."""
    b = np.asarray(blocks, dtype=np.int64)
    L = len(lambdas)
    fov, k = np.divmod(b, L)
    m, n = np.divmod(fov, num_fov_y)
    lam = np.asarray(lambdas, dtype=np.int64)[k]
    return (lam * num_fov_y + n) * num_fov_x + m


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


def run_steps(trace_fn, rays, rng, eb, gid: GidMap, steps: int, per_call: int = 1, hook=None) -> list[int]:
    """The reference's loop of chained launches (MAIN:169-177) over one shard: ``steps`` traces
    of every ray, each starting from the RNG states the previous one left, issued as calls of
    at most ``per_call`` traces (``trace_fn(..., num_iter=k)``; a fused call gives the results
    of k separate ones).  ``hook(j, "start" | "end")`` brackets call j (HIP events in bench.py).
    Returns the traces per call."""
    calls = split_calls(steps, per_call)
    for j, k in enumerate(calls):
        if hook is not None:
            hook(j, "start")
        trace_fn(rays, rng, eb, gid, k)
        if hook is not None:
            hook(j, "end")
    return calls


def _world(group):
    import torch.distributed as dist
    return dist.get_world_size(group) if dist.is_initialized() else 1


def reduce_eyebox(eb, group=None, dst: int = 0):
    """Sum-reduce the eyebox grid to ``dst`` (exact: integer counts in float32 < 2**24)."""
    import torch.distributed as dist
    if _world(group) > 1:
        if getattr(eb, "is_cuda", False) and dist.get_backend(group) == "gloo":
            # gloo reduces device tensors only as an all-reduce (the bench's one-GPU rehearsal)
            dist.all_reduce(eb, op=dist.ReduceOp.SUM, group=group)
        else:
            dist.reduce(eb, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return eb


class EyeboxGather:
    """Gather of each rank's own eyebox slabs (+ their spill) to rank 0, and the assembly there.

    ``all_blocks[r]``: global block ids of rank r (every rank knows the whole assignment, so
    the message sizes and placements need no exchange).  A rank's payload is one flat buffer,
    ``[nb x 9600 slab floats | nb x SPILL spill floats, padded to 4]`` (include/wgrt.h
    wgrt_eyebox_*), padded to the largest shard (the collective needs equal sizes).  The send buffer
    and rank 0's receive buffer are allocated once (first call per device and dtype) and reused;
    every index is precomputed on the host here, so a call makes no host round trip before the
    collective.  On a HIP device the pack and the assembly are the library's row-copy kernels
    (``wgrt_eyebox_pack`` / ``wgrt_eyebox_assemble``: one launch each, 16-B loads and stores, each
    owned slab written once from the rank that traced it); host tensors (the gloo CPU tests) take the
    same steps as torch gathers and scatters.  Slabs no rank owns are zeroed, spills added last."""

    def __init__(self, all_blocks, num_fov_x: int, num_fov_y: int, lambdas, n_lambda_scene: int, device=None):
        import torch
        self.n_slabs = n_lambda_scene * num_fov_y * num_fov_x
        self.world = len(all_blocks)
        self.nb = max(len(b) for b in all_blocks)
        self.spill_len = (self.nb * SPILL + 3) // 4 * 4
        self.payload_len = self.nb * EB_SLAB + self.spill_len
        self.device = device
        t = lambda a, dt=torch.int64: torch.as_tensor(np.asarray(a), dtype=dt, device=device)
        self.slabs, self.nxt, self.spill_mask, self.spill_rows, self.spill_dst = [], [], [], [], []
        self.has_spill, self.counts = [], []
        owned = np.zeros(self.n_slabs, dtype=bool)
        for b in all_blocks:
            s = slab_ids(b, num_fov_x, num_fov_y, lambdas)
            own = set(s.tolist())
            owned[s] = True
            # the spill of slab s lands in s + 1; it must travel unless s + 1 is this rank's own
            # slab (then it is already in that slab's copy) or past the grid (dropped, as the
            # kernel's guard drops it)
            sp = np.array([(v + 1) not in own and v + 1 < self.n_slabs for v in s.tolist()], dtype=bool)
            self.counts.append(len(s))
            self.slabs.append(t(s))
            self.nxt.append(t(np.minimum(s + 1, self.n_slabs - 1)))
            self.spill_mask.append(t(sp, torch.float32))
            self.spill_rows.append(t(np.nonzero(sp)[0]))
            self.spill_dst.append(t(s[sp] + 1))
            self.has_spill.append(bool(sp.any()))
        self.unowned = t(np.nonzero(~owned)[0])
        self.any_unowned = bool((~owned).any())
        # the assembly's row maps (wgrt_eyebox_assemble): payload row j of rank r -> its slab and the slab
        # its spill row adds to, -1 for padding rows and rows without a spill to move
        dst = np.full((self.world, self.nb), -1, dtype=np.int64)
        sdst = np.full((self.world, self.nb), -1, dtype=np.int64)
        for r, b in enumerate(all_blocks):
            sl = slab_ids(b, num_fov_x, num_fov_y, lambdas)
            dst[r, :len(sl)] = sl
            sp = self.spill_mask[r].cpu().numpy() > 0
            sdst[r, :len(sl)][sp] = sl[sp] + 1
        self.dst_rows, self.spill_dst_rows = t(dst.reshape(-1)), t(sdst.reshape(-1))
        self._bufs = {}
        self._dev_idx = {}

    def _idx(self, device):
        """The index tensors on ``device`` (moved once per device and cached): the HIP kernels take their
        raw pointers, so they must live on the grid's own device whatever ``device=`` the gather was
        built with."""
        key = str(device)
        if key not in self._dev_idx:
            mv = lambda v: v.to(device)
            self._dev_idx[key] = dict(slabs=[mv(v) for v in self.slabs], nxt=[mv(v) for v in self.nxt],
                                      spill_mask=[mv(v) for v in self.spill_mask], dst_rows=mv(self.dst_rows),
                                      spill_dst_rows=mv(self.spill_dst_rows), unowned=mv(self.unowned))
        return self._dev_idx[key]

    def buffers(self, device, dtype, dst: bool):
        """(send, recv): the payload buffer and, on the gathering rank, the [world, payload] receive
        buffer (None elsewhere); allocated on first use, zeroed once (padding rows stay zero)."""
        import torch
        key = (str(device), dtype, dst)
        if key not in self._bufs:
            send = torch.zeros(self.payload_len, dtype=dtype, device=device)
            recv = torch.zeros((self.world, self.payload_len), dtype=dtype, device=device) if dst else None
            self._bufs[key] = (send, recv)
        return self._bufs[key]

    def _views(self, buf):
        nb = self.nb
        return buf[:nb * EB_SLAB].view(nb, EB_SLAB), buf[nb * EB_SLAB:nb * EB_SLAB + nb * SPILL].view(nb, SPILL)

    @staticmethod
    def _hip(t) -> bool:
        return getattr(t, "is_cuda", False) and t.dtype.is_floating_point and t.element_size() == 4

    def pack(self, eb, rank: int, out=None):
        """Rank ``rank``'s payload, into ``out`` (the collective passes its reused send buffer) or a new
        zeroed buffer."""
        import torch
        flat = eb.reshape(self.n_slabs, EB_SLAB)
        buf = out if out is not None else torch.zeros(self.payload_len, dtype=eb.dtype, device=eb.device)
        n = self.counts[rank]
        if self._hip(eb) and eb.is_contiguous():
            from ._lib import check, load
            from .engine import _stream_handle
            if buf.device != eb.device or not buf.is_contiguous() or buf.numel() < self.payload_len:
                raise ValueError("EyeboxGather.pack: out must be a contiguous payload buffer on the grid's device")
            ix = self._idx(eb.device)
            check(load().wgrt_eyebox_pack(eb.data_ptr(), self.n_slabs, ix["slabs"][rank].data_ptr(),
                                          ix["nxt"][rank].data_ptr(), ix["spill_mask"][rank].data_ptr(), n, self.nb,
                                          buf.data_ptr(), _stream_handle(eb.device)), "wgrt_eyebox_pack")
            return buf
        main, spill = self._views(buf)
        torch.index_select(flat, 0, self.slabs[rank], out=main[:n])
        if self.has_spill[rank]:
            torch.index_select(flat[:, :SPILL], 0, self.nxt[rank], out=spill[:n])
            spill[:n].mul_(self.spill_mask[rank].to(eb.dtype)[:, None])
        return buf

    def assemble(self, eb, parts) -> None:
        """Rank 0: rebuild the whole grid in ``eb`` from every rank's payload (``parts[r]``: rank r's
        flat payload; on a HIP device ``parts`` may be the [world, payload] receive buffer itself)."""
        flat = eb.reshape(self.n_slabs, EB_SLAB)
        ix = self._idx(eb.device)
        if self.any_unowned:
            flat.index_fill_(0, ix["unowned"], 0)
        recv = parts if hasattr(parts, "shape") else None
        if self._hip(eb) and eb.is_contiguous():
            import torch
            if recv is None or not recv.is_contiguous():
                recv = torch.stack(list(parts)) if not hasattr(parts, "shape") else parts.contiguous()
            if recv.device != eb.device:
                recv = recv.to(eb.device)
            from ._lib import check, load
            from .engine import _stream_handle
            check(load().wgrt_eyebox_assemble(eb.data_ptr(), self.n_slabs, recv.data_ptr(), self.world, self.nb,
                                              ix["dst_rows"].data_ptr(), ix["spill_dst_rows"].data_ptr(),
                                              _stream_handle(eb.device)), "wgrt_eyebox_assemble")
            return
        parts = [recv[r] for r in range(self.world)] if recv is not None else parts
        for r, p in enumerate(parts):
            n = self.counts[r]
            if n:
                flat.index_copy_(0, self.slabs[r], self._views(p)[0][:n])
        head = flat[:, :SPILL]
        for r, p in enumerate(parts):
            if self.has_spill[r]:
                head.index_add_(0, self.spill_dst[r], self._views(p)[1].index_select(0, self.spill_rows[r]))

    def __call__(self, eb, group=None, dst: int = 0):
        import torch.distributed as dist
        if _world(group) <= 1:
            return eb
        rank = dist.get_rank(group)
        on_gloo_dev = getattr(eb, "is_cuda", False) and dist.get_backend(group) == "gloo"
        send, recv = self.buffers(eb.device, eb.dtype, rank == dst)
        payload = self.pack(eb, rank, out=send)
        if on_gloo_dev:
            # gloo gathers host tensors (the bench's one-GPU rehearsal)
            payload = payload.cpu()
            parts = [recv[r].cpu() for r in range(self.world)] if rank == dst else None
        else:
            parts = [recv[r] for r in range(self.world)] if rank == dst else None
        dist.gather(payload, gather_list=parts, dst=dst, group=group)
        if rank == dst:
            if on_gloo_dev:
                for r in range(self.world):
                    recv[r].copy_(parts[r])
            self.assemble(eb, recv)
        return eb


def trace_job(shard: Shard, build_rays_fn, trace_fn, new_eb, num_iter: int = 4, per_call: int = 1, group=None,
              collect=None):
    """Run the reference's job (``num_iter`` chained launches, MAIN:169-177) on this rank's
    shard and collect the eyebox grid on rank 0.

    build_rays_fn(shard) -> (rays, rng) for the shard (rng seeded with the global ids);
    trace_fn(rays, rng, eb, gid, num_iter) performs num_iter chained traces in place;
    new_eb() -> zeroed eyebox grid (numpy array or torch tensor); collect(eb, group) ->
    the collective (default ``reduce_eyebox``; an ``EyeboxGather`` moves 1/N of the bytes).
    Returns (eb, rng): eb holds the full-job grid on rank 0 (this rank's partial elsewhere).
    """
    rays, rng = build_rays_fn(shard)
    eb = new_eb()
    if shard.n_rays:
        run_steps(trace_fn, rays, rng, eb, shard.gid, num_iter, per_call)
    return (collect or reduce_eyebox)(eb, group), rng


def timed_run(trace_fn, rays, rng, eb, gid: GidMap, steps: int, per_call: int, stats, sync=None, hook=None,
              group=None, collect=None):
    """bench.py's timed region on one rank: barrier + ``sync()``, ``steps`` chained traces of the
    shard (``run_steps``), the eyebox collective to rank 0 (``collect``, default the reduce),
    ``sync()`` + barrier.  ``stats[0]`` (the device bounce counter, zeroed here) is what the
    tracer adds to.  Returns ``(elapsed, bounces, bounces_local)``: the wall time MAX over ranks,
    the bounce total SUM over ranks, this rank's own bounces.  The two small all-reduces run on
    ``stats``'s device (RCCL on the GPU box, gloo in the CPU tests)."""
    import time

    import torch
    import torch.distributed as dist
    multi = _world(group) > 1
    sync = sync or (lambda: None)
    stats.zero_()
    if multi:
        dist.barrier(group)
    sync()
    t0 = time.perf_counter()
    if steps and (rng.numel() if hasattr(rng, "numel") else len(rng)):
        run_steps(trace_fn, rays, rng, eb, gid, steps, per_call, hook)
    (collect or reduce_eyebox)(eb, group)
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
    ``stats`` (int64[STATS_LEN] device tensor) is added to by every call.  A shard of several
    block ranges passes its global ids as ``gid_blocks``, uploaded once per map and device and kept
    on the GidMap itself (``GidMap.device_blocks``: released with the map, no tracer-side cache)."""
    from .engine import trace_fullcolor

    def fn(rays, rng, eb, gid: GidMap, num_iter=1):
        off = gid.offset
        if off is not None:
            trace_fullcolor(scene, rays, rng, eb, gid_offset=off, stats=stats, variant=variant, num_iter=num_iter)
            return
        trace_fullcolor(scene, rays, rng, eb, stats=stats, variant=variant, num_iter=num_iter,
                        gid_blocks=gid.device_blocks(rng.device), gid_block_rays=gid.rays_per_block)
    return fn


def hip_shard_builder(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, device):
    """build_rays_fn for ``trace_job`` that lays the shard out on the device (``wgrt_rays_init``,
    MAIN:59-158 without host arrays): only the eight columns the kernel reads."""
    from .engine import init_rays

    def build(shard: Shard):
        rays, rng = init_rays(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, block_list=shard.blocks,
                              device=device, all_columns=False)
        if shard.gid_base:   # a replica: the same columns, its own global ids
            seeds_like(rng, shard.gid)
        return rays, rng
    return build


def shard_rays_host(points, num_fov_x, num_fov_y, lambdas, rays_per_fov, blocks, gid_base: int = 0):
    """Host SoA columns + seeds of the global blocks ``blocks`` laid back to back (rays.build_rays
    restricted to each run of consecutive blocks); ``gid_base`` offsets the global ids (a replica
    shard)."""
    from .rays import build_rays, rng_seeds
    parts, seeds = [], []
    R = rays_per_fov
    for lo_r, hi_r, g in GidMap(np.asarray(blocks, dtype=np.int64) * R, R).runs():
        b0 = g // R
        nb = (hi_r - lo_r) // R
        parts.append(build_rays(points, num_fov_x, num_fov_y, lambdas, R, blocks=(b0, b0 + nb)))
        seeds.append(rng_seeds(nb * R, g))
    if not parts:
        empty = build_rays(points, num_fov_x, num_fov_y, lambdas, R, blocks=(0, 0))
        return empty, rng_seeds(0, 0)
    rays = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    seeds = np.concatenate(seeds)
    if gid_base:
        seeds_like(seeds, GidMap(gid_base + np.asarray(blocks, dtype=np.int64) * R, R))
    return rays, seeds


__all__ = ["block_range", "rank_blocks", "GidMap", "Shard", "make_shard", "replica_shard", "seeds_like", "slab_ids", "split_calls", "run_steps",
           "reduce_eyebox", "EyeboxGather", "trace_job", "timed_run", "hip_tracer", "hip_shard_builder",
           "shard_rays_host", "MAX_TRACES_PER_CALL", "EB_SLAB", "SPILL"]
