"""Device-side entry points over torch ROCm tensors (PyTorch is the memory/stream plumbing).

``trace_fullcolor`` is one launch of the bounce kernel (the reference's
``process_rays_kernel_pro_fullColor[blocks, 256](...)``, GRTF:833-1246) through the
PyTorch-ROCm operator ``torch.ops.wgrt.trace`` (csrc/wgrt_torch.cpp), which forwards to the
C ABI ``wgrt_trace_opts``; it validates every buffer and raises on misuse instead of
corrupting memory.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import STATS_LEN, DebugOpts, Rays, Scene, TraceStats, WgrtError, check, load, ops

RAY_COLUMNS = ("x", "y", "gap_x", "gap_y", "pol", "azi", "m", "n", "lmd_num", "te", "tm", "delta_phase")
READ_COLUMNS = ("x", "y", "m", "n", "lmd_num", "te", "tm", "delta_phase")

VARIANT_AUTO, VARIANT_GRID, VARIANT_JONES32, VARIANT_JONES64 = 0, 1, 7, 9   # include/wgrt.h
CHUNK = 64   # rays per work-queue chunk of the persistent kernels (wgrt_launch_opts.chunk_order)


def _stream_handle(device: torch.device, stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


def _as_dev(t, dtype, name, device, n=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch tensor, got {type(t).__name__}")
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if n is not None and t.numel() != n:
        raise ValueError(f"{name} has {t.numel()} elements, expected {n}")
    return t


def rays_to_device(rays: dict, device="cuda") -> dict:
    """Copy the twelve float32 host columns (rays.build_rays) to device tensors."""
    return {k: torch.from_numpy(np.ascontiguousarray(rays[k], dtype=np.float32)).to(device)
            for k in RAY_COLUMNS if k in rays}


def trace_fullcolor(scene: Scene, rays: dict, rng_states: torch.Tensor, matrix_EB: torch.Tensor,
                    gid_offset: int = 0, n_rays: int | None = None, stats: torch.Tensor | None = None,
                    per_ray_bounces: torch.Tensor | None = None, stream=None, variant: int = VARIANT_AUTO,
                    workgroups: int = 0, chunk_order: torch.Tensor | None = None, num_iter: int = 1,
                    gid_blocks: torch.Tensor | None = None, gid_block_rays: int = 0, debug: dict | None = None,
                    grid_sqrt_k: float = 0.0) -> None:
    """Asynchronous launch on ``stream`` (default: torch's current stream).

    rays: dict of device float32 tensors keyed like the reference columns
    (``x, y, m, n, lmd_num, te, tm, delta_phase`` required; the four columns the
    kernel never reads may be absent).  rng_states uint32 -> torch.int32 view is
    accepted too.  stats: optional int64[STATS_LEN] device tensor that is added to
    (bounces, bad_rays, eyebox_hits, replayed, handoff_giveups, interactions, libm_rays; ``check_stats`` raises
    on a hand-off give-up).  chunk_order: optional int32 device permutation of the 64-ray chunks
    (``schedule_by_lifetime``); results do not depend on it.  num_iter: chained traces of every
    ray (the reference's ``num_iter`` loop of launches, MAIN:169-177) in one call -- results
    identical to ``num_iter`` calls; the Jones-vector variants run them in one persistent launch
    (``wgrt_launch_opts.num_iter``).  gid_blocks / gid_block_rays: global ray ids of a shard made of
    several block ranges (int64 device tensor, first global id of each local block of
    ``gid_block_rays`` rays; ``gid_offset`` must then be 0).  debug: ``wgrt_debug_opts`` fields
    (cert_tol, cert_tol32, chunk_rays, timeline (uint64 device tensor), fail_after_trace,
    handoff_wait_ticks) -- test / profiling hooks.  grid_sqrt_k: the single-trace grid rule
    (``wgrt_launch_opts.grid_sqrt_k``; 0 the default, < 0 the resident grid).
    """
    if scene.single_lambda:
        raise ValueError("trace_fullcolor needs a full-colour scene; use trace_single for a single-wavelength one")
    _trace(scene, rays, rng_states, matrix_EB, gid_offset, n_rays, stats, per_ray_bounces, stream, variant,
           workgroups, single=False, chunk_order=chunk_order, num_iter=num_iter, gid_blocks=gid_blocks,
           gid_block_rays=gid_block_rays, debug=debug, grid_sqrt_k=grid_sqrt_k)


def new_stats(device) -> torch.Tensor:
    """A zeroed int64 device tensor laid out as ``wgrt_trace_stats``."""
    return torch.zeros(STATS_LEN, dtype=torch.int64, device=device)


def check_stats(stats: torch.Tensor) -> None:
    """Raise if a fused launch gave up a hand-off (``wgrt_trace_stats.handoff_giveups``): the
    eyebox grid and RNG states of that call are then wrong.  Warn (``luts.EnerUnderflowWarning``, a
    ``LUTPrecisionWarning``) if traces were decided in the ener-underflow regime
    (``wgrt_trace_stats.libm_rays``, ABI 7): their paths depend on the libm's last bits, so they may
    differ from a CPU run of the reference.  Synchronises on ``stats``."""
    st = stats.cpu()
    g = int(st[4])
    if g:
        raise WgrtError(f"{g} fused-launch traces gave up waiting for their ray's previous trace "
                        "(hand-off failure; results of this call are invalid)")
    lm = int(st[6]) if st.numel() > 6 else 0
    if lm:
        import warnings
        from .luts import EnerUnderflowWarning
        warnings.warn(f"{lm} traces reached the ener-underflow regime (a guard product ener * e below 2^-1000, "
                      "GRTF:1020): their decisions hang on the last bits of cos / sin / atan2, so they may differ "
                      "from the reference run on another libm (wgrt_trace_stats.libm_rays)",
                      EnerUnderflowWarning, stacklevel=2)


def reserve(scene: Scene, n_rays: int, num_iter: int = 1, stream=None) -> None:
    """Pre-allocate the Jones-vector variants' launch scratch for up to ``n_rays`` rays x
    ``num_iter`` chained traces on ``stream`` (``wgrt_scene_reserve``): later launches within
    those sizes neither allocate nor synchronise."""
    device = torch.device("cuda", scene.device)
    check(load().wgrt_scene_reserve(scene.handle, int(n_rays), int(num_iter),
                                    ctypes.c_void_p(_stream_handle(device, stream))), "wgrt_scene_reserve")


def trace_single(scene: Scene, rays: dict, rng_states: torch.Tensor, matrix_EB: torch.Tensor,
                 gid_offset: int = 0, n_rays: int | None = None, stats: torch.Tensor | None = None,
                 per_ray_bounces: torch.Tensor | None = None, stream=None, variant: int = VARIANT_AUTO,
                 workgroups: int = 0, chunk_order: torch.Tensor | None = None, num_iter: int = 1,
                 gid_blocks: torch.Tensor | None = None, gid_block_rays: int = 0, debug: dict | None = None,
                 grid_sqrt_k: float = 0.0) -> None:
    """One launch of the single-wavelength kernel (``process_rays_kernel_pro``, GRTF:419-831)
    through ``wgrt_trace_single_ex``: no ``lmd_num`` column (ignored if present),
    matrix_EB [NY, NX, 80, 120], branch guard ener * efficiency > 1e-15.  The scene must be
    a single-wavelength one (``Scene.from_geometry(..., wavelength=l)`` or 3-D LUTs)."""
    if not scene.single_lambda:
        raise ValueError("trace_single needs a single-wavelength scene (Scene.from_geometry(..., wavelength=l))")
    _trace(scene, rays, rng_states, matrix_EB, gid_offset, n_rays, stats, per_ray_bounces, stream, variant,
           workgroups, single=True, chunk_order=chunk_order, num_iter=num_iter, gid_blocks=gid_blocks,
           gid_block_rays=gid_block_rays, debug=debug, grid_sqrt_k=grid_sqrt_k)


def _debug_opts(debug: dict | None):
    if not debug:
        return None
    unknown = set(debug) - {f for f, _ in DebugOpts._fields_} - {"timeline"}
    if unknown:
        raise ValueError(f"unknown debug options {sorted(unknown)}")
    d = DebugOpts()
    for k, v in debug.items():
        if k == "timeline":
            if v is not None:
                if v.dtype != torch.int64 or not v.is_contiguous() or v.numel() % 8:
                    raise ValueError("timeline must be a contiguous int64 tensor of 8 words per wave")
                d.timeline = ctypes.c_void_p(v.data_ptr())
                d.timeline_waves = v.numel() // 8
        elif k != "timeline_waves":
            setattr(d, k, v)
    return d


def _trace(scene, rays, rng_states, matrix_EB, gid_offset, n_rays, stats, per_ray_bounces, stream, variant,
           workgroups, single, chunk_order=None, num_iter=1, gid_blocks=None, gid_block_rays=0, debug=None,
           grid_sqrt_k=0.0):
    device = torch.device("cuda", scene.device)
    x = rays["x"]
    N = x.numel() if n_rays is None else int(n_rays)
    if N < 0 or N > x.numel():
        raise ValueError(f"n_rays={N} out of range for {x.numel()} rays")
    cols = {}
    for k in READ_COLUMNS:
        if single and k == "lmd_num":
            continue
        if k not in rays:
            raise ValueError(f"missing ray column {k!r}")
        cols[k] = _as_dev(rays[k], torch.float32, k, device, x.numel())
    if rng_states.dtype not in (torch.int32, torch.uint32):
        raise TypeError(f"rng_states must be uint32 (or an int32 view), got {rng_states.dtype}")
    _as_dev(rng_states, rng_states.dtype, "rng_states", device, x.numel())
    _as_dev(matrix_EB, torch.float32, "matrix_EB", device)
    if tuple(matrix_EB.shape) != scene.eb_shape():
        raise ValueError(f"matrix_EB shape {tuple(matrix_EB.shape)} != {scene.eb_shape()}")
    if stats is not None:
        _as_dev(stats, torch.int64, "stats", device, STATS_LEN)
    if per_ray_bounces is not None:
        if per_ray_bounces.dtype not in (torch.int32, torch.uint32):
            raise TypeError("per_ray_bounces must be uint32 / int32")
        _as_dev(per_ray_bounces, per_ray_bounces.dtype, "per_ray_bounces", device, x.numel())
    n_chunks = (N + CHUNK - 1) // CHUNK
    if chunk_order is not None:
        _as_dev(chunk_order, torch.int32, "chunk_order", device, n_chunks)
    if gid_blocks is not None:
        if gid_block_rays < 1:
            raise ValueError("gid_blocks needs gid_block_rays >= 1")
        _as_dev(gid_blocks, torch.int64, "gid_blocks", device, (N + gid_block_rays - 1) // gid_block_rays if N else None)
    dbg = _debug_opts(debug)
    # the launch: torch.ops.wgrt.trace (csrc/wgrt_torch.cpp) -> wgrt_trace_opts on the caller's stream
    status = ops().trace(scene.handle.value, cols["x"], cols["y"], cols["m"], cols["n"], cols.get("lmd_num"),
                         cols["te"], cols["tm"], cols["delta_phase"], rng_states, matrix_EB, stats, per_ray_bounces,
                         N, int(gid_offset), _stream_handle(device, stream), 1 if single else 0, int(variant),
                         int(workgroups), chunk_order, int(num_iter), gid_blocks,
                         int(gid_block_rays) if gid_blocks is not None else 0,
                         ctypes.addressof(dbg) if dbg is not None else 0, float(grid_sqrt_k))
    check(status, "wgrt_trace_single" if single else "wgrt_trace_fullcolor")


def timeline_summary(buf, percentiles: bool = True) -> dict:
    """Summary of one launch's wave timeline (``debug=dict(timeline=buf)``: 8 int64 words per wave --
    start, queue exhausted, end (s_memrealtime, 100 MHz), passes, lane-passes, XCD, passes and
    lane-passes up to the queue running dry): when the work queue ran dry, when the waves ended,
    and the pass durations and lane occupancy before (bulk) and after (drain) -- where a single
    launch's time goes."""
    t = buf.cpu().numpy().reshape(-1, 8)
    t = t[t[:, 0] > 0]
    start, exh, end, passes, lanes, xcc, p_exh, l_exh = (t[:, k].astype(np.float64) for k in range(8))
    t0 = start.min()
    us = lambda v: (v - t0) / 100.0   # 100 MHz ticks -> us
    drain_passes = passes - p_exh
    last = us(end) >= np.percentile(us(end), 99)
    pc = lambda v, qs: [round(float(np.percentile(v, q)), 3) for q in qs]
    return {"waves": int(len(t)),
            "exhausted_us": pc(us(exh), (0, 50, 100)),
            "end_us": pc(us(end), (0, 50, 99, 100)),
            "drain_frac": round(float((us(end).max() - np.median(us(exh))) / max(us(end).max(), 1e-9)), 4),
            "bulk_us_per_pass": round(float(np.median(us(exh) / np.maximum(p_exh, 1))), 3),
            "drain_us_per_pass": round(float(np.median((end - exh) / 100.0 / np.maximum(drain_passes, 1))), 3),
            "bulk_lanes_per_pass": round(float(l_exh.sum() / max(p_exh.sum(), 1)), 2),
            "drain_lanes_per_pass": round(float((lanes - l_exh).sum() / max(drain_passes.sum(), 1)), 2),
            "last1pct_drain_passes": round(float(np.median(drain_passes[last])), 1),
            "last1pct_drain_us_per_pass": round(float(np.median(((end - exh) / 100.0 /
                                                                   np.maximum(drain_passes, 1))[last])), 3)}


def schedule_by_lifetime(per_ray_bounces, tile_of_ray, n_tiles: int | None = None):
    """Issue order of the 64-ray chunks for ``chunk_order``: the chunks whose rays belong to the
    (wavelength, FoV) tiles with the longest mean lifetime in a previous launch go first, so the
    rays that outlive the work queue come from short-lived tiles.  The kernel's work queue hands
    out chunk positions in stripes of 16 (stripe s on head s % 8, each head's stripes in
    increasing order, wgrt_trace.hip), so a global longest-first order is also longest-first on
    every head.  ``per_ray_bounces`` from an earlier launch of the same batch
    (``trace_*(per_ray_bounces=...)``), ``tile_of_ray`` any integer tile key per ray (e.g.
    ``(lmd_num * NX + m) * NY + n``).  Device tensors in, int32 device permutation out (a few
    small torch ops, no host sync).  A pure scheduling hint: results are unchanged (DESIGN.md
    §5.4: it measured within noise on C3)."""
    b = per_ray_bounces.to(torch.float32)
    key = tile_of_ray.to(torch.int64)
    nt = int(n_tiles) if n_tiles is not None else int(key.max().item()) + 1
    tot = torch.zeros(nt, dtype=torch.float32, device=b.device).index_add_(0, key, b)
    cnt = torch.zeros(nt, dtype=torch.float32, device=b.device).index_add_(0, key, torch.ones_like(b))
    mean = tot / cnt.clamp_min(1.0)
    N = b.numel()
    first = torch.arange(0, N, CHUNK, device=b.device)
    chunk_key = mean[key[first]]
    return torch.argsort(-chunk_key.to(torch.float64), stable=True).to(torch.int32)


def block_runs(block_list) -> list[tuple[int, int, int]]:
    """Runs of consecutive global block ids: ``(local_block_lo, global_block_lo, count)``."""
    ids = [int(v) for v in block_list]
    runs, i = [], 0
    while i < len(ids):
        j = i + 1
        while j < len(ids) and ids[j] == ids[j - 1] + 1:
            j += 1
        runs.append((i, ids[i], j - i))
        i = j
    return runs


def init_rays(points, num_fov_x: int, num_fov_y: int, lambdas, rays_per_fov: int, blocks=None,
              device="cuda", all_columns: bool = True, stream=None, block_list=None):
    """Build a ray batch on the device (``wgrt_rays_init``; replaces MAIN:59-115 and the RNG
    seeding at MAIN:158, bit-identical to ``rays.build_rays`` + ``rays.rng_seeds``).

    ``points``: the R/2 origins (numpy or torch float64 [R/2, 2]); ``blocks=(lo, hi)``
    builds FoV x wavelength blocks [lo, hi) only (one rank's shard, global ids from lo * R);
    ``block_list`` (any sequence of global block ids) builds those blocks back to back (an
    interleaved shard: local block j is global block block_list[j], RNG seeded with its global
    ids).  ``all_columns=False`` allocates only the eight columns the kernel reads.
    Returns ``(rays, rng_states)``: a dict of float32 tensors and an int32 view of the
    uint32 RNG states."""
    device = torch.device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    R = int(rays_per_fov)
    lam = np.ascontiguousarray(list(lambdas), dtype=np.int32)
    nblk = num_fov_x * num_fov_y * len(lam)
    if block_list is not None:
        if blocks is not None:
            raise ValueError("give blocks or block_list, not both")
        ids = [int(v) for v in block_list]
        if any(not 0 <= v < nblk for v in ids):
            raise ValueError(f"block_list has ids outside [0, {nblk})")
        runs = block_runs(ids)
        nb = len(ids)
    else:
        lo, hi = (0, nblk) if blocks is None else (int(blocks[0]), int(blocks[1]))
        if not 0 <= lo <= hi <= nblk:
            raise ValueError(f"block range {blocks} outside [0, {nblk}]")
        runs, nb = [(0, lo, hi - lo)], hi - lo
    pts = points if isinstance(points, torch.Tensor) else torch.from_numpy(np.asarray(points, dtype=np.float64))
    pts = pts.to(device=device, dtype=torch.float64).contiguous()
    if tuple(pts.shape) != (R // 2, 2):
        raise ValueError(f"points must have shape ({R // 2}, 2), got {tuple(pts.shape)}")
    N = nb * R
    names = RAY_COLUMNS if all_columns else READ_COLUMNS
    rays = {k: torch.empty(N, dtype=torch.float32, device=device) for k in names}
    rng = torch.empty(N, dtype=torch.int32, device=device)
    for loc, glo, cnt in runs:
        off = loc * R * 4   # bytes into every 4-byte column
        cols = Rays(**{k: ctypes.c_void_p(v.data_ptr() + off) for k, v in rays.items()})
        check(load().wgrt_rays_init(ctypes.c_void_p(pts.data_ptr()), R, int(num_fov_x), int(num_fov_y),
                                    lam.ctypes.data_as(ctypes.c_void_p), len(lam), glo, glo + cnt,
                                    ctypes.byref(cols), ctypes.c_void_p(rng.data_ptr() + off),
                                    ctypes.c_void_p(_stream_handle(device, stream))),
              "wgrt_rays_init")
    return rays, rng


def classify_points(scene: Scene, xy: torch.Tensor, stream=None) -> torch.Tensor:
    """Per-point polygon membership bitmask through the scene's exact locator."""
    device = torch.device("cuda", scene.device)
    xy = _as_dev(xy, torch.float64, "xy", device)
    n = xy.shape[0]
    out = torch.empty(n, dtype=torch.int64, device=device)
    check(load().wgrt_scene_classify(scene.handle, ctypes.c_void_p(xy.data_ptr()), n,
                                     ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(_stream_handle(device, stream))), "wgrt_scene_classify")
    return out


SHADOW_DEPTHS = ("[1,10)", "[10,30)", "[30,100)", "[100,300)", "[300,1000)", "[1000,inf)")


def shadow(scene: Scene, rays: dict, rng_states: torch.Tensor, gid_offset: int = 0, n_rays: int | None = None,
           per_ray_bounces: torch.Tensor | None = None, stream=None) -> dict:
    """Certification shadow of the Jones-vector lane (``wgrt_debug_shadow``): traces the rays with
    the reference's own arithmetic and measures, at every Monte-Carlo decision, how far the
    product lane's thresholds stray from the reference's relative to its certification bound.
    ``rng_states`` / ``per_ray_bounces`` are updated as one exact launch would.  Synchronous;
    returns the statistics as a dict (``max_ratio``, ``silent_flips``, ``uncertain``, ...)."""
    device = torch.device("cuda", scene.device)
    x = rays["x"]
    N = x.numel() if n_rays is None else int(n_rays)
    single = scene.single_lambda
    cols = {k: _as_dev(rays[k], torch.float32, k, device, x.numel()) for k in READ_COLUMNS
            if not (single and k == "lmd_num")}
    _as_dev(rng_states, rng_states.dtype, "rng_states", device, x.numel())
    r = Rays(**{k: ctypes.c_void_p(v.data_ptr()) for k, v in cols.items()})
    nbytes = ctypes.sizeof(_lib.ShadowStats)
    buf = torch.zeros(nbytes // 8, dtype=torch.int64, device=device)
    check(load().wgrt_debug_shadow(scene.handle, ctypes.byref(r), N, int(gid_offset), int(single),
                                   ctypes.c_void_p(rng_states.data_ptr()),
                                   ctypes.c_void_p(per_ray_bounces.data_ptr()) if per_ray_bounces is not None else None,
                                   ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(_stream_handle(device, stream))),
          "wgrt_debug_shadow")
    host = buf.cpu().numpy()
    st = _lib.ShadowStats.from_buffer_copy(host.tobytes())
    return {"decisions": st.decisions, "uncertain": st.uncertain, "silent_flips": st.silent_flips,
            "bounces": st.bounces, "fallbacks": st.fallbacks, "max_ratio": st.max_ratio,
            "max_ratio32": st.max_ratio32,
            "max_ratio32_by_depth": dict(zip(SHADOW_DEPTHS, list(st.max_ratio_by_depth))),
            "decisions_by_depth": dict(zip(SHADOW_DEPTHS, [int(v) for v in st.decisions_by_depth])),
            "ratio32_hist_log10": {f"1e{b - 18}": int(v) for b, v in enumerate(st.ratio_hist) if v},
            "max_ener_ratio": st.max_ener_ratio, "max_amp": st.max_amp}


def selftest_math(a: torch.Tensor, b: torch.Tensor, stream=None) -> torch.Tensor:
    """Device sqrt, div, hypot_cr, atan2, sin, cos, wrap on (a, b) -> [7, n] float64."""
    n = a.numel()
    out = torch.empty((7, n), dtype=torch.float64, device=a.device)
    check(load().wgrt_selftest_math(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), n,
                                    ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(_stream_handle(a.device, stream))), "wgrt_selftest_math")
    return out


__all__ = ["Scene", "WgrtError", "TraceStats", "STATS_LEN", "new_stats", "check_stats", "block_runs",
           "trace_fullcolor", "trace_single", "init_rays", "schedule_by_lifetime",
           "rays_to_device", "classify_points", "shadow", "selftest_math", "RAY_COLUMNS", "_lib"]
