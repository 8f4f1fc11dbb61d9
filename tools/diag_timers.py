#!/usr/bin/env python3
"""Per-phase latency of the bounce loop (diagnostic build, grid kernel): shader-clock
cycles per interaction (tile fetch + sincos + branch fields / decision / take or eyebox)
and per advance() call, at a near-idle GPU (n = 1024 rays) and at the full C3 batch."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _build, _lib  # noqa: E402

import torch  # noqa: E402
torch.cuda.init()
out = "/tmp/libwgrt_timers.so"
cmd = [_build._hipcc(), *_build.FLAGS, "-DWGRT_TIMERS=1", "-I", os.path.join(REPO, "include"), "-o", out] + \
      [os.path.join(_build.CSRC, f) for f in _build.SOURCES]
subprocess.run(cmd, check=True)
_lib.load(out)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, init_rays, trace_fullcolor  # noqa
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import generate_points_in_polygon  # noqa: E402

dev = torch.device("cuda", 0)
geom = design_geometry(21, 21)
luts = synthetic_luts(geom, seed=0)
pts = generate_points_in_polygon(geom.IC, 512, rng=np.random.default_rng(1))
scene = Scene.from_geometry(geom, luts)
rays, seeds = init_rays(pts, 21, 21, [0, 1, 2], 1024, device=dev)
N = seeds.numel()
perm = torch.from_numpy(np.random.default_rng(0).permutation(N)).to(dev)
rays = {k: v[perm].contiguous() for k, v in rays.items()}
seeds = seeds[perm].contiguous()
L = _lib._lib
L.wgrt_diag_read_timers.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
for n in (1024, 65536, N):
    for rep in range(3):
        rng = seeds.clone()
        eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
        st = torch.zeros(4, dtype=torch.int64, device=dev)
        L.wgrt_diag_read_timers(buf)   # reset
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        trace_fullcolor(scene, rays, rng, eb, n_rays=n, stats=st, variant=1)
        b.record()
        torch.cuda.synchronize()
        L.wgrt_diag_read_timers(buf)
    d = list(buf)
    ni, na = max(d[4], 1), max(d[5], 1)
    print(json.dumps({"n": n, "ms": round(a.elapsed_time(b), 4), "bounces": int(st[0]), "interacts": d[4],
                      "advance_calls": d[5], "cyc_per_interact_fields": round(d[0] / ni, 1),
                      "cyc_per_interact_decide": round(d[1] / ni, 1), "cyc_per_interact_take": round(d[2] / ni, 1),
                      "cyc_per_advance": round(d[3] / na, 1),
                      "cyc_per_advance_iteration": round(d[3] / max(int(st[0]) - n, 1), 1)}), flush=True)
