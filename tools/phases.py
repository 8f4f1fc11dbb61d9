#!/usr/bin/env python3
"""Per-phase cycle breakdown of the persistent loop (build with -DWGRT_PHASES into /tmp):
advance / refill / interact shader cycles per pass, before and after the work queue ran dry,
and the per-wave timeline (start, queue exhausted, end).  Usage: phases.py [variant] [R]"""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _build, _lib  # noqa: E402

import torch  # noqa: E402
torch.cuda.init()
variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
R = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
extra = os.environ.get("PHASE_FLAGS", "").split()
out = "/tmp/libwgrt_phases.so"
cmd = [_build._hipcc(), *_build.FLAGS, "-DWGRT_PHASES=1", *extra, "-I", os.path.join(REPO, "include"), "-o", out] + \
      [os.path.join(_build.CSRC, f) for f in _build.SOURCES]
subprocess.run(cmd, check=True)
_lib.load(out)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, init_rays, trace_fullcolor  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import generate_points_in_polygon  # noqa: E402

g = design_geometry(21, 21)
luts = synthetic_luts(g, seed=0)
pts = generate_points_in_polygon(g.IC, R // 2, rng=np.random.default_rng(1))
dev = torch.device("cuda", 0)
sc = Scene.from_geometry(g, luts)
rays, seeds = init_rays(pts, 21, 21, [0, 1, 2], R, device=dev)
eb = torch.zeros(sc.eb_shape(), dtype=torch.float32, device=dev)
L = _lib._lib
L.wgrt_diag_read_phases.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]
ph = (ctypes.c_ulonglong * 16)()
wt = (ctypes.c_ulonglong * (16384 * 3))()
for it in range(4):
    rng = seeds.clone()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    trace_fullcolor(sc, rays, rng, eb, variant=variant, workgroups=int(os.environ.get("PHASE_WG", "0")),
                    num_iter=int(os.environ.get("PHASE_ITER", "1")))
    b.record()
    torch.cuda.synchronize()
    L.wgrt_diag_read_phases(ph, wt)
ms = a.elapsed_time(b)
p = list(ph)
print(f"variant={variant} R={R} num_iter={os.environ.get('PHASE_ITER', '1')} flags={extra} kernel {ms:.3f} ms")
for tag, o in (("before dry", 0), ("after dry ", 4)):
    n = max(p[o + 3], 1)
    tot = p[o] + p[o + 1] + p[o + 2]
    print(f"{tag}: passes={p[o + 3]} cycles/pass advance={p[o] / n:.0f} refill={p[o + 1] / n:.0f} "
          f"interact={p[o + 2] / n:.0f} total={tot / n:.0f}")
if p[11] or p[12]:
    print(f"drain at pass start (cycles/pass): before dry {p[11] / max(p[3], 1):.0f}, after dry {p[12] / max(p[7], 1):.0f}")
w = np.array(wt, dtype=np.float64).reshape(-1, 3)
w = w[w[:, 0] > 0]
t0 = w[:, 0].min()
st, ex, en = (w[:, 0] - t0) / 100.0, (w[:, 1] - t0) / 100.0, (w[:, 2] - t0) / 100.0
ex = np.where(w[:, 1] > 0, ex, en)
q = lambda a: " ".join(f"{v:.1f}" for v in np.percentile(a, [0, 10, 50, 90, 100]))
print(f"waves={len(w)}  [p0 p10 p50 p90 max] us")
print(f"  start      {q(st)}")
print(f"  exhausted  {q(ex)}")
print(f"  end        {q(en)}")
print(f"  tail       {q(en - ex)}")
