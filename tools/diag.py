#!/usr/bin/env python3
"""Wave-loop diagnostics: builds libwgrt with -DWGRT_DIAG into /tmp and reports, per launch
of the persistent kernel on the C3 workload: loop passes, mean active lanes at the
interaction step (overall and after the work queue ran dry), miss hops and the SIMT cost of
the hop loop, and how often the certified branch decision fell back to the exact path."""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _build, _lib  # noqa: E402

import torch  # noqa: E402  (load torch's HIP runtime first, as the package always does)
torch.cuda.init()
out = "/tmp/libwgrt_diag.so"
cmd = [_build._hipcc(), *_build.FLAGS, "-DWGRT_DIAG=1", *os.environ.get("DIAG_FLAGS", "").split(),
       "-I", os.path.join(REPO, "include"), "-o", out] + \
      [os.path.join(_build.CSRC, f) for f in _build.SOURCES]
subprocess.run(cmd, check=True)
_lib.load(out)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, rays_to_device, trace_fullcolor  # noqa
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import build_rays, generate_points_in_polygon, rng_seeds  # noqa

R = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 3
K = int(sys.argv[3]) if len(sys.argv) > 3 else 1   # chained traces per launch (fused for variants 7-9)
geom = design_geometry(21, 21)
luts = synthetic_luts(geom, seed=0)
pts = generate_points_in_polygon(geom.IC, R // 2, rng=np.random.default_rng(1))
host = build_rays(pts, 21, 21, [0, 1, 2], R)
dev = torch.device("cuda", 0)
scene = Scene.from_geometry(geom, luts)
rays = rays_to_device(host, dev)
rng = torch.from_numpy(rng_seeds(host["x"].shape[0]).view(np.int32)).to(dev)
eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
st = torch.zeros(4, dtype=torch.int64, device=dev)
L = _lib._lib
L.wgrt_diag_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 17)()
acts = (ctypes.c_ulonglong * 16)()
L.wgrt_diag_read_wave_times.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
L.wgrt_diag_read_regions.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
# warm-up launch (caches, clocks), counters discarded
trace_fullcolor(scene, rays, rng.clone(), eb.clone(), variant=variant, num_iter=K)
torch.cuda.synchronize()
L.wgrt_diag_read(buf)
L.wgrt_diag_read_regions(acts)
L.wgrt_diag_read_wave_times((ctypes.c_ulonglong * (16384 * 3))())
trace_fullcolor(scene, rays, rng, eb, stats=st, variant=variant, num_iter=K)
torch.cuda.synchronize()
L.wgrt_diag_read_regions.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
L.wgrt_diag_read_regions(acts)
L.wgrt_diag_read(buf)
d = list(buf)
b = int(st[0])
print(f"R={R} variant={variant} num_iter={K} bounces={b} rays={host['x'].shape[0]} info={scene.info()}")
print(f"passes={d[0]} mean_active_at_interact={d[1] / max(d[0], 1):.1f}/64 "
      f"passes_after_exhaust={d[2]} ({d[2] / max(d[0], 1):.1%}) mean_active_after={d[3] / max(d[2], 1):.1f}")
print(f"lane_hops={d[4]} hops/pass(lane-mean)={d[4] / max(d[1], 1):.2f} simt_hop_cost/pass={d[5] / max(d[0], 1):.2f} "
      f"exact_fallbacks={d[16]} interactions~={d[1]} (variants 7-9: d5 = waiting lanes/pass {d[5] / max(d[0], 1):.2f})")
nb = max(d[0] - d[2], 1)
print(f"before dry, lanes per pass: interacting={(d[1] - d[3]) / nb:.1f} transit={d[14] / nb:.1f} free={d[13] / nb:.1f} "
      f"waiting={d[15] / nb:.1f} (variants 7-9)")
wt = (ctypes.c_ulonglong * (16384 * 3))()
L.wgrt_diag_read_wave_times.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
L.wgrt_diag_read_wave_times(wt)
w = np.array(wt, dtype=np.float64).reshape(-1, 3)
w = w[w[:, 0] > 0]
if len(w):
    t0 = w[:, 0].min()
    st, ex, en = (w[:, 0] - t0) / 100.0, (w[:, 1] - t0) / 100.0, (w[:, 2] - t0) / 100.0   # us
    ex = np.where(w[:, 1] > 0, ex, en)
    q = lambda a: " ".join(f"{v:.1f}" for v in np.percentile(a, [0, 10, 50, 90, 100]))
    print(f"waves={len(w)} start us [p0 p10 p50 p90 max]: {q(st)}")
    print(f"  queue-exhausted us: {q(ex)}")
    print(f"  end us:             {q(en)}")
    print(f"  tail (end - exhausted) us: {q(en - ex)}")
for r, name in enumerate(["interact", "take", "eyebox", "advance-iter", "edge-test", "ic-check", "refill-load"]):
    n, act = d[6 + r], acts[r]
    print(f"  region {name:13s} wave-execs={n:9d} mean_active={act / max(n, 1):5.1f}/64")
