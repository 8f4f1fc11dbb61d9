#!/usr/bin/env python3
"""A/B of library builds: times the C3 launch (default variant) with each given libwgrt
build in a fresh process, alternating A B A B ... for --rounds rounds.
Usage: python tools/ab_libs.py [--rounds 3] [--variant 0] [--n N] lib1.so lib2.so ..."""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, %(repo)r)
torch.cuda.init()
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _lib
_lib.load(%(lib)r)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, init_rays, trace_fullcolor
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import generate_points_in_polygon
g = design_geometry(21, 21); L = synthetic_luts(g, seed=0)
pts = generate_points_in_polygon(g.IC, 512, rng=np.random.default_rng(1))
dev = torch.device("cuda", 0)
sc = Scene.from_geometry(g, L)
rays, seeds = init_rays(pts, 21, 21, [0, 1, 2], 1024, device=dev)
n = %(n)d or seeds.numel()
eb = torch.zeros(sc.eb_shape(), dtype=torch.float32, device=dev)
ts = []; bs = []; rs = None
for k in range(15):
    rng = seeds.clone(); st = torch.zeros(4, dtype=torch.int64, device=dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); trace_fullcolor(sc, rays, rng, eb, n_rays=n, stats=st, variant=%(variant)d, num_iter=%(k)d); b.record()
    torch.cuda.synchronize()
    if k >= 3: ts.append(a.elapsed_time(b)); bs.append(int(st[0]))
    if rs is None: rs = int(rng[:n].double().sum().item())
print(json.dumps({"ms": float(np.median(ts)), "min_ms": float(np.min(ts)), "bounces": bs[0], "rng_sum": rs}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--num-iter", type=int, default=1)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    res = {lib: [] for lib in a.libs}
    for _ in range(a.rounds):
        for lib in a.libs:
            r = subprocess.run([sys.executable, "-c", RUN % dict(repo=REPO, lib=os.path.abspath(lib), n=a.n,
                                                                  variant=a.variant, k=a.num_iter)],
                               capture_output=True, text=True, timeout=300)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if not line:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            res[lib].append(json.loads(line[-1]))
    for lib, rs in res.items():
        ms = sorted(x["ms"] for x in rs)
        print(json.dumps({"lib": os.path.basename(lib), "median_ms": ms[len(ms) // 2], "all_ms": ms,
                          "bounces": rs[0]["bounces"], "rng_sum": rs[0]["rng_sum"]}), flush=True)


if __name__ == "__main__":
    main()
