#!/usr/bin/env python3
"""A/B timing of library builds (exp_libs/<name>/libwgrt.so, tools/ab_build.py) on the bench
workload: rounds of one subprocess per build (tools/with_lib.py), interleaved, each timing `--launches`
single-trace launches and one fused `--fused`-trace call with HIP events; prints the per-build
medians.  Usage: python tools/ab.py NAME [NAME ...] [--rounds 4] [--config C3]"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
import numpy as np
sys.path.insert(0, os.environ["REPO"])
import torch
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import CONFIGS, build_inputs
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import hip_shard_builder, make_shard
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, trace_fullcolor, reserve, new_stats
import dataclasses
w = CONFIGS[os.environ["AB_CONFIG"]]
if os.environ.get("AB_PROFILE"):
    w = dataclasses.replace(w, profile=os.environ["AB_PROFILE"])
nx, ny, lam, R = w.nx, w.ny, list(w.lambdas), w.R
dev = torch.device("cuda", 0)
g, L, pts = build_inputs(w)
sc = Scene.from_geometry(g, L, **json.loads(os.environ.get("AB_SCENE") or "{}"))
lk = json.loads(os.environ.get("AB_LAUNCH") or "{}")
_dbg = {k[4:]: lk.pop(k) for k in [k for k in lk if k.startswith("dbg_")]}   # +dbg_<field>=v: wgrt_debug_opts
if _dbg: lk["debug"] = _dbg
nshard = int(os.environ.get("AB_SHARD") or 1)   # trace rank 0's interleaved shard of nshard (strong scaling)
shard = make_shard(nx, ny, len(lam), R, nshard, 0)
rays, rng = hip_shard_builder(pts, nx, ny, lam, R, dev)(shard)
if nshard > 1:
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import hip_tracer
    _gb = torch.as_tensor(shard.gid.block_gid, dtype=torch.int64, device=dev)
    _tf = trace_fullcolor
    def trace_fullcolor(sc, rays, rng, eb, **kw):
        _tf(sc, rays, rng, eb, gid_blocks=_gb, gid_block_rays=R, **kw)
eb = torch.zeros(sc.eb_shape(), dtype=torch.float32, device=dev)
st = new_stats(dev)
nl, nf = int(os.environ["AB_LAUNCHES"]), int(os.environ["AB_FUSED"])
reserve(sc, rays["x"].numel(), nf)
order = None
if os.environ.get("AB_ORDER"):   # lifetime-ordered chunk issue from one earlier launch
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import schedule_by_lifetime, CHUNK
    pb = torch.zeros(rays["x"].numel(), dtype=torch.int32, device=dev)
    trace_fullcolor(sc, rays, rng.clone(), eb.clone(), per_ray_bounces=pb)
    key = ((rays["lmd_num"].to(torch.int64) * nx + rays["m"].to(torch.int64)) * ny + rays["n"].to(torch.int64))
    if os.environ["AB_ORDER"] == "seg":
        order = schedule_by_lifetime(pb, key, nx * ny * 3)
    else:
        tot = torch.zeros(nx * ny * 3, device=dev).index_add_(0, key, pb.float())
        cnt = torch.zeros(nx * ny * 3, device=dev).index_add_(0, key, torch.ones_like(pb, dtype=torch.float32))
        ck = (tot / cnt.clamp_min(1))[key[::CHUNK]]
        order = torch.argsort(-ck, stable=True).to(torch.int32)
for _ in range(3): trace_fullcolor(sc, rays, rng, eb, chunk_order=order, **lk)
trace_fullcolor(sc, rays, rng, eb, num_iter=2)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nl + 1)]
st.zero_()
for k in range(nl):
    ev[k][0].record(); trace_fullcolor(sc, rays, rng, eb, stats=st, chunk_order=order, **lk); ev[k][1].record()
torch.cuda.synchronize()
b1 = int(st[0]) / nl
st.zero_()
ev[nl][0].record(); trace_fullcolor(sc, rays, rng, eb, stats=st, num_iter=nf); ev[nl][1].record()
torch.cuda.synchronize()
single = [ev[k][0].elapsed_time(ev[k][1]) for k in range(nl)]
print(json.dumps({"single_ms": float(np.median(single)), "fused_ms_per_step": ev[nl][0].elapsed_time(ev[nl][1]) / nf,
                  "bounces_per_launch": b1, "fused_bounces": int(st[0])}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--fused", type=int, default=20)
    ap.add_argument("--profile", default="", help="LUT profile override (luts.synthetic_luts)")
    ap.add_argument("--shard", type=int, default=1, help="time rank 0's interleaved shard of N instead of the batch")
    a = ap.parse_args()
    res = {n: [] for n in a.names}
    for r in range(a.rounds):
        for n in a.names:
            # NAME[:seg|:glob][@scene_opt=v,...][+launch_opt=v,...]: the build ("tree" = the in-tree
            # library), optionally with lifetime-ordered chunk issue, scene options (e.g. coarse_shift=-1)
            # and launch options (e.g. grid_sqrt_k=4.5)
            n0, _, lopts = n.partition("+")
            n0, _, sopts = n0.partition("@")
            build, _, order = n0.partition(":")
            num = lambda v: float(v) if "." in v else int(v)
            scene_kw = {k: num(v) for k, v in (kv.split("=") for kv in sopts.split(",") if kv)}
            launch_kw = {k: num(v) for k, v in (kv.split("=") for kv in lopts.split(",") if kv)}
            lib = os.path.join(REPO, "exp_libs", build, "libwgrt.so") if build != "tree" else ""
            env = dict(os.environ, REPO=REPO, AB_CONFIG=a.config, AB_LAUNCHES=str(a.launches),
                       AB_FUSED=str(a.fused), AB_ORDER=order, AB_SCENE=json.dumps(scene_kw),
                       AB_LAUNCH=json.dumps(launch_kw), AB_PROFILE=a.profile, AB_SHARD=str(a.shard))
            p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "with_lib.py"), lib, "--abi", "4,5,6,7", "-c",
                                CHILD], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode:
                print(p.stderr[-3000:])
                sys.exit(p.returncode)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res[n].append(d)
            print(r, n, json.dumps(d), flush=True)
    for n, v in res.items():
        s = np.median([d["single_ms"] for d in v])
        f = np.median([d["fused_ms_per_step"] for d in v])
        b = v[0]["bounces_per_launch"]
        print(f"SUMMARY {n}: single {s:.4f} ms ({b / s / 1e6:.3e} b/s), fused {f:.4f} ms/step ({b / f / 1e6:.3e} b/s)")


if __name__ == "__main__":
    main()
