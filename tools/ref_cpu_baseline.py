#!/usr/bin/env python3
"""CPU baseline of the REFERENCE's own kernel code: GRTF's
``process_rays_kernel_pro_fullColor`` imported unmodified under the test-only numba stub
(tests/golden/_stub_numba, sequential CUDA-simulator semantics -- what NUMBA_ENABLE_CUDASIM
does, without numba), sharded by global ray index over ``--procs`` forked processes.

Runs only in the build container (it needs /root/reference).  The bounce count of the job
comes from the CPU oracle (oracle/), which is bit-identical to the reference on the golden
fixtures; the reference run itself is what is timed (one launch, num_iter = 1).
Usage: python tools/ref_cpu_baseline.py --config C1|C2 [--procs 8] [--json out.json]
"""
import argparse
import builtins
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = os.environ.get("WGRT_REFERENCE", "/root/reference")
# BASELINE.json configs 1 and 2: single wavelength 532 nm (full-colour kernel, lmd index 1)
CONFIGS = {"C1": dict(nx=3, ny=3, R=64), "C2": dict(nx=11, ny=11, R=1024)}

_job = {}


def _setup(cfg):
    sys.path.insert(0, os.path.join(REPO, "tests", "golden", "_stub_numba"))
    sys.path.insert(1, REFERENCE)
    sys.path.insert(2, REPO)
    import numba.cuda as stub_cuda
    import GPU_ray_tracing_functions as G
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import build_rays
    G.range = lambda *a: builtins.range(*(int(v) for v in a))   # GRTF:905 range(1e5), as compiled numba accepts
    geom = design_geometry(cfg["nx"], cfg["ny"])
    luts = synthetic_luts(geom, seed=0)
    np.random.seed(1)
    pts = G.generate_points_in_polygon(geom.IC, cfg["R"] // 2)
    rays = build_rays(pts, cfg["nx"], cfg["ny"], [1], cfg["R"])
    N = rays["x"].shape[0]
    rng = np.uint32(0x9E3779B9) * (np.arange(N, dtype=np.uint32) + np.uint32(1))
    eb = np.zeros((len(geom.lmd), cfg["ny"], cfg["nx"], 80, 120), np.float32)
    args = (rays["x"], rays["y"], rays["gap_x"], rays["gap_y"], rays["pol"], rays["azi"], rays["m"], rays["n"],
            rays["lmd_num"], rays["te"], rays["tm"], rays["delta_phase"], rng, geom.IC, geom.FC, geom.FC_offset,
            geom.OC, geom.OC_offset, geom.n_g, geom.eff_reg1, geom.eff_reg2, geom.eff_reg_FOV,
            geom.eff_reg_FOV_range, luts["lut_ic1"], luts["lut_ic2"], luts["lut_ic3"], luts["lut_fc1"],
            luts["lut_fc2"], luts["lut_oc1"], luts["lut_oc2"], geom.lut_TIR, geom.lut_gap, eb)
    _job.update(G=G, stub=stub_cuda, args=args, N=N, geom=geom, luts=luts, rays=rays)


def _run(lo_hi):
    lo, hi = lo_hi
    G, stub, args = _job["G"], _job["stub"], _job["args"]
    fn = G.process_rays_kernel_pro_fullColor.fn
    t0 = time.perf_counter()
    for gid in range(lo, hi):
        stub._state.gid = gid
        fn(*args)
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1", choices=sorted(CONFIGS))
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    _setup(cfg)
    N = _job["N"]
    cuts = np.linspace(0, N, a.procs + 1).astype(int)
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(a.procs) as pool:
        per = pool.map(_run, list(zip(cuts[:-1], cuts[1:])))
    wall = time.perf_counter() - t0
    from oracle import OracleScene
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import rng_seeds
    sc = OracleScene.from_geometry(_job["geom"], _job["luts"])
    eb = np.zeros(sc.eb_shape(), np.float32)
    bounces, _ = sc.trace(_job["rays"], rng_seeds(N), eb, threads=8)
    res = dict(config=a.config, what="reference GRTF process_rays_kernel_pro_fullColor under the numba stub, "
                                     "one launch, 532 nm", nx=cfg["nx"], ny=cfg["ny"], R=cfg["R"], rays=int(N),
               bounces=int(bounces), procs=a.procs, wall_s=wall, max_proc_s=max(per),
               bounces_per_s=bounces / wall, host=os.uname().nodename, cpus=os.cpu_count())
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
