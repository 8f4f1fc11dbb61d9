#!/usr/bin/env python3
"""Host-side cost of one trace call against its GPU time (GPU box; analysis tool).

For the C3 batch and rank 0's shard of N (interleaved, strong scaling), times K back-to-back
single-trace calls through the bench's tracer (distributed.hip_tracer -> engine.trace_fullcolor ->
wgrt_trace_opts): the host time per call (enqueue only, perf_counter around each call), the wall
time per step of the K calls with one synchronize at the end, and the GPU time per step (HIP
events around the K calls).  A wall time above the GPU time means the host cannot keep the GPU fed.

    python tools/host_overhead.py --shards 1 8 --steps 200
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args(argv)

    import torch
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import CONFIGS, build_inputs
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import (hip_shard_builder, hip_tracer,
                                                                                make_shard)
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, new_stats, reserve

    w = CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    geom, luts, points = build_inputs(w)
    scene = Scene.from_geometry(geom, luts)
    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    stats = new_stats(dev)
    tracer = hip_tracer(scene, 0, stats)
    for n in a.shards:
        shard = make_shard(w.nx, w.ny, len(w.lambdas), w.R, n, 0)
        rays, rng = hip_shard_builder(points, w.nx, w.ny, list(w.lambdas), w.R, dev)(shard)
        reserve(scene, shard.n_rays, 1)
        for _ in range(5):
            tracer(rays, rng, eb, shard.gid)
        torch.cuda.synchronize()
        host = []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(a.steps):
            h0 = time.perf_counter()
            tracer(rays, rng, eb, shard.gid)
            host.append(time.perf_counter() - h0)
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        gpu = e0.elapsed_time(e1) / a.steps
        print(json.dumps({"config": a.config, "shard_of": n, "rays": shard.n_rays, "steps": a.steps,
                          "host_ms_per_call_median": round(float(np.median(host)) * 1e3, 4),
                          "host_ms_per_call_p90": round(float(np.percentile(host, 90)) * 1e3, 4),
                          "wall_ms_per_step": round(wall, 4), "gpu_ms_per_step": round(gpu, 4)}), flush=True)
        del rays, rng
    scene.close()


if __name__ == "__main__":
    main()
