#!/usr/bin/env python3
"""Kernel time vs batch size: how much of a launch is the longest ray's serial chain.

Traces the first n rays of the C3 batch (21x21x3, R=1024) for several n and prints the
kernel time (HIP events, median of 10), the total and the maximum per-ray bounce count.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, init_rays, trace_fullcolor
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import generate_points_in_polygon

    variant = int(os.environ.get("PROBE_VARIANT", "0"))
    dev = torch.device("cuda", 0)
    geom = design_geometry(21, 21)
    luts = synthetic_luts(geom, seed=0)
    pts = generate_points_in_polygon(geom.IC, 512, rng=np.random.default_rng(1))
    scene = Scene.from_geometry(geom, luts)
    rays, seeds = init_rays(pts, 21, 21, [0, 1, 2], 1024, device=dev)
    N = seeds.numel()
    # shuffle so a prefix is a fair sample of FoV x wavelength blocks
    perm = torch.from_numpy(np.random.default_rng(0).permutation(N)).to(dev)
    rays = {k: v[perm].contiguous() for k, v in rays.items()}
    seeds = seeds[perm].contiguous()
    for n in (1024, 8192, 65536, 262144, N):
        times = []
        for _ in range(10):
            rng = seeds.clone()
            eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
            cnt = torch.zeros(N, dtype=torch.int32, device=dev)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            trace_fullcolor(scene, rays, rng, eb, n_rays=n, per_ray_bounces=cnt, variant=variant)
            e.record()
            torch.cuda.synchronize()
            times.append(s.elapsed_time(e))
        c = cnt[:n].cpu().numpy()
        print(json.dumps({"n": n, "ms": round(float(np.median(times)), 4), "bounces": int(c.sum()),
                          "max_bounces": int(c.max()), "p99": float(np.percentile(c, 99)),
                          "mean": round(float(c.mean()), 2)}), flush=True)


if __name__ == "__main__":
    main()
