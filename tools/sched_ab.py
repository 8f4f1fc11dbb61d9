#!/usr/bin/env python3
"""Interleaved A/B of chunk issue orders for the persistent kernel on the C3 batch:
natural order vs. lifetime-scheduled order (engine.schedule_by_lifetime) learned from one
earlier launch; checks that outputs are identical from the same starting state."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import (Scene, init_rays, schedule_by_lifetime,
                                                                           trace_fullcolor)
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import generate_points_in_polygon

    variant = int(os.environ.get("SCHED_VARIANT", "2"))
    dev = torch.device("cuda", 0)
    nx = ny = 21
    geom = design_geometry(nx, ny)
    luts = synthetic_luts(geom, seed=0)
    pts = generate_points_in_polygon(geom.IC, 512, rng=np.random.default_rng(1))
    scene = Scene.from_geometry(geom, luts)
    rays, seeds = init_rays(pts, nx, ny, [0, 1, 2], 1024, device=dev)
    N = seeds.numel()
    tile = (rays["lmd_num"].long() * nx + rays["m"].long()) * ny + rays["n"].long()
    cnt = torch.zeros(N, dtype=torch.int32, device=dev)
    rng = seeds.clone()
    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    trace_fullcolor(scene, rays, rng, eb, per_ray_bounces=cnt, variant=variant)
    learned = rng.clone()   # the state a second launch starts from
    orders = {"natural": None, "tile_mean": schedule_by_lifetime(cnt, tile, 3 * nx * ny)}
    # reversed (worst case) for contrast
    orders["tile_mean_reversed"] = orders["tile_mean"].flip(0).contiguous()
    ref = None
    for name, o in orders.items():
        r = learned.clone()
        e = torch.zeros_like(eb)
        st = torch.zeros(4, dtype=torch.int64, device=dev)
        trace_fullcolor(scene, rays, r, e, stats=st, variant=variant, chunk_order=o)
        torch.cuda.synchronize()
        out = (r.cpu(), e.cpu(), st.cpu())
        if ref is None:
            ref = out
        else:
            same = all(torch.equal(a, b) for a, b in zip(out, ref))
            print(json.dumps({"order": name, "identical_to_natural": same}), flush=True)
    times = {k: [] for k in orders}
    for _ in range(10):
        for name, o in orders.items():
            r = learned.clone()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            trace_fullcolor(scene, rays, r, eb, variant=variant, chunk_order=o)
            e.record()
            torch.cuda.synchronize()
            times[name].append(s.elapsed_time(e))
    for name, t in times.items():
        print(json.dumps({"order": name, "variant": variant, "median_ms": round(float(np.median(t)), 4),
                          "min_ms": round(float(np.min(t)), 4)}), flush=True)


if __name__ == "__main__":
    main()
