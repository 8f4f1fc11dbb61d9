#!/usr/bin/env python3
"""Where a launch-tail (drain) pass spends its cycles: the segment stamps of a -DWGRT_SEG build.

Build the diagnostic library first (never the product):
    python tools/ab_build.py seg=-DWGRT_SEG
then, on the GPU:
    python tools/with_lib.py exp_libs/seg/libwgrt.so tools/segments.py --out profiles/r06_pass_segments.json

For each workload (C3 whole batch, rank 0's interleaved eighth of C3, C2) it runs the timeline
instantiation of the trace kernel with the segment stamps (wgrt_device.h SegAcc): per wave, the shader
cycles of every launch-tail pass split into
    advance | retire + ballots | line-0 round trip | estimate + decision | taken loads round trip |
    field update | rest of the pass (in-coupler test, outcome, out-coupling queue)
The build forces vmcnt(0) at the end of the two round-trip segments and stamps with s_memtime, so its
passes run slower than the product's: read the SHARES.  Reported for all waves and for
the 1 % of waves that end last (the chain the launch waits for).  16 words per wave: the 8 timeline
words (engine.timeline_summary) and the 8 segment sums.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SEGS = ["advance", "retire_ballot", "line0_round_trip", "estimate_decision", "taken_loads_round_trip",
        "field_update", "rest_of_pass"]


def run(spec, reps):
    import torch
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import CONFIGS, build_inputs
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import hip_shard_builder, make_shard
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, trace_fullcolor

    cfg, _, nsh = spec.partition("/")
    nsh = int(nsh or 1)
    dev = torch.device("cuda", 0)
    w = CONFIGS[cfg]
    nx, ny, lam, R = w.nx, w.ny, list(w.lambdas), w.R
    geom, luts, pts = build_inputs(w)
    scene = Scene.from_geometry(geom, luts)
    shard = make_shard(nx, ny, len(lam), R, nsh, 0)
    rays, rng = hip_shard_builder(pts, nx, ny, lam, R, dev)(shard)
    kw = {} if nsh == 1 else dict(gid_blocks=torch.as_tensor(shard.gid.block_gid, dtype=torch.int64, device=dev),
                                  gid_block_rays=R)
    eb = torch.zeros(scene.eb_shape(), dtype=torch.float32, device=dev)
    nw = 256 * 8 * 4 * 2
    buf = torch.zeros(16 * nw, dtype=torch.int64, device=dev)   # engine: timeline_waves = numel / 8 = 2 nw
    for _ in range(2):
        trace_fullcolor(scene, rays, rng, eb, variant=7, **kw)
    out = []
    for _ in range(reps):
        buf.zero_()
        trace_fullcolor(scene, rays, rng, eb, variant=7, debug=dict(timeline=buf), **kw)
        torch.cuda.synchronize()
        t = buf.cpu().numpy().reshape(-1, 16)
        t = t[t[:, 0] > 0]
        start, exh, end = (t[:, k].astype(np.float64) for k in (0, 1, 2))
        seg = t[:, 8:15].astype(np.float64)
        npass = t[:, 15].astype(np.float64)
        tail_ticks = end - exh                          # s_memrealtime, 100 MHz
        cyc = seg.sum(axis=1)
        ok = (npass > 0) & (tail_ticks > 0)
        clock_ghz = float(cyc[ok].sum() / (tail_ticks[ok].sum() / 100e6) / 1e9)
        last = end >= np.percentile(end, 99)

        def shares(sel):
            tot = seg[sel].sum(axis=0)
            p = max(npass[sel].sum(), 1.0)
            return {"passes": float(p), "cycles_per_pass": round(float(tot.sum() / p), 1),
                    "segments_cycles_per_pass": {n: round(float(v / p), 1) for n, v in zip(SEGS, tot)},
                    "segments_share": {n: round(float(v / max(tot.sum(), 1.0)), 4) for n, v in zip(SEGS, tot)}}

        out.append({"waves": int(len(t)), "tail_waves": int(ok.sum()), "shader_clock_ghz": round(clock_ghz, 3),
                    "all_waves": shares(ok), "last_1pct_waves": shares(ok & last)})
        print(spec, json.dumps(out[-1]), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--specs", nargs="+", default=["C3", "C3/8", "C2"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {s: run(s, a.reps) for s in a.specs}
    if a.out:
        import hashlib
        from gpu_ray_tracing_for_waveguide_based_ar_display_amd._lib import loaded_path
        with open(loaded_path(), "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()[:16]
        with open(a.out, "w") as f:
            json.dump({"build": "-DWGRT_SEG", "lib_sha16": sha, "segments": SEGS, "runs": res,
                       "note": "diagnostic build: forced vmcnt(0) at the ends of the round-trip segments and "
                               "s_memtime stamps; read shares, not lengths (tools/segments.py)"}, f, indent=1)


if __name__ == "__main__":
    main()
