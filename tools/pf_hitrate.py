#!/usr/bin/env python3
"""How often the launch tail's line-0 prefetch (commit 6b094d1, DESIGN.md §5.2 "The lever") predicted the
block of the next interaction: a diagnostic build of that commit counts, per tail interaction, a hit
(blk == the prefetched block), a miss, or no prediction, into two stats words it does not otherwise use
in single launches (libm_rays: hits; handoff_giveups: misses | none << 32).

    (on 6b094d1's sources, with the ballot counters added under WGRT_PF_DIAG)
    python tools/ab_build.py pfdiag=-DWGRT_TAIL_PREFETCH=1,-DWGRT_PF_DIAG
    python tools/with_lib.py exp_libs/pfdiag/libwgrt.so tools/pf_hitrate.py --out gpurun_out/pf_hitrate.json
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(spec):
    import torch
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.configs import CONFIGS, build_inputs
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.distributed import hip_shard_builder, make_shard
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, new_stats, trace_fullcolor

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
    st = new_stats(dev)
    trace_fullcolor(scene, rays, rng, eb, variant=7, stats=st, **kw)
    torch.cuda.synchronize()
    s = [int(v) for v in st.cpu().tolist()]
    hit, miss, none = s[6], s[4] & 0xFFFFFFFF, s[4] >> 32
    tot = max(hit + miss + none, 1)
    rec = {"tail_interactions": hit + miss + none, "hit": hit, "miss": miss, "none": none,
           "hit_frac": round(hit / tot, 4), "miss_frac": round(miss / tot, 4), "none_frac": round(none / tot, 4),
           "interactions_total": s[5]}
    scene.close()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--specs", default="C3,C3/8,C2")
    a = ap.parse_args()
    res = {}
    for spec in a.specs.split(","):
        res[spec] = run(spec)
        print(spec, json.dumps(res[spec]), flush=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
