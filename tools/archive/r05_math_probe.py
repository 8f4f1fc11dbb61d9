#!/usr/bin/env python3
"""Round-5 probe: the device's sin / cos / atan2 (wgrt_selftest_math) against glibc (numpy) over the
argument ranges the reference's unwrapped delta_phase reaches: ulp differences by |x|."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import selftest_math  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
out = {}
for lo, hi in ((0, 4), (4, 64), (64, 1024), (1024, 16384), (16384, 262144), (262144, 4194304)):
    x = rng.uniform(lo, hi, 200000) * rng.choice([-1, 1], 200000)
    y = rng.uniform(-1, 1, 200000)
    r = selftest_math(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)).cpu().numpy().reshape(7, -1)
    d = {}
    for k, name, ref in ((4, "sin", np.sin(x)), (5, "cos", np.cos(x)), (3, "atan2", np.arctan2(x, y))):
        g = r[k]
        ulp = np.abs(g - ref) / np.spacing(np.abs(ref))
        d[name] = {"differ_frac": float((g != ref).mean()), "max_ulp": float(ulp.max()),
                   "max_abs": float(np.abs(g - ref).max())}
    out[f"[{lo},{hi})"] = d
    print(lo, hi, json.dumps(d), flush=True)
json.dump(out, open("gpurun_out/r05_math_probe.json", "w"), indent=1)
