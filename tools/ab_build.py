#!/usr/bin/env python3
"""Build variants of libwgrt.so with extra compile definitions for A/B timing (tools/ab.py).
Usage: python tools/ab_build.py NAME=-DFOO,-DBAR ...   -> exp_libs/NAME/libwgrt.so
(exp_libs/ is git-ignored; it travels to the GPU box with the tree.)"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _build  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition("=")
    out = os.path.join(REPO, "exp_libs", name)
    os.makedirs(out, exist_ok=True)
    lib = os.path.join(out, "libwgrt.so")
    cmd = [_build._hipcc(), *_build.FLAGS, *[d for d in defs.split(",") if d], "-I", os.path.join(REPO, "include"),
           "-o", lib] + [os.path.join(_build.CSRC, f) for f in _build.SOURCES]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr)
    print(name, lib)
