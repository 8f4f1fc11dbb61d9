"""The C ABI from a plain C99 host (tests/capi_host.c: include/wgrt.h + the HIP runtime, no
Python or torch in the process): it uploads the scene (MAIN:40-57), runs the reference's
launch loop (MAIN:169-177) and copies the results back, and they must equal the reference's
own outputs for the same inputs (the golden fixture)."""
import os
import subprocess

import numpy as np
import pytest

from tests._capi import BIN, build_capi_host, read_output, write_input
from tests._fixtures import GoldenCase


def test_capi_host_compiles_against_header(tmp_path):
    """The header and the exported symbols are enough for a C99 host (-Wall -Wextra -Werror)."""
    out = build_capi_host(str(tmp_path / "capi_host"))
    assert os.access(out, os.X_OK)


def test_capi_host_rejects_bad_input(tmp_path):
    """A truncated input file is refused before any GPU call (no device needed)."""
    exe = build_capi_host(str(tmp_path / "capi_host"))
    bad = tmp_path / "bad.bin"
    bad.write_bytes(b"\x01\x00")
    p = subprocess.run([exe, str(bad), str(tmp_path / "out.bin")], capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "truncated input" in p.stderr


@pytest.mark.gpu
def test_capi_host_matches_golden(tmp_path):
    """c1_rgb (3x3 FoV x 3 lambda x 64 rays) x 4 launches through the C host: RNG states,
    eyebox grid and bounce count equal the reference kernel's outputs bit for bit."""
    if not os.access(BIN, os.X_OK):
        pytest.fail(f"{BIN} is missing: run __graft_entry__.build()")
    case = GoldenCase("c1_rgb")
    n_iter = int(case.f["num_iter"])
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    write_input(str(src), case.geom, case.luts, case.rays, case.fresh_rng(), n_iter)
    p = subprocess.run([BIN, str(src), str(dst)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    rng, eb, stats = read_output(str(dst), case.N, case.eb_shape())
    np.testing.assert_array_equal(rng, case.f["rng_after4"])
    np.testing.assert_array_equal(eb, case.eb_expected(4))
    assert int(stats[0]) == int(case.f["bounces"].sum())   # wgrt_trace_stats.bounces
    assert int(stats[2]) == int(case.eb_expected(4).sum())  # eyebox_hits
