"""Pin the CPU oracle (oracle/wgrt_oracle.c) to the reference's own kernel outputs.

The fixtures were produced by running GPU_ray_tracing_functions.py:833-1246
(full colour) and :419-831 (single wavelength, ``s*`` cases) unmodified
(tests/golden/gen_golden.py).  Bar: bit-exact rng_states,
matrix_EB and per-ray bounce counts after 1 and after 4 launches.
"""
import numpy as np
import pytest

from oracle import OracleScene
from tests._fixtures import CASES, GoldenCase


@pytest.fixture(scope="module", params=CASES)
def case(request):
    return GoldenCase(request.param)


def test_inputs_regenerate_bit_identically(case):
    assert case.digest_ok(), "geometry / synthetic-LUT generator drifted from the fixture"


@pytest.mark.parametrize("threads", [1, 4])
def test_oracle_matches_reference(case, threads):
    sc = OracleScene.from_geometry(case.geom, case.luts, wavelength=case.wavelength)
    rng = case.fresh_rng()
    eb = np.zeros(case.eb_shape(), np.float32)
    num_iter = int(case.f["num_iter"])
    for it in range(num_iter):
        tot, per_ray = sc.trace(case.rays, rng, eb, threads=threads, per_ray_bounces=True)
        np.testing.assert_array_equal(per_ray, case.f["bounces"][it])
        assert tot == int(case.f["bounces"][it].sum())
        if it == 0:
            np.testing.assert_array_equal(rng, case.f["rng_after1"])
            np.testing.assert_array_equal(eb, case.eb_expected(1))
    np.testing.assert_array_equal(rng, case.f["rng_after4"])
    np.testing.assert_array_equal(eb, case.eb_expected(4))


def test_oracle_sharding_invariance(case):
    """Tracing R-aligned gid ranges separately (with gid_offset) equals one pass."""
    sc = OracleScene.from_geometry(case.geom, case.luts, wavelength=case.wavelength)
    rng_full = case.fresh_rng()
    eb_full = np.zeros(case.eb_shape(), np.float32)
    sc.trace(case.rays, rng_full, eb_full)
    rng_sh = case.fresh_rng()
    eb_sh = np.zeros(case.eb_shape(), np.float32)
    cuts = [0, case.R, 3 * case.R, case.N]
    for a, b in zip(cuts[:-1], cuts[1:]):
        part = {k: v[a:b] for k, v in case.rays.items()}
        r = np.ascontiguousarray(rng_sh[a:b])
        sc.trace(part, r, eb_sh, gid_offset=a)
        rng_sh[a:b] = r
    np.testing.assert_array_equal(rng_sh, rng_full)
    np.testing.assert_array_equal(eb_sh, eb_full)


def test_single_wavelength_threshold_is_pinned():
    """s5_thr_532 reaches the 1e-15 energy guard of process_rays_kernel_pro (GRTF:444):
    the same trace with the full-colour kernel's guard (0, GRTF:859) must differ, so the
    fixture really pins the threshold."""
    case = GoldenCase("s5_thr_532")
    sc = OracleScene.from_geometry(case.geom, case.luts, wavelength=case.wavelength)
    sc._s.threshold = 0.0
    rng = case.fresh_rng()
    eb = np.zeros(case.eb_shape(), np.float32)
    _, per_ray = sc.trace(case.rays, rng, eb, per_ray_bounces=True)
    assert (per_ray != case.f["bounces"][0]).sum() > 10


def test_h6_fixture_exercises_eyebox_aliasing():
    """h6_edge_rgb pins GRTF:154-165's compiled-numba addressing: its four crafted out-couplings
    (gen_golden.craft_h6) land where only the aliasing puts them -- x == xmax on column 0 of the
    next row, the on-edge band left of xmin on column 119, y == ymax on row 0 of the next FoV's
    slab, the band below ymin on row 79 -- and each is counted after launch 1."""
    case = GoldenCase("h6_edge_rgb")
    ev = case.f["h6_events"]
    assert sorted(ev[:, 0].tolist()) == [0, 1, 2, 3]
    slab = case.ny * case.nx * 80 * 120
    eb1 = case.eb_expected(1).reshape(-1)
    for kind, gid, m, n, lam, off in ev:
        assert eb1[lam * slab + off] >= 1
        row, col, fov = (off // 120) % 80, off % 120, off // (80 * 120)
        if kind == 0:
            assert col == 0 and fov == n * case.nx + m
        elif kind == 1:
            assert col == 119 and fov == n * case.nx + m
        elif kind == 2:
            assert row == 0 and fov == n * case.nx + m + 1
        else:
            assert row == 79 and fov == n * case.nx + m


def test_event_hook_build_matches_reference(case):
    """The oracle's event-hook build (oracle/wgrt_oracle_ev.c: interaction counter, ener-underflow
    flags) is the same arithmetic: bit-exact on the fixtures too, with no ray in the underflow regime
    and fewer interactions than loop iterations."""
    sc = OracleScene.from_geometry(case.geom, case.luts, wavelength=case.wavelength)
    rng = case.fresh_rng()
    eb = np.zeros(case.eb_shape(), np.float32)
    tot, per_ray, inter, flags = sc.trace(case.rays, rng, eb, per_ray_bounces=True, interactions=True,
                                          underflow=True)
    np.testing.assert_array_equal(per_ray, case.f["bounces"][0])
    np.testing.assert_array_equal(rng, case.f["rng_after1"])
    np.testing.assert_array_equal(eb, case.eb_expected(1))
    traced = int((per_ray > 0).sum())
    assert 0 <= inter <= tot - traced
    assert not flags.any()
