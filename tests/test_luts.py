"""The RCWA LUT loader (reference MAIN:28-34, download_lut.py:5-19): ``.npy`` round trips in
both precisions, rejection of tables that do not match the geometry, and a loaded set tracing
exactly like the in-memory set it was written from.

The reference's own files are not available offline, so the tables are the seeded synthetic
set written with ``save_luts`` (``np.save``) -- the same on-disk format the reference reads.
"""
import os
import warnings

import numpy as np
import pytest

from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import (LUT_NAMES, LUTPrecisionWarning, load_luts,
                                                                     save_luts, synthetic_luts, validate_luts)

NX, NY = 3, 2


@pytest.fixture(scope="module")
def setup():
    geom = design_geometry(NX, NY)
    return geom, synthetic_luts(geom, seed=3)


def _validate(geom, luts):
    return validate_luts(luts, len(geom.lmd), NX, NY, geom.num_fc_slices, geom.num_oc_slices)


def test_npy_roundtrip_complex128(setup, tmp_path):
    geom, luts = setup
    save_luts(luts, str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == sorted(n + "_fullColor.npy" for n in LUT_NAMES)
    got = load_luts(str(tmp_path))
    with warnings.catch_warnings():
        warnings.simplefilter("error", LUTPrecisionWarning)
        v = _validate(geom, got)
    for n in LUT_NAMES:
        assert got[n].dtype == np.complex128
        np.testing.assert_array_equal(v[n], luts[n])
    assert validate_luts.last_dtypes["lut_ic1"] == np.complex128


def test_npy_roundtrip_complex64(setup, tmp_path):
    """complex64 files load as stored and widen exactly; the precision caveat is raised."""
    geom, luts = setup
    save_luts(luts, str(tmp_path), dtype=np.complex64)
    got = load_luts(str(tmp_path))
    assert all(got[n].dtype == np.complex64 for n in LUT_NAMES)
    with pytest.warns(LUTPrecisionWarning, match="complex128"):
        v = _validate(geom, got)
    for n in LUT_NAMES:
        assert v[n].dtype == np.complex128
        np.testing.assert_array_equal(v[n], luts[n].astype(np.complex64).astype(np.complex128))
    assert validate_luts.last_dtypes["lut_oc2"] == np.complex64


def test_real_tables_accepted(setup):
    geom, luts = setup
    real = {n: luts[n].real.copy() for n in LUT_NAMES}
    v = _validate(geom, real)
    np.testing.assert_array_equal(v["lut_fc1"].real, luts["lut_fc1"].real)
    assert not v["lut_fc1"].imag.any()


@pytest.mark.parametrize("name,mutate,msg", [
    ("lut_ic1", lambda a: a[:, :-1], "does not match grid"),                 # FoV x one short
    ("lut_fc2", lambda a: a[:-1], "does not match grid"),                    # one FC slice short
    ("lut_oc1", lambda a: a[None], "does not match grid"),                   # extra leading axis
    ("lut_ic1", lambda a: a[..., :40], "kernel reads channel 40"),           # ic1 channel 40 (GRTF:866-869)
    ("lut_fc1", lambda a: a[..., :18], "kernel reads channel 18"),
    ("lut_ic2", lambda a: a.astype(object), "is not complex/real floating"),
    ("lut_oc2", lambda a: np.zeros(a.shape, np.int32), "is not complex/real floating"),
])
def test_rejects_mismatched_tables(setup, name, mutate, msg):
    geom, luts = setup
    bad = dict(luts)
    bad[name] = mutate(luts[name])
    with pytest.raises(ValueError, match=msg):
        _validate(geom, bad)


def test_rejects_missing_table(setup):
    geom, luts = setup
    bad = {n: luts[n] for n in LUT_NAMES if n != "lut_fc2"}
    with pytest.raises(ValueError, match="missing LUT lut_fc2"):
        _validate(geom, bad)


def test_missing_file_and_pickled_file_refused(setup, tmp_path):
    geom, luts = setup
    save_luts(luts, str(tmp_path))
    os.remove(tmp_path / "lut_oc1_fullColor.npy")
    with pytest.raises(FileNotFoundError):
        load_luts(str(tmp_path))
    # an object array can only be stored pickled: the loader never unpickles
    np.save(tmp_path / "lut_oc1_fullColor.npy", np.empty(3, dtype=object), allow_pickle=True)
    with pytest.raises(ValueError):
        load_luts(str(tmp_path))


def test_loaded_set_traces_like_in_memory(setup, tmp_path):
    """A set written to .npy and loaded back traces bit-identically (CPU oracle)."""
    from oracle import OracleScene
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import build_rays, generate_points_in_polygon, rng_seeds
    geom, luts = setup
    save_luts(luts, str(tmp_path))
    loaded = _validate(geom, load_luts(str(tmp_path)))
    R = 64
    pts = generate_points_in_polygon(geom.IC, R // 2, rng=np.random.default_rng(7))
    rays = build_rays(pts, NX, NY, [0, 1, 2], R)
    res = []
    for tabs in (luts, loaded):
        sc = OracleScene.from_geometry(geom, tabs)
        rng = rng_seeds(rays["x"].shape[0])
        eb = np.zeros(sc.eb_shape(), np.float32)
        tot, cnt = sc.trace(rays, rng, eb, threads=2, per_ray_bounces=True)
        res.append((tot, cnt, rng, eb))
    assert res[0][0] == res[1][0] > 0
    for a, b in zip(res[0][1:], res[1][1:]):
        np.testing.assert_array_equal(a, b)


def test_complex64_tables_take_float32_cosines():
    """Compiled numba takes math.cos of a complex64 table's float32 .real in float32 (GRTF:866-869);
    the oracle does so for the tables lut_f32_mask flags, and on the crafted case that flips ray 0's
    in-coupling decision (tests/_fixtures.complex64_case)."""
    import ctypes
    import math
    from oracle import OracleScene
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import lut_f32_mask
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import rng_seeds
    from tests._fixtures import complex64_case
    libm = ctypes.CDLL("libm.so.6")
    libm.cosf.restype, libm.cosf.argtypes = ctypes.c_float, [ctypes.c_float]
    th = 0.7000002264976501
    assert float(libm.cosf(th)) == 0.7648420333862305 and math.cos(th) == 0.7648420413706765
    geom, luts, rays = complex64_case()
    assert lut_f32_mask(luts) == 0x7f
    assert lut_f32_mask({k: v.astype(np.complex128) for k, v in luts.items()}) == 0
    wide = {k: v.astype(np.complex128) for k, v in luts.items()}
    out = {}
    for mask in (0, 0x7f):
        rng = rng_seeds(rays["x"].shape[0])
        eb = np.zeros((3, 3, 3, 80, 120), np.float32)
        _, per = OracleScene.from_geometry(geom, wide, f32_mask=mask).trace(rays, rng, eb, per_ray_bounces=True)
        out[mask] = (per, rng)
    assert out[0][0][0] != out[0x7f][0][0] or out[0][1][0] != out[0x7f][1][0]   # ray 0 decided differently
    np.testing.assert_array_equal(out[0][0][1:], out[0x7f][0][1:])              # every other ray alike


def test_adversarial_profiles():
    """luts.PROFILES' adversarial sets: near-singular Jones matrices whose largest
    singular value squared is the target efficiency, and lossless even splits summing to 1 - 1e-9."""
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import PROFILES, _jones_singular
    rng = np.random.default_rng(3)
    scale = rng.uniform(0.1, 0.9, 500)
    a, b, c, d = _jones_singular(rng, scale.shape, scale, 1e6)
    M = np.stack([np.stack([a, b], -1), np.stack([c, d], -1)], -2)
    sv = np.linalg.svd(M, compute_uv=False)
    np.testing.assert_allclose(sv[:, 0] ** 2, scale, rtol=1e-12)
    assert (sv[:, 0] / sv[:, 1]).min() > 1e5
    p = PROFILES["adversarial_lossless"]
    assert p["jitter"] == 0.0
    assert abs(sum(p["ic"]) - (1 - 1e-9)) < 1e-15
    assert abs(p["oc_turn"] + p["oc_out"][0] + (p["oc_keep"] - p["oc_turn"] - p["oc_out"][0]) - (1 - 1e-9)) < 1e-15
