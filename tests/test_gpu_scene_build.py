"""The device scene build (wgrt_scene_create: locator cell words by edge_mark_kernel /
classify_cells_kernel, LUT tiles by pack_tiles_kernel) against the host build of the same rules
(wgrt_scene_opts.host_build): identical cell words and tiles, byte for byte.  The one exception
allowed is the certification bound W of the Jones tiles (kJBlockW, and its sum in the float slot
kJBlockF32), which takes hypot on each side's libm: within 1e-14 relative (measured: 5 ulp), and
the float sum within 1e-6.  Also records the scene-creation time of both builds
at the reference's default 100x75 FoV grid (MAIN:16-17)."""
import json
import os
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

RESULTS = os.environ.get("WGRT_RESULTS_DIR", os.path.join(os.path.dirname(os.path.dirname(__file__)), "gpurun_out"))
KJ_HEADER, KJ_BLOCK, KJ_W, KJ_F32 = 16, 48, 40, 2


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _lib
    return _lib.load()


def _scene(geom, luts, host, wavelength=None):
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene
    t = time.perf_counter()
    sc = Scene.from_geometry(geom, luts, wavelength=wavelength, host_build=host)
    torch.cuda.synchronize()
    return sc, time.perf_counter() - t


def _w_mask(jd):
    """(W[k] doubles, the {Wsum, cosA_2} float pair) of every Jones block"""
    m, f = np.zeros(jd, bool), np.zeros(jd, bool)
    for b in range((jd - KJ_HEADER) // KJ_BLOCK):
        o = KJ_HEADER + KJ_BLOCK * b
        m[o + KJ_W:o + KJ_W + 3] = True
        f[o + KJ_F32] = True
    return m, f


@pytest.mark.parametrize("nx,ny,profile,wl", [(3, 3, "default", None), (21, 21, "default", None),
                                              (21, 21, "deep", None), (9, 7, "balanced", 2),
                                              (9, 7, "adversarial_singular", None),
                                              (100, 75, "default", None)])
def test_device_scene_equals_host_build(lib, nx, ny, profile, wl):
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    geom = design_geometry(nx, ny)
    luts = synthetic_luts(geom, seed=1, profile=profile)
    dev, t_dev = _scene(geom, luts, host=False, wavelength=wl)
    hst, t_host = _scene(geom, luts, host=True, wavelength=wl)
    try:
        assert dev.info()["grid_edge_cells"] == hst.info()["grid_edge_cells"] > 0
        np.testing.assert_array_equal(dev.debug_copy("cells"), hst.debug_copy("cells"))
        assert dev.debug_copy("tiles").tobytes() == hst.debug_copy("tiles").tobytes()
        jd, jh = dev.debug_copy("jtiles"), hst.debug_copy("jtiles")
        w, f = _w_mask(jd.shape[1])
        assert jd[:, ~(w | f)].tobytes() == jh[:, ~(w | f)].tobytes()
        np.testing.assert_allclose(jd[:, w], jh[:, w], rtol=1e-14, atol=0)
        fd, fh = np.ascontiguousarray(jd[:, f]).view(np.float32), np.ascontiguousarray(jh[:, f]).view(np.float32)
        np.testing.assert_array_equal(fd[:, 1::2], fh[:, 1::2])            # cosA_2: exact
        np.testing.assert_allclose(fd[:, 0::2], fh[:, 0::2], rtol=1e-6, atol=0)   # Wsum
    finally:
        dev.close()
        hst.close()
    if (nx, ny) == (100, 75):
        os.makedirs(RESULTS, exist_ok=True)
        rec = {"fov": [nx, ny], "lambdas": 3, "tiles": 3 * nx * ny, "device_build_s": round(t_dev, 3),
               "host_build_s": round(t_host, 3)}
        with open(os.path.join(RESULTS, "scene_create_100x75.json"), "w") as f:
            json.dump(rec, f, indent=1)
        print(rec)


@pytest.mark.parametrize("profile,flagged", [("default", False), ("stress", False), ("adversarial_singular", True),
                                             ("adversarial_rank1", True), ("adversarial_polarizing", True)])
def test_nonunitary_blocks_flagged(lib, profile, flagged):
    """The sign bit of a Jones block's float Wsum (wgrt_pack.h) flags a block whose taken branches' matrices are
    not scaled-unitary (kappa^2 > 1 + 1e-6): the Jones lane runs its amplification step there only.  The
    synthetic profiles' matrices are scaled-unitary (luts._jones) -- no block flagged -- and the adversarial
    near-singular / rank-one ones are not -- every block with a taken branch flagged, the in-coupling
    event's block 0 and every interaction block."""
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    geom = design_geometry(9, 7)
    sc, _ = _scene(geom, synthetic_luts(geom, seed=1, profile=profile), host=False)
    try:
        j = sc.debug_copy("jtiles")
        _, f = _w_mask(j.shape[1])
        wsum = np.ascontiguousarray(j[:, f]).view(np.float32)[:, 0::2]
        assert bool((wsum < 0).all()) if flagged else bool((wsum > 0).all()), (profile, int((wsum < 0).sum()), wsum.size)
        assert sc.info()["nonunitary_blocks"] == int((wsum < 0).sum())   # ABI 7: the AMP kernels run iff > 0
    finally:
        sc.close()
