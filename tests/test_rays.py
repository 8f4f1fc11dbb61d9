"""Host ray layout (rays.build_rays / rng_seeds) against a literal restatement of the
reference's setup loop (gpu_ray_tracing_pro_fullColor.py:65-115, 158), including its
float index arithmetic for odd num_rays_per_FoV."""
import numpy as np
import pytest

from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import build_rays, rng_seeds

COLS = ("x", "y", "gap_x", "gap_y", "pol", "azi", "m", "n", "lmd_num", "te", "tm", "delta_phase")


def main_loop(points, nx, ny, lambdas, R):
    """MAIN:65-115 statement by statement (lmd_num takes the listed wavelength indices)."""
    size = R * nx * ny * len(lambdas)
    c = {k: np.zeros(size, dtype=np.float32) for k in COLS}
    num = 0
    for ii in range(nx):
        for jj in range(ny):
            for lam in lambdas:
                for te, tm in ((1, 0), (0, 1)):
                    start = int(num * R) if te else int(start + R / 2)
                    end = int(start + R / 2)
                    c["x"][start:end] = points[:, 0]
                    c["y"][start:end] = points[:, 1]
                    c["m"][start:end] = ii
                    c["n"][start:end] = jj
                    c["lmd_num"][start:end] = lam
                    c["te"][start:end] = te
                    c["tm"][start:end] = tm
                num += 1
    return c


@pytest.mark.parametrize("R", [64, 7, 2, 1])
@pytest.mark.parametrize("lambdas", [[0, 1, 2], [1]])
def test_build_rays_matches_main_loop(R, lambdas):
    rng = np.random.default_rng(R)
    pts = rng.uniform(-3, 3, size=(R // 2, 2))
    ref = main_loop(pts, 3, 2, lambdas, R)
    got = build_rays(pts, 3, 2, lambdas, R)
    for k in COLS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    lo, hi = 2, 5
    part = build_rays(pts, 3, 2, lambdas, R, blocks=(lo, hi)) if hi <= 6 * len(lambdas) else None
    if part is not None:
        for k in COLS:
            np.testing.assert_array_equal(part[k], ref[k][lo * R:hi * R], err_msg=k)


def test_rng_seeds_match_main():
    n = 1000
    ref = np.uint32(0x9E3779B9) * (np.arange(n, dtype=np.uint32) + np.uint32(1))   # MAIN:158
    np.testing.assert_array_equal(rng_seeds(n), ref)
    np.testing.assert_array_equal(rng_seeds(10, gid_offset=990), ref[990:])
