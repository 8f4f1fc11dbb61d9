"""System evaluation of the eyebox grid (reference ``AR_system_evaluation_functions.py``).

Restates ``evaluation(matrix_EB)`` (EVAL:45-163) without colour-science or OpenCV, which
are absent here.  Returns the same four outputs ``(delta_e, U_fov, U_EB, output_image)``:

* eye positions: the reference samples a 30-px circular pupil at every 8 px (y) and every
  12 px (x) of the 80 x 120 eyebox grid instead of convolving (EVAL:66-109);
* the pure-white sRGB image is mapped to per-wavelength weights with the inverse sensor
  matrix (EVAL:47-52, 112-118) and multiplied by the FoV-flipped pupil-integrated eyebox
  efficiency (EVAL:121);
* per eye position the image is mapped back to sRGB, gamma-encoded, brightness-normalised
  in HSV (EVAL:18-43, via cv2 in the reference), and converted to XYZ / CIELAB to take the
  mean CIEDE2000 difference to D65 white, the FoV uniformity min(Y)/max(Y), and the mean Y
  for the eyebox uniformity (EVAL:122-163).

Third-party pieces restated here (parity unpinned -- neither library is available to pin
against, and the reference has no tests):

* ``colour.XYZ_to_Lab``: the CIE 1976 formula with the CIE 1931 2-degree D65 white point
  xy = (0.3127, 0.3290), applied to XYZ as given (the reference feeds XYZ scaled to Y = 100
  for both the image and the white, which the formula then treats as 100x the white);
* ``colour.sd_to_XYZ(SDS_ILLUMINANTS['D65'])`` normalised to Y = 100: the ASTM E308 D65 /
  2-degree white point (95.047, 100, 108.883), since the spectral tables are not available;
* ``colour.delta_E(..., method='CIE 2000')``: CIEDE2000 after Sharma, Wu & Dalal (2005),
  k_L = k_C = k_H = 1;
* ``cv2.cvtColor`` RGB <-> HSV on float32: OpenCV's float HSV conversion (H in degrees).
"""
from __future__ import annotations

import numpy as np

M_SENSOR = np.array([
    [1.67430115, -0.76582385, -0.06172232],
    [-0.12551154, 1.47840695, -0.04124377],
    [-0.01826868, -0.13098157, 1.61444037],
])
M_XYZ = np.array([
    [6.424000e-01, 1.891400e-01, 2.511000e-01],
    [2.650000e-01, 8.849624e-01, 7.390000e-02],
    [4.999999e-05, 3.693564e-02, 1.528100e+00],
])
D65_XY = (0.3127, 0.3290)
XYZ_D65_ASTM = np.array([95.047, 100.0, 108.883])
_FLT_EPS = np.float32(np.finfo(np.float32).eps)


def linearize_srgb(image_srgb):
    """sRGB (0-1) -> linear RGB (EVAL:5-9)."""
    return np.where(image_srgb <= 0.04045, image_srgb / 12.92, ((image_srgb + 0.055) / 1.055) ** 2.4)


def apply_srgb_gamma(image_linear):
    """Linear RGB (0-1) -> sRGB (EVAL:11-15)."""
    return np.where(image_linear <= 0.0031308, image_linear * 12.92, 1.055 * (image_linear ** (1 / 2.4)) - 0.055)


def rgb_to_hsv_f32(img):
    """OpenCV float RGB -> HSV (H in [0, 360), S and V in [0, 1])."""
    img = img.astype(np.float32)
    r, g, b = img[..., 0], img[..., 1], img[..., 2]
    v = np.maximum(np.maximum(r, g), b)
    vmin = np.minimum(np.minimum(r, g), b)
    diff = v - vmin
    s = diff / (np.abs(v) + _FLT_EPS)
    k = np.float32(60.0) / (diff + _FLT_EPS)
    h = np.where(v == r, (g - b) * k, np.where(v == g, (b - r) * k + np.float32(120.0),
                                               (r - g) * k + np.float32(240.0)))
    h = np.where(h < 0, h + np.float32(360.0), h)
    return np.stack([h, s, v], axis=-1).astype(np.float32)


def hsv_to_rgb_f32(hsv):
    """OpenCV float HSV -> RGB."""
    h = hsv[..., 0].astype(np.float32) * np.float32(6.0 / 360.0)
    s = hsv[..., 1].astype(np.float32)
    v = hsv[..., 2].astype(np.float32)
    h = np.mod(h, np.float32(6.0))
    sector = np.floor(h).astype(np.int64)
    f = (h - sector).astype(np.float32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    f = np.where(bad, np.float32(0), f)
    tab = np.stack([v, v * (np.float32(1) - s), v * (np.float32(1) - s * f),
                    v * (np.float32(1) - s * (np.float32(1) - f))], axis=-1)
    # OpenCV sector table (b, g, r) indices into tab
    sector_data = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    idx = sector_data[sector]
    take = lambda j: np.take_along_axis(tab, idx[..., j:j + 1], axis=-1)[..., 0]
    bb, gg, rr = take(0), take(1), take(2)
    grey = s == 0
    rgb = np.stack([np.where(grey, v, rr), np.where(grey, v, gg), np.where(grey, v, bb)], axis=-1)
    return rgb.astype(np.float32)


def normalize_brightness_without_changing_color(img_srgb_float):
    """Scale the HSV value channel so its maximum is 1 (EVAL:18-43)."""
    hsv = rgb_to_hsv_f32(img_srgb_float)
    max_v = np.max(hsv[..., 2])
    if max_v > 0:
        hsv[..., 2] = hsv[..., 2] / max_v
    return hsv_to_rgb_f32(hsv)


def _lab_f(t):
    eps3 = (24 / 116) ** 3
    return np.where(t > eps3, np.cbrt(t), (841 / 108) * t + 16 / 116)


def xyz_to_lab(xyz, white_xy=D65_XY):
    """CIE 1976 L*a*b* (colour.XYZ_to_Lab with the CIE 1931 2-degree D65 white)."""
    x, y = white_xy
    Xn, Yn, Zn = x / y, 1.0, (1 - x - y) / y
    fx, fy, fz = _lab_f(xyz[..., 0] / Xn), _lab_f(xyz[..., 1] / Yn), _lab_f(xyz[..., 2] / Zn)
    return np.stack([116 * fy - 16, 500 * (fx - fy), 200 * (fy - fz)], axis=-1)


def delta_e_ciede2000(lab1, lab2):
    """CIEDE2000 colour difference (Sharma, Wu & Dalal 2005), k_L = k_C = k_H = 1."""
    lab1 = np.asarray(lab1, dtype=np.float64)
    lab2 = np.broadcast_to(np.asarray(lab2, dtype=np.float64), lab1.shape)
    L1, a1, b1 = lab1[..., 0], lab1[..., 1], lab1[..., 2]
    L2, a2, b2 = lab2[..., 0], lab2[..., 1], lab2[..., 2]
    C1, C2 = np.hypot(a1, b1), np.hypot(a2, b2)
    Cb7 = ((C1 + C2) / 2) ** 7
    G = 0.5 * (1 - np.sqrt(Cb7 / (Cb7 + 25.0 ** 7)))
    a1p, a2p = (1 + G) * a1, (1 + G) * a2
    C1p, C2p = np.hypot(a1p, b1), np.hypot(a2p, b2)
    h1p = np.where((a1p == 0) & (b1 == 0), 0.0, np.degrees(np.arctan2(b1, a1p)) % 360)
    h2p = np.where((a2p == 0) & (b2 == 0), 0.0, np.degrees(np.arctan2(b2, a2p)) % 360)
    dLp = L2 - L1
    dCp = C2p - C1p
    dh = h2p - h1p
    prod = C1p * C2p
    dhp = np.where(prod == 0, 0.0, np.where(dh > 180, dh - 360, np.where(dh < -180, dh + 360, dh)))
    dHp = 2 * np.sqrt(prod) * np.sin(np.radians(dhp / 2))
    Lbp = (L1 + L2) / 2
    Cbp = (C1p + C2p) / 2
    hsum = h1p + h2p
    hbp = np.where(prod == 0, hsum,
                   np.where(np.abs(h1p - h2p) <= 180, hsum / 2,
                            np.where(hsum < 360, (hsum + 360) / 2, (hsum - 360) / 2)))
    T = (1 - 0.17 * np.cos(np.radians(hbp - 30)) + 0.24 * np.cos(np.radians(2 * hbp))
         + 0.32 * np.cos(np.radians(3 * hbp + 6)) - 0.20 * np.cos(np.radians(4 * hbp - 63)))
    dtheta = 30 * np.exp(-(((hbp - 275) / 25) ** 2))
    Cbp7 = Cbp ** 7
    RC = 2 * np.sqrt(Cbp7 / (Cbp7 + 25.0 ** 7))
    SL = 1 + 0.015 * (Lbp - 50) ** 2 / np.sqrt(20 + (Lbp - 50) ** 2)
    SC = 1 + 0.045 * Cbp
    SH = 1 + 0.015 * Cbp * T
    RT = -np.sin(np.radians(2 * dtheta)) * RC
    return np.sqrt((dLp / SL) ** 2 + (dCp / SC) ** 2 + (dHp / SH) ** 2 + RT * (dCp / SC) * (dHp / SH))


def pupil_mask(size: int = 30) -> np.ndarray:
    """Circular eye-pupil mask (EVAL:66-73)."""
    radius = size / 2
    y, x = np.ogrid[:size, :size]
    c = radius - 0.5
    return (np.sqrt((x - c) ** 2 + (y - c) ** 2) <= radius).astype(np.float32)


def eye_perceive(matrix_EB, mask=None, step_y: int = 8, step_x: int = 12):
    """Pupil-integrated eyebox efficiency at the sampled eye positions (EVAL:89-109).

    Accepts a numpy array or a torch tensor (computed on its device) of shape
    [L, NY, NX, 80, 120]; returns an array of shape [L, NY, NX, n_epy, n_epx]."""
    mask = pupil_mask() if mask is None else mask
    ms = mask.shape[0]
    nl, ny, nx, neby, nebx = matrix_EB.shape
    y0s = np.arange(0, neby - ms + 1, step_y)
    x0s = np.arange(0, nebx - ms + 1, step_x)
    try:
        import torch
        is_torch = isinstance(matrix_EB, torch.Tensor)
    except ImportError:  # pragma: no cover
        is_torch = False
    if is_torch:
        m = torch.as_tensor(mask, dtype=matrix_EB.dtype, device=matrix_EB.device)
        out = torch.empty((nl, ny, nx, len(y0s), len(x0s)), dtype=matrix_EB.dtype, device=matrix_EB.device)
        for iy, y0 in enumerate(y0s):
            for ix, x0 in enumerate(x0s):
                out[..., iy, ix] = (matrix_EB[..., y0:y0 + ms, x0:x0 + ms] * m).sum(dim=(-1, -2))
        return out.cpu().numpy()
    out = np.zeros((nl, ny, nx, len(y0s), len(x0s)), dtype=matrix_EB.dtype)
    mb = mask[None, None, None]
    for iy, y0 in enumerate(y0s):
        for ix, x0 in enumerate(x0s):
            out[..., iy, ix] = np.sum(matrix_EB[..., y0:y0 + ms, x0:x0 + ms] * mb, axis=(-1, -2))
    return out


def evaluation(matrix_EB):
    """Drop-in for the reference's ``evaluation`` (EVAL:45-163)."""
    M_inv = np.linalg.inv(M_SENSOR)
    LAB_D65 = xyz_to_lab(XYZ_D65_ASTM / XYZ_D65_ASTM[1] * 100.0)
    perceive = eye_perceive(matrix_EB)
    n_lambda, n_FOVy, n_FOVx, n_epy, n_epx = perceive.shape
    white = linearize_srgb(np.zeros((n_FOVy, n_FOVx, 3)) + 1.0)
    wl = (M_inv @ white.reshape(-1, 3).T).T.reshape(n_FOVy, n_FOVx, 3)[..., None, None]
    adjusted = wl * np.flip(np.transpose(perceive, (1, 2, 0, 3, 4)), axis=2)
    output_image = np.empty_like(adjusted)
    delta_e = 0.0
    U_fov = 0.0
    U_EB = np.zeros((n_epy, n_epx))
    for i in range(n_epy):
        for j in range(n_epx):
            px = adjusted[:, :, :, i, j].reshape(-1, 3)
            rgb = np.clip((M_SENSOR @ px.T).T.reshape(n_FOVy, n_FOVx, 3), 0, 1)
            output_image[:, :, :, i, j] = normalize_brightness_without_changing_color(apply_srgb_gamma(rgb))
            xyz = (M_XYZ @ px.T).T.reshape(n_FOVy, n_FOVx, 3)
            Y = xyz[:, :, 1]
            xyz_norm = xyz / np.maximum(Y, 1e-10)[..., None] * 100
            lab = xyz_to_lab(xyz_norm)
            lab[Y == 0] = 0
            delta_e += np.mean(delta_e_ciede2000(lab, LAB_D65))
            if np.any(Y == 0):
                U_EB[i, j] = 0
            else:
                U_fov += np.min(Y) / np.max(Y)
                U_EB[i, j] = np.mean(Y)
    delta_e = delta_e / n_epx / n_epy
    U_fov = U_fov / n_epx / n_epy
    U_EB = 0 if np.max(U_EB) == 0 else np.min(U_EB) / np.max(U_EB)
    return delta_e, U_fov, U_EB, output_image
