"""RCWA diffraction look-up tables: loader for the real files and a seeded synthetic generator.

The reference loads seven complex ``.npy`` tables fetched from Google Drive
(``gpu_ray_tracing_pro_fullColor.py:28-34``, ``download_lut.py:5-19``).  They
are not available offline, so every benchmark and test uses a *seeded
synthetic* table on the configuration's FoV grid; the generator and its seed
are part of the benchmark definition.

Channel layout (inferred from the kernel's indexing):

* 5-order tables (``ic*``, ``oc*``; order slot ``o`` = 0..4 for -2..+2), 42 channels:
  0 theta, 1 phi, 2+o R te->te, 7+o R te->tm, 12+o T te->te, 17+o T te->tm,
  22+o R tm->te, 27+o R tm->tm, 32+o T tm->te, 37+o T tm->tm.
* 3-order tables (``fc*``; o = 0..2 for -1..+1), 26 channels:
  0 theta, 1 phi, 2+o R te->te, 5+o R te->tm, 8+o T te->te, 11+o T te->tm,
  14+o R tm->te, 17+o R tm->tm, 20+o T tm->te, 23+o T tm->tm.

Shapes: ``lut_ic{1,2,3}`` ``[L, NX, NY, 42]``; ``lut_fc{1,2}`` ``[nFC, L, NX, NY, 26]``;
``lut_oc{1,2}`` ``[nOC, L, NX, NY, 42]`` (complex128).

The synthetic generator puts the physical propagation angles of the design
(``couplers_coor`` outputs) in channel 0 so the cos-ratios the kernel forms
are physical, and fills every Jones matrix the kernel reads with a scaled
unitary matrix whose scale is chosen so that the branch efficiency the kernel
computes equals a per-interaction target (jittered per FoV / wavelength /
slice).  The ``deep`` profile raises the 0th-order reflection and lowers the
out-coupling (BASELINE config 5, deep-bounce stress).
"""
from __future__ import annotations

import os
import warnings

import numpy as np

LUT_NAMES = ("lut_ic1", "lut_ic2", "lut_ic3", "lut_fc1", "lut_fc2", "lut_oc1", "lut_oc2")
N_CH5 = 42
N_CH3 = 26

# (R/T, order-slot) -> (te->te, te->tm, tm->te, tm->tm) channel numbers
def _chan5(kind: str, o: int):
    base = {"R": (2, 7, 22, 27), "T": (12, 17, 32, 37)}[kind]
    return tuple(b + o for b in base)


def _chan3(kind: str, o: int):
    base = {"R": (2, 5, 14, 17), "T": (8, 11, 20, 23)}[kind]
    return tuple(b + o for b in base)


# Target branch efficiencies per interaction.  The fold
# efficiency of the folding-coupler slices and the out-coupling efficiency of the
# out-coupler slices are graded linearly along the slices (slice 0 is the one a ray
# meets first), as a uniformity-optimised design would be; "keep" is the total
# reflected fraction (stay + turn [+ out]), the rest is lost.
PROFILES = {
    "default": dict(ic=(0.40, 0.05), r0=(0.85, 0.05), r1=(0.05, 0.85),
                    fc_fold=(0.08, 0.30), fc_keep=0.97, fc_back=0.04, fc2_keep=0.93,
                    oc_turn=0.03, oc_out=(0.06, 0.25), oc_keep=0.96),
    "deep": dict(ic=(0.40, 0.05), r0=(0.90, 0.03), r1=(0.03, 0.90),
                 fc_fold=(0.03, 0.10), fc_keep=0.985, fc_back=0.03, fc2_keep=0.955,
                 oc_turn=0.02, oc_out=(0.02, 0.06), oc_keep=0.985),
    # BASELINE config 5's deep-bounce stress LUT (configs.CONFIGS["C5"], with hops scaled by 0.05):
    # a better in-coupler (20 % of rays lost there instead of 55 %), 0th-order reflection kept at
    # 99.5-99.8 %, out-coupling 2-6 % per OC interaction (the default's 6-25 %)
    "stress": dict(ic=(0.70, 0.10), r0=(0.95, 0.03), r1=(0.03, 0.95),
                   fc_fold=(0.02, 0.05), fc_keep=0.998, fc_back=0.05, fc2_keep=0.995,
                   oc_turn=0.03, oc_out=(0.02, 0.06), oc_keep=0.998),
    # Lossless, evenly split interactions: with shortened hops (tests scale lut_gap) rays
    # live for 100+ bounces and ener = prod(e) falls below the single-wavelength kernel's
    # 1e-15 guard (GRTF:444), which the other profiles practically never reach.
    "balanced": dict(ic=(0.45, 0.45), r0=(0.5, 0.5), r1=(0.5, 0.5),
                     fc_fold=(0.5, 0.5), fc_keep=1.0, fc_back=0.5, fc2_keep=1.0,
                     oc_turn=0.33, oc_out=(0.33, 0.33), oc_keep=1.0),
    # Adversarial profiles for the Jones lane's certified decisions, where its
    # bound is weakest:
    # * near-singular Jones matrices (condition number ~1e6: a rank-one matrix plus 1e-6 of a
    #   unitary one), so a branch's efficiency depends steeply on the ray's polarisation and the
    #   carried Jones vector is far from the matrices' well-conditioned directions; targets are the
    #   default profile's, reached for the most-transmitted polarisation;
    "adversarial_singular": dict(ic=(0.40, 0.05), r0=(0.85, 0.05), r1=(0.05, 0.85),
                                 fc_fold=(0.08, 0.30), fc_keep=0.97, fc_back=0.04, fc2_keep=0.93,
                                 oc_turn=0.03, oc_out=(0.06, 0.25), oc_keep=0.96, jones="singular", cond=1e6),
    # * rank-one Jones matrices plus 1e-9 of a unitary one (condition ~1e9): the taken branch contracts the
    #   state's polarisation onto one direction, and the least-transmitted one is ~1e-18 of the most;
    "adversarial_rank1": dict(ic=(0.40, 0.05), r0=(0.85, 0.05), r1=(0.05, 0.85),
                              fc_fold=(0.08, 0.30), fc_keep=0.97, fc_back=0.04, fc2_keep=0.93,
                              oc_turn=0.03, oc_out=(0.06, 0.25), oc_keep=0.96, jones="singular", cond=1e9),
    # * moderately polarisation-selective matrices (rank one plus 1/10 of a unitary one, condition ~10):
    #   unlike the two above, a ray's state often lies nearer a taken matrix's weak direction than its
    #   strong one, so the amplification factor a = |det M| |E|^2 / |M E|^2 exceeds 1 on a sizeable share
    #   of interactions and the amplification-tracked bound grows along a ray;
    "adversarial_polarizing": dict(ic=(0.40, 0.05), r0=(0.85, 0.05), r1=(0.05, 0.85),
                                   fc_fold=(0.08, 0.30), fc_keep=0.97, fc_back=0.04, fc2_keep=0.93,
                                   oc_turn=0.03, oc_out=(0.06, 0.25), oc_keep=0.96, jones="singular", cond=10.0),
    # * lossless interactions whose branch efficiencies sum to 1 - 1e-9 and split (nearly) evenly, no
    #   jitter: every interaction's last threshold sits 1e-9 below 1 (draws near 1 decide against it)
    #   and the branch thresholds sit near the common draw 0.5; with shortened hops (tests scale
    #   lut_gap) rays live for hundreds to thousands of bounces, so the reference's unwrapped phase
    #   (delta_phase += 2 lut_TIR per miss hop, GRTF:1052, 1108, 1178) grows long.
    "adversarial_lossless": dict(ic=(0.5, 0.5 - 1e-9), r0=(0.5, 0.5 - 1e-9), r1=(0.5 - 1e-9, 0.5),
                                 fc_fold=(0.5, 0.5), fc_keep=1.0 - 1e-9, fc_back=0.5, fc2_keep=1.0 - 1e-9,
                                 oc_turn=1.0 / 3.0, oc_out=(1.0 / 3.0, 1.0 / 3.0), oc_keep=1.0 - 1e-9, jitter=0.0),
}


def _graded(lo_hi, n):
    lo, hi = lo_hi
    return np.linspace(lo, hi, n) if n > 1 else np.array([lo])


def _jones(rng, shape, scale):
    """Scaled random unitary 2x2 Jones matrices [[tete, tmte], [tetm, tmtm]]."""
    alpha = rng.uniform(0.0, 0.5, shape)
    pa, pb, psi = (rng.uniform(-np.pi, np.pi, shape) for _ in range(3))
    a = np.cos(alpha) * np.exp(1j * pa)
    b = np.sin(alpha) * np.exp(1j * pb)
    ep = np.exp(1j * psi)
    amp = np.sqrt(scale)
    return amp * a, amp * b, amp * (-ep * np.conj(b)), amp * (ep * np.conj(a))


def _jones_singular(rng, shape, scale, cond):
    """Random near-singular 2x2 Jones matrices: u v^H + (1 / cond) U (u, v random unit complex
    vectors, U random unitary), scaled so the largest singular value squared is ``scale`` -- the
    efficiency of the most-transmitted polarisation -- while the other is ~scale / cond^2."""
    def unit():
        th = rng.uniform(0.0, np.pi / 2, shape)
        p1, p2 = (rng.uniform(-np.pi, np.pi, shape) for _ in range(2))
        return np.cos(th) * np.exp(1j * p1), np.sin(th) * np.exp(1j * p2)
    u0, u1 = unit()
    v0, v1 = unit()
    e = 1.0 / cond
    a, b, c, d = _jones(rng, shape, np.ones(shape))
    m00, m01 = u0 * np.conj(v0) + e * a, u0 * np.conj(v1) + e * b
    m10, m11 = u1 * np.conj(v0) + e * c, u1 * np.conj(v1) + e * d
    # largest singular value of [[m00, m01], [m10, m11]]
    fro = abs(m00) ** 2 + abs(m01) ** 2 + abs(m10) ** 2 + abs(m11) ** 2
    det = abs(m00 * m11 - m01 * m10)
    smax2 = 0.5 * (fro + np.sqrt(np.maximum(fro * fro - 4.0 * det * det, 0.0)))
    amp = np.sqrt(scale / smax2)
    return amp * m00, amp * m01, amp * m10, amp * m11


def synthetic_luts(geom, seed: int = 0, profile: str = "default", jitter: float = 0.25):
    """Seeded synthetic LUT set matching ``geom`` (a :class:`CouplerGeometry`)."""
    tgt = PROFILES[profile]
    jitter = tgt.get("jitter", jitter)
    singular = tgt.get("jones") == "singular"
    rng = np.random.default_rng(seed)
    ang = geom.angles
    th_in, th_ic, th_ic2 = ang["th_in_ic"], ang["th_out_ic"], ang["th_out_ic2"]
    th_fc, th_oc = ang["th_out_fc"], ang["th_out_oc"]
    ph_in, ph_ic, ph_ic2 = ang["phi_in_ic"], ang["phi_out_ic"], ang["phi_out_ic2"]
    ph_fc, ph_oc = ang["phi_out_fc"], ang["phi_out_oc"]
    n_g = geom.n_g
    L, NX, NY = th_in.shape
    nfc, noc = geom.num_fc_slices, geom.num_oc_slices
    cos = np.cos

    def noise(shape, nch):
        return 0.1 * (rng.uniform(0, 1, shape + (nch,)) * np.exp(1j * rng.uniform(-np.pi, np.pi, shape + (nch,))))

    def fill(tab, chans, target, ratio):
        shape = tab.shape[:-1]
        eta = target * (1.0 + jitter * rng.uniform(-1.0, 1.0, shape))
        tete, tmte, tetm, tmtm = (_jones_singular(rng, shape, eta / ratio, tgt["cond"]) if singular else
                                  _jones(rng, shape, eta / ratio))
        p, q, r, s = chans            # EF(p, q, r, s): Ete' = c_p te + c_r tm; Etm' = c_q te + c_s tm
        tab[..., p] = tete
        tab[..., r] = tmte
        tab[..., q] = tetm
        tab[..., s] = tmtm

    base = (L, NX, NY)
    ic1 = noise(base, N_CH5)
    ic2 = noise(base, N_CH5)
    ic3 = noise(base, N_CH5)
    fc1 = noise((nfc,) + base, N_CH3)
    fc2 = noise((nfc,) + base, N_CH3)
    oc1 = noise((noc,) + base, N_CH5)
    oc2 = noise((noc,) + base, N_CH5)
    for tab, th, ph in ((ic1, th_in, ph_in), (ic2, th_ic, ph_ic), (ic3, th_ic2, ph_ic2),
                        (fc1, th_ic, ph_ic), (fc2, th_fc, ph_fc), (oc1, th_fc, ph_fc),
                        (oc2, th_oc, ph_oc)):
        tab[..., 0] = th
        tab[..., 1] = ph

    # in-coupling (GRTF:860-869): T -1 -> ic2 direction, T +1 -> ic3 direction
    fill(ic1, _chan5("T", 1), tgt["ic"][0], cos(th_ic) / cos(th_in) * n_g)
    fill(ic1, _chan5("T", 3), tgt["ic"][1], cos(th_ic2) / cos(th_in) * n_g)
    # R0 (GRTF:909-918): R 0 stays, R +2 -> ic3 direction
    fill(ic2, _chan5("R", 2), tgt["r0"][0], 1.0)
    fill(ic2, _chan5("R", 4), tgt["r0"][1], cos(th_ic2) / cos(th_ic))
    # R1 (GRTF:955-964): the reference's swapped cross-pol call (2, 22, 7, 27), then R 0
    fill(ic3, (2, 22, 7, 27), tgt["r1"][0], cos(th_ic) / cos(th_ic2))
    fill(ic3, _chan5("R", 2), tgt["r1"][1], 1.0)
    # R2 / R3 (GRTF:1007-1016, 1060-1069): per-slice graded fold
    fold = _graded(tgt["fc_fold"], nfc).reshape(-1, 1, 1, 1)
    fill(fc1, _chan3("R", 1), tgt["fc_keep"] - fold, 1.0)
    fill(fc1, _chan3("R", 0), fold, cos(th_fc) / cos(th_ic))
    fill(fc2, _chan3("R", 2), tgt["fc_back"], cos(th_ic) / cos(th_fc))
    fill(fc2, _chan3("R", 1), tgt["fc2_keep"], 1.0)
    # R4 / R5 (GRTF:1117-1131, 1186-1200): per-slice graded out-coupling
    out = _graded(tgt["oc_out"], noc).reshape(-1, 1, 1, 1)
    turn = tgt["oc_turn"]
    stay = tgt["oc_keep"] - turn - out
    fill(oc1, _chan5("R", 2), stay, 1.0)
    fill(oc1, _chan5("R", 0), turn, cos(th_oc) / cos(th_fc))
    fill(oc1, _chan5("T", 1), out, cos(th_in) / cos(th_fc) / n_g)
    fill(oc2, _chan5("R", 4), turn, cos(th_fc) / cos(th_oc))
    fill(oc2, _chan5("R", 2), stay, 1.0)
    fill(oc2, _chan5("T", 3), out, cos(th_in) / cos(th_oc) / n_g)
    return dict(lut_ic1=ic1, lut_ic2=ic2, lut_ic3=ic3, lut_fc1=fc1, lut_fc2=fc2,
                lut_oc1=oc1, lut_oc2=oc2)


class LUTPrecisionWarning(UserWarning):
    """A LUT was given in single precision (complex64 / float32)."""


class EnerUnderflowWarning(LUTPrecisionWarning):
    """Traces were decided in the ener-underflow regime (``wgrt_trace_stats.libm_rays``, ABI 7): a LUT
    whose rays live so long without loss that ``ener = prod(e)`` nears the subnormal range, where the
    full-colour guard ``ener * e > 0`` (GRTF:1020) depends on the libm's last bits."""


def lut_f32_mask(luts: dict) -> int:
    """wgrt_scene_opts.lut_f32_angles of a LUT set as given: bit k for each table k (ic1, ic2, ic3,
    fc1, fc2, oc1, oc2) held in single precision.  The reference loads the .npy files as stored
    (MAIN:28-34); compiled numba then takes math.cos of a complex64 table's float32 ``.real`` in
    float32 (GRTF:866-869, ...), which the scene reproduces for the flagged tables."""
    mask = 0
    for k, name in enumerate(LUT_NAMES):
        a = luts.get(name)
        if a is not None and np.asarray(a).dtype in (np.complex64, np.float32, np.float16):
            mask |= 1 << k
    return mask


def validate_luts(luts: dict, num_lmd: int, nx: int, ny: int, nfc: int, noc: int) -> dict:
    """Shape / dtype checks for a LUT set (real or synthetic); returns complex128 copies.

    Raises ``ValueError`` naming the first table that does not match the
    geometry (the reference indexes them without checks, MAIN:28-34).

    Single-precision tables (complex64, as ``np.save`` of a complex64 array gives) are
    accepted and widened exactly to complex128, with a :class:`LUTPrecisionWarning`: the
    compiled reference kernel takes ``math.cos`` of a complex64 table's float32 ``.real``
    (GRTF:866-869 and every cos ratio after it) in single precision.  Pass
    ``lut_f32_mask`` of the tables AS LOADED to the scene (``Scene(..., lut_f32_angles=mask)``;
    the reference-flow driver does) and the scene takes those cosines as float32 ``cosf``
    too.  Parity for such tables is pinned against the oracle's same semantics; against the
    reference it is unpinned (CUDA's libdevice ``cosf`` and glibc's may differ in the last
    bit, and the real files are not available offline).  The input dtypes are in
    ``validate_luts.last_dtypes``.
    """
    want = {"lut_ic1": (num_lmd, nx, ny), "lut_ic2": (num_lmd, nx, ny), "lut_ic3": (num_lmd, nx, ny),
            "lut_fc1": (nfc, num_lmd, nx, ny), "lut_fc2": (nfc, num_lmd, nx, ny),
            "lut_oc1": (noc, num_lmd, nx, ny), "lut_oc2": (noc, num_lmd, nx, ny)}
    min_ch = {"lut_ic1": 41, "lut_ic2": 32, "lut_ic3": 30, "lut_fc1": 19, "lut_fc2": 20,
              "lut_oc1": 39, "lut_oc2": 41}
    out, dtypes, single = {}, {}, []
    for name in LUT_NAMES:
        if name not in luts:
            raise ValueError(f"missing LUT {name}")
        a = np.asarray(luts[name])
        if a.shape[:-1] != want[name]:
            raise ValueError(f"{name}: shape {a.shape} does not match grid {want[name]} + (channels,)")
        if a.shape[-1] < min_ch[name]:
            raise ValueError(f"{name}: {a.shape[-1]} channels, kernel reads channel {min_ch[name] - 1}")
        if not (np.iscomplexobj(a) or np.issubdtype(a.dtype, np.floating)):
            raise ValueError(f"{name}: dtype {a.dtype} is not complex/real floating")
        dtypes[name] = a.dtype
        if a.dtype in (np.complex64, np.float32, np.float16):
            single.append(name)
        out[name] = np.ascontiguousarray(a, dtype=np.complex128)
    validate_luts.last_dtypes = dtypes
    if single:
        warnings.warn(f"single-precision LUTs {single} widened to complex128: give the scene their lut_f32_mask so "
                      "their angles' cosines are taken in float32 as compiled numba does (see validate_luts)",
                      LUTPrecisionWarning, stacklevel=2)
    return out


validate_luts.last_dtypes = {}


def load_luts(directory: str = ".", suffix: str = "_fullColor.npy") -> dict:
    """Load the seven reference LUT files (MAIN:28-34) with ``allow_pickle=False``, dtypes as stored
    (``validate_luts`` checks and widens them)."""
    luts = {}
    for name in LUT_NAMES:
        path = os.path.join(directory, name + suffix)
        luts[name] = np.load(path, allow_pickle=False)
    return luts


def save_luts(luts: dict, directory: str, suffix: str = "_fullColor.npy", dtype=None) -> None:
    """Write a LUT set as the reference's seven ``.npy`` files (``load_luts``'s inverse)."""
    os.makedirs(directory, exist_ok=True)
    for name in LUT_NAMES:
        a = np.asarray(luts[name])
        np.save(os.path.join(directory, name + suffix), a if dtype is None else a.astype(dtype))


def single_wavelength(luts: dict, lut_TIR: np.ndarray, lut_gap: np.ndarray, l: int):
    """Wavelength ``l`` of a full-colour set, in the single-wavelength kernel's shapes
    (process_rays_kernel_pro, GRTF:419-427): lut_ic* / lut_TIR / lut_gap [NX, NY, C],
    lut_fc* / lut_oc* [n_slices, NX, NY, C].  Returns ``(luts, lut_TIR, lut_gap)``."""
    out = {}
    for k in ("lut_ic1", "lut_ic2", "lut_ic3"):
        out[k] = np.ascontiguousarray(luts[k][l])
    for k in ("lut_fc1", "lut_fc2", "lut_oc1", "lut_oc2"):
        out[k] = np.ascontiguousarray(luts[k][:, l])
    return out, np.ascontiguousarray(lut_TIR[l]), np.ascontiguousarray(lut_gap[l])
