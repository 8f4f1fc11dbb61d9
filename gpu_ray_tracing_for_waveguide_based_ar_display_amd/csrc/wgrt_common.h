// wgrt_common.h -- arithmetic shared by the device kernels and the host-side scene builder.
//
// Every function here is written with IEEE basic operations (+ - * / sqrt fma),
// so a host and a device evaluation are bit-identical when compiled with
// -ffp-contract=off (the build does).  Each one restates a device function of
// the reference kernel module GPU_ray_tracing_functions.py (GRTF).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WGRT_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define WGRT_HD inline
#endif

namespace wgrt {

#if !defined(__HIPCC__)
using std::fabs;
using std::floor;
using std::fma;
using std::frexp;
using std::isinf;
using std::isnan;
using std::ldexp;
using std::sqrt;
#endif

constexpr double kPi = 3.141592653589793;
constexpr int kEbNy = 80;     // eyebox grid rows    (MAIN:37)
constexpr int kEbNx = 120;    // eyebox grid columns (MAIN:37)
constexpr double kOnEdgeTol = 1e-12;   // GRTF:68
constexpr int64_t kMaxLoop = 100000;   // range(1e5), GRTF:905

// ---------------------------------------------------------------------------
// Packed per-(lambda, m, n) tile, in doubles.  Interaction "blocks" hold, for one
// FSM state (and one coupler slice), the numerator cosines of the branch
// efficiencies and the four complex Jones coefficients of every E_field_cal call in
// the reference's argument order (p, q, r, s) -- see GRTF:860-1200.
// ---------------------------------------------------------------------------
constexpr int kTileTir = 0;       // lut_TIR[4]
constexpr int kTileGap = 4;       // lut_gap[8]
constexpr int kTileEbRange = 12;  // eff_reg_FOV_range[m, n, 4]
constexpr int kTileEbRect = 16;   // eff_reg_FOV[m, n, 4, 2]
constexpr int kTileCosIc1 = 24;   // cos(lut_ic1[l, m, n, 0].real)
constexpr int kTileTirRot = 28;   // (cos, sin) of lut_TIR[k], k = 0..3: the phase step of a taken branch
constexpr int kTileHopRot = 36;   // (cos, sin) of 2 * lut_TIR[k], k = 0, 1: the phase step of a miss hop
constexpr int kTileHeader = 40;
constexpr int kBlock = 28;        // cosA[3], pad, rec[3][8]
constexpr int kBlockCos = 0;
constexpr int kBlockRec = 4;

// ---------------------------------------------------------------------------
// Jones-vector tile (variants 7-9): the same interaction blocks, laid out in 128-B lines,
// with the TIR phase step of each taken branch folded into its TM output row (rec q and s
// multiplied by e^{i lut_TIR[k]}; the branch efficiency |M E|^2 is unchanged by it) and the
// certification weights of the branch decisions.
// ---------------------------------------------------------------------------
constexpr int kJGap = 0;          // lut_gap[8]
constexpr int kJHop = 8;          // (cos, sin) of 2 lut_TIR[0] (R2 miss hop), of 2 lut_TIR[1] (R3 / R4)
constexpr int kJCosIc1 = 12;      // cos(lut_ic1[l, m, n, 0].real)
constexpr int kJGrowth = 13;      // max(1, max_k |lut_TIR[k]| / pi): bounds the reference's unwrapped phase growth
constexpr int kJHeader = 16;
// Block line 0 (the estimate's input, read by every interaction): cosA_0, cosA_1 (double), then
// four floats {Wsum, cosA_2, 0, 0}, then per branch the Hermitian form H = M^H M of its matrix
// M = [[p, r], [q, s]] as four floats {h11, h22, Re h12, Im h12}: |M E|^2 = h11 |Ete|^2 +
// h22 |Etm|^2 + 2 Re(h12 conj(Ete) Etm) -- half the bytes and a quarter of the products of
// evaluating M E.  Lines 1-2: the matrices in double precision (the taken branch's field, the
// rare double-precision re-evaluation), the bounds W[k] and cosA_2 in double.
constexpr int kJBlock = 48;       // line 0: cosA[2], f32 {Wsum, cosA_2}, herm32[3][4]; rec[3][8], W[3], cosA_2
constexpr int kJBlockCos = 0;     // cosA_0, cosA_1
constexpr int kJBlockF32 = 2;     // floats: Wsum (sum of W[k], rounded up), cosA_2, the tile's kJGrowth (rounded up), 0;
                                  // block 0 (two branches, the in-coupling event): Wsum, kJGrowth (rounded up), and
                                  // the bits of the double kJCosIc1 in the last two
constexpr int kJBlockHerm = 4;    // floats [3][4]: h11, h22, Re h12, Im h12
constexpr int kJBlockRec = 16;    // the three matrices in double precision
constexpr int kJBlockCos2 = 43;   // cosA_2 in double
// W[k] = ((|p|+|r|)^2 + (|q|+|s|)^2) * |cosA_k| * f_k (f_k the n_g factor of the branch): for a
// field state E, |M_k E|^2 * cosA_k * f_k is computed to within D * W[k] * |E|^2 by any two
// evaluations whose states and matrices agree to within D / 4 (relative) -- the bound the
// Jones-vector variants certify their Monte-Carlo decisions against (D = cert_tol for the
// double-precision evaluation, cert_tol32 for the single-precision estimate).
constexpr int kJBlockW = 40;
WGRT_HD int jtile_doubles(int nfc, int noc) { return kJHeader + kJBlock * (3 + 2 * nfc + 2 * noc); }

// block index: 0 in-coupling, 1 R0, 2 R1, 3 + k R2 slice k, 3 + nfc + k R3,
//              3 + 2 nfc + k R4, 3 + 2 nfc + noc + k R5
WGRT_HD int tile_doubles(int nfc, int noc) { return kTileHeader + kBlock * (3 + 2 * nfc + 2 * noc); }

// ---------------------------------------------------------------------------
// Correctly rounded hypot.  CPython 3.10's math.hypot (what the reference calls,
// GRTF:145-146) is correctly rounded; so is this: exact double-double square sum
// (FMA error terms) followed by one Newton correction of the square root.
// ---------------------------------------------------------------------------
WGRT_HD double hypot_cr(double x, double y) {
    double ax = fabs(x), ay = fabs(y);
    if (isinf(ax) || isinf(ay)) return INFINITY;
    if (isnan(ax) || isnan(ay)) return NAN;
    if (ax < ay) { double t = ax; ax = ay; ay = t; }
    if (ay == 0.0) return ax;
    if (ax <= 0x1p400 && ay >= 0x1p-400) {
        // No scaling needed: every intermediate below stays normal, so the result is
        // bit-identical to the power-of-two-scaled evaluation (rounding is scale-invariant).
        const double h = ax * ax, hl = fma(ax, ax, -h);
        const double k = ay * ay, kl = fma(ay, ay, -k);
        const double s = h + k;
        const double lo = ((h - s) + k) + (hl + kl);
        double r = sqrt(s);
        const double rr = fma(-r, r, s);
        return r + (rr + lo) / (2.0 * r);
    }
    int e;
    (void)frexp(ax, &e);
    const double sx = ldexp(ax, -e), sy = ldexp(ay, -e);
    const double h = sx * sx, hl = fma(sx, sx, -h);
    const double k = sy * sy, kl = fma(sy, sy, -k);
    const double s = h + k;
    const double lo = ((h - s) + k) + (hl + kl);
    double r = sqrt(s);
    const double rr = fma(-r, r, s);
    r = r + (rr + lo) / (2.0 * r);
    return ldexp(r, e);
}

// GRTF:124-130
WGRT_HD double wrap_pi(double x) {
    const double two_pi = 2.0 * kPi;
    x = x + kPi;
    x = x - two_pi * floor(x / two_pi);
    return x - kPi;
}

// GRTF:52-61 + GRTF:36-50 fused into one edge pass.  The reference makes an
// on-edge pass and then a crossing pass; both are order-independent (an "any" and
// a parity), so one pass over the edges gives the identical result.
WGRT_HD bool on_segment(double px, double py, double x1, double y1, double x2, double y2) {
    const double lo_x = (x2 < x1 ? x2 : x1), hi_x = (x2 > x1 ? x2 : x1);
    const double lo_y = (y2 < y1 ? y2 : y1), hi_y = (y2 > y1 ? y2 : y1);
    if (px < lo_x - kOnEdgeTol || px > hi_x + kOnEdgeTol || py < lo_y - kOnEdgeTol ||
        py > hi_y + kOnEdgeTol)
        return false;
    return fabs((x2 - x1) * (py - y1) - (y2 - y1) * (px - x1)) <= kOnEdgeTol;
}

// is_inside_or_on_edge(px, py, poly, 0, nv) (GRTF:63-71); xy = [nv][2]
WGRT_HD bool inside_or_on_edge(double px, double py, const double *xy, int nv) {
    bool inside = false;
    int j = nv - 1;
    for (int i = 0; i < nv; ++i) {
        const double xi = xy[2 * i], yi = xy[2 * i + 1];
        const double xj = xy[2 * j], yj = xy[2 * j + 1];
        if (on_segment(px, py, xj, yj, xi, yi)) return true;
        if (((yi > py) != (yj > py)) && (px < (xj - xi) * (py - yi) / (yj - yi + 1e-20) + xi))
            inside = !inside;
        j = i;
    }
    return inside;
}

// The same predicate over a subset of the polygon's edges (edge = end-vertex index i,
// start vertex i - 1 mod nv).  Equal to inside_or_on_edge whenever the omitted edges can
// neither pass on_segment's bounding-box check nor straddle py (see the row-band lists in
// wgrt_scene_build.cpp).
WGRT_HD bool inside_or_on_edge_subset(double px, double py, const double *xy, int nv,
                                      const int32_t *edges, int ne) {
    bool inside = false;
    for (int e = 0; e < ne; ++e) {
        const int i = edges[e];
        const int j = (i == 0) ? nv - 1 : i - 1;
        const double xi = xy[2 * i], yi = xy[2 * i + 1];
        const double xj = xy[2 * j], yj = xy[2 * j + 1];
        if (on_segment(px, py, xj, yj, xi, yi)) return true;
        if (((yi > py) != (yj > py)) && (px < (xj - xi) * (py - yi) / (yj - yi + 1e-20) + xi))
            inside = !inside;
    }
    return inside;
}

// xorshift32 (13, 17, 5) of GRTF:25-34.  gid() returns the GLOBAL ray index; it is evaluated
// only for the zero-state fix-up (GRTF:28-29), so a kernel may look it up lazily.
template <class GidFn>
WGRT_HD double rng_draw_lazy(uint32_t &s, GidFn gid) {
    uint32_t v = s;
    if (__builtin_expect(v == 0u, 0)) v = 0x6D2B79F5u ^ (uint32_t)(gid() + 1);
    v ^= v << 13;
    v ^= v >> 17;
    v ^= v << 5;
    s = v;
    return (double)v * (1.0 / 4294967296.0);
}

WGRT_HD double rng_draw(uint32_t &s, int64_t gid) {
    return rng_draw_lazy(s, [gid]() { return gid; });
}

}  // namespace wgrt
