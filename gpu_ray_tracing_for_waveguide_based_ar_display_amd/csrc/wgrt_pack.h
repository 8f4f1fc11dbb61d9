// wgrt_pack.h -- scene-building steps compiled for the host AND the device, so the scene the
// kernels read is the same whichever side builds it (wgrt_scene_create builds it on the device;
// the host build remains for wgrt_locator_classify_host and as the device build's check):
//
//  * edge_row_span: which cells of one grid row an edge of a polygon reaches (the EDGE class of
//    the exact locator, wgrt_scene_build.cpp's header);
//  * pack_tile: one (lambda, m, n) tile of the exact-arithmetic lane and its Jones-vector tile
//    from the raw scene arrays and the host-evaluated trig table (every cos / sin the reference
//    takes with Python's math module, GRTF:868-1200 and couplers_coor's lut_TIR, is evaluated
//    on the host libm -- the same function -- and only copied here).
//
// The arithmetic here is IEEE + - * / (no contraction: -ffp-contract=off) plus hypot in the
// certification bound W, which is a bound, not a reference value (the device's hypot may round
// differently from the host's in the last place; the bound's 1.01 factors cover it).
#pragma once

#include "wgrt_common.h"

namespace wgrt {

#if !defined(__HIPCC__)
using std::hypot;
#endif

constexpr double kPad = 1e-6;          // mm; >> tol (1e-12) and >> float64 rounding at |x| ~ 60 mm
constexpr double kShortEdge = 1e-4;    // mm; shorter edges use the bbox criterion

// Cells [cx0, cx1] of row cy that edge (ax, ay)-(bx, by) reaches within 2 kPad (the part of the
// edge inside the row's y-range, padded, widened by 2 kPad); false if it misses the row.
WGRT_HD bool edge_row_span(double ax, double ay, double bx, double by, int cy, double x0, double y0, double h,
                           int ncx, int &cx0, int &cx1) {
    const double pad2 = 2 * kPad;
    const double dxe = bx - ax, dye = by - ay;
    const double len = sqrt(dxe * dxe + dye * dye);
    const double ey0 = (ay < by ? ay : by) - pad2, ey1 = (ay < by ? by : ay) + pad2;
    const double ry0 = y0 + cy * h - pad2, ry1 = y0 + (cy + 1) * h + pad2;
    double lo, hi;
    if (len < kShortEdge || fabs(by - ay) < 1e-300) {
        if (ey1 < ry0 || ey0 > ry1) return false;
        lo = ax < bx ? ax : bx;
        hi = ax < bx ? bx : ax;
    } else {
        // parameter range of the segment inside [ry0, ry1]
        double t0 = (ry0 - ay) / (by - ay), t1 = (ry1 - ay) / (by - ay);
        if (t0 > t1) {
            const double t = t0;
            t0 = t1;
            t1 = t;
        }
        t0 = t0 > 0.0 ? t0 : 0.0;
        t1 = t1 < 1.0 ? t1 : 1.0;
        if (t0 > t1 + 1e-12) return false;
        const double xa = ax + t0 * (bx - ax), xb = ax + t1 * (bx - ax);
        lo = xa < xb ? xa : xb;
        hi = xa < xb ? xb : xa;
    }
    lo -= pad2 + 1e-9;
    hi += pad2 + 1e-9;
    const int a = (int)floor((lo - x0) / h), b = (int)floor((hi - x0) / h);
    cx0 = a > 0 ? a : 0;
    cx1 = b < ncx - 1 ? b : ncx - 1;
    return cx0 <= cx1;
}

// Rows [cy0, cy1] an edge can reach (edge_row_span decides each).
WGRT_HD void edge_rows(double ay, double by, double y0, double h, int ncy, int &cy0, int &cy1) {
    const double pad2 = 2 * kPad;
    const double ey0 = (ay < by ? ay : by) - pad2, ey1 = (ay < by ? by : ay) + pad2;
    const int a = (int)floor((ey0 - y0) / h) - 1, b = (int)floor((ey1 - y0) / h) + 1;
    cy0 = a > 0 ? a : 0;
    cy1 = b < ncy - 1 ? b : ncy - 1;
}

// The raw scene arrays one tile is packed from (wgrt_scene_desc's, or their device copies).
struct PackView {
    const double *ic1, *ic2, *ic3, *fc1, *fc2, *oc1, *oc2;   // complex interleaved
    const double *tir, *gap;                                 // lut_TIR [g][4], lut_gap [g][8]
    const double *fov, *fovr;                                // eff_reg_FOV [m][n][4][2], _range [m][n][4]
    const double *trig;                                      // per tile, trig_doubles() (build_trig)
    int64_t L, NX, NY;
    int ch5, ch3, nfc, noc;
    double n_g;
};

// Per-tile trig table: cos of the LUT polar angles (channel 0 of ic1, ic2, ic3, fc1[k], fc2[k],
// oc1[k], oc2[k]), then (cos, sin) of lut_TIR[k] (k = 0..3) and of 2 lut_TIR[k] (k = 0, 1).
WGRT_HD int trig_doubles(int nfc, int noc) { return 3 + 2 * nfc + 2 * noc + 12; }

WGRT_HD const double *lut_at(const double *p, int64_t s, int64_t l, int64_t m, int64_t n, int64_t c,
                             const PackView &v, int ch) {
    return p + 2 * ((((s * v.L + l) * v.NX + m) * v.NY + n) * ch + c);
}

WGRT_HD void put_rec(double *dst, const double *lut, int ch, const PackView &v, int64_t s, int64_t l, int64_t m,
                     int64_t n, int p, int q, int r, int t) {
    const int c4[4] = {p, q, r, t};
    for (int k = 0; k < 4; ++k) {
        const double *c = lut_at(lut, s, l, m, n, c4[k], v, ch);
        dst[2 * k] = c[0];
        dst[2 * k + 1] = c[1];
    }
}

// Tile g = (l * NX + m) * NY + n: T (tile_doubles, zeroed by the caller) and J (jtile_doubles, zeroed).
WGRT_HD void pack_tile(const PackView &v, int64_t g, double *T, double *J) {
    const int nfc = v.nfc, noc = v.noc;
    const int64_t n = g % v.NY, m = g / v.NY % v.NX, l = g / (v.NY * v.NX);
    const double *tg = v.trig + g * trig_doubles(nfc, noc);
    const double *cf1 = tg + 3, *cf2 = cf1 + nfc, *co1 = cf2 + nfc, *co2 = co1 + noc, *rot = co2 + noc;
    for (int k = 0; k < 4; ++k) {
        T[kTileTir + k] = v.tir[4 * g + k];
        T[kTileTirRot + 2 * k] = rot[2 * k];
        T[kTileTirRot + 2 * k + 1] = rot[2 * k + 1];
    }
    for (int k = 0; k < 4; ++k) T[kTileHopRot + k] = rot[8 + k];
    for (int k = 0; k < 8; ++k) T[kTileGap + k] = v.gap[8 * g + k];
    const int64_t f = m * v.NY + n;
    for (int k = 0; k < 4; ++k) T[kTileEbRange + k] = v.fovr[4 * f + k];
    for (int k = 0; k < 8; ++k) T[kTileEbRect + k] = v.fov[8 * f + k];
    const double c_ic1 = tg[0], c_ic2 = tg[1], c_ic3 = tg[2];
    T[kTileCosIc1] = c_ic1;
    double *B = T + kTileHeader;
    // in-coupling event (GRTF:860-869)
    B[0] = c_ic2, B[1] = c_ic3;
    put_rec(B + kBlockRec, v.ic1, v.ch5, v, 0, l, m, n, 13, 18, 33, 38);
    put_rec(B + kBlockRec + 8, v.ic1, v.ch5, v, 0, l, m, n, 15, 20, 35, 40);
    // R0 (GRTF:909-918)
    B = T + kTileHeader + kBlock;
    B[0] = c_ic2, B[1] = c_ic3;
    put_rec(B + kBlockRec, v.ic2, v.ch5, v, 0, l, m, n, 4, 9, 24, 29);
    put_rec(B + kBlockRec + 8, v.ic2, v.ch5, v, 0, l, m, n, 6, 11, 26, 31);
    // R1 (GRTF:955-964) -- the reference's (2, 22, 7, 27) argument order kept
    B = T + kTileHeader + 2 * kBlock;
    B[0] = c_ic2, B[1] = c_ic3;
    put_rec(B + kBlockRec, v.ic3, v.ch5, v, 0, l, m, n, 2, 22, 7, 27);
    put_rec(B + kBlockRec + 8, v.ic3, v.ch5, v, 0, l, m, n, 4, 9, 24, 29);
    for (int k = 0; k < nfc; ++k) {
        B = T + kTileHeader + kBlock * (3 + k);   // R2 (GRTF:1007-1016)
        B[0] = cf1[k], B[1] = cf2[k];
        put_rec(B + kBlockRec, v.fc1, v.ch3, v, k, l, m, n, 3, 6, 15, 18);
        put_rec(B + kBlockRec + 8, v.fc1, v.ch3, v, k, l, m, n, 2, 5, 14, 17);
        B = T + kTileHeader + kBlock * (3 + nfc + k);   // R3 (GRTF:1060-1069)
        B[0] = cf1[k], B[1] = cf2[k];
        put_rec(B + kBlockRec, v.fc2, v.ch3, v, k, l, m, n, 4, 7, 16, 19);
        put_rec(B + kBlockRec + 8, v.fc2, v.ch3, v, k, l, m, n, 3, 6, 15, 18);
    }
    for (int k = 0; k < noc; ++k) {
        B = T + kTileHeader + kBlock * (3 + 2 * nfc + k);   // R4 (GRTF:1117-1131)
        B[0] = co1[k], B[1] = co2[k], B[2] = c_ic1;
        put_rec(B + kBlockRec, v.oc1, v.ch5, v, k, l, m, n, 4, 9, 24, 29);
        put_rec(B + kBlockRec + 8, v.oc1, v.ch5, v, k, l, m, n, 2, 7, 22, 27);
        put_rec(B + kBlockRec + 16, v.oc1, v.ch5, v, k, l, m, n, 13, 18, 33, 38);
        B = T + kTileHeader + kBlock * (3 + 2 * nfc + noc + k);   // R5 (GRTF:1186-1200)
        B[0] = co1[k], B[1] = co2[k], B[2] = c_ic1;
        put_rec(B + kBlockRec, v.oc2, v.ch5, v, k, l, m, n, 6, 11, 26, 31);
        put_rec(B + kBlockRec + 8, v.oc2, v.ch5, v, k, l, m, n, 4, 9, 24, 29);
        put_rec(B + kBlockRec + 16, v.oc2, v.ch5, v, k, l, m, n, 15, 20, 35, 40);
    }

    // the Jones-vector tile (wgrt_common.h kJ*)
    const double *tir = v.tir + 4 * g;
    for (int k = 0; k < 8; ++k) J[kJGap + k] = T[kTileGap + k];
    for (int k = 0; k < 4; ++k) J[kJHop + k] = T[kTileHopRot + k];
    J[kJCosIc1] = T[kTileCosIc1];
    double tir_max = 0.0;
    for (int k = 0; k < 4; ++k) tir_max = fabs(tir[k]) > tir_max ? fabs(tir[k]) : tir_max;
    J[kJGrowth] = tir_max / kPi > 1.0 ? tir_max / kPi : 1.0;
    const int nblk = 3 + 2 * nfc + 2 * noc;
    for (int b = 0; b < nblk; ++b) {
        const double *Bt = T + kTileHeader + kBlock * b;
        double *O = J + kJHeader + kJBlock * b;
        const bool three = b >= 3 + 2 * nfc;
        // TIR step of the taken branches (GRTF:877, 926, 942, 1026, 1039, ...): block 0-2 (IC
        // states) TIR[0] / TIR[2], FC blocks TIR[0] / TIR[1], OC blocks TIR[1] / TIR[3]
        const int ta = b < 3 ? 0 : (three ? 1 : 0), tb = b < 3 ? 2 : (three ? 3 : 1);
        double sum = 0.0;
        bool nonunitary = false;   // a taken branch (k < 2) whose matrix is not scaled-unitary
        O[kJBlockCos] = Bt[kBlockCos];
        O[kJBlockCos + 1] = Bt[kBlockCos + 1];
        O[kJBlockCos2] = Bt[kBlockCos + 2];
        float *const f32 = (float *)(O + kJBlockF32);
        for (int k = 0; k < 3; ++k) {
            double *rec = O + kJBlockRec + 8 * k;
            for (int j = 0; j < 8; ++j) rec[j] = Bt[kBlockRec + 8 * k + j];
            double w = 0.0;
            if (k < 2 || three) {
                const double p = hypot(rec[0], rec[1]), q = hypot(rec[2], rec[3]);
                const double r = hypot(rec[4], rec[5]), s = hypot(rec[6], rec[7]);
                const double fk = (b == 0) ? v.n_g : (k == 2 ? 1.0 / v.n_g : 1.0);
                // 1.01: covers the rounding of this bound itself
                w = ((p + r) * (p + r) + (q + s) * (q + s)) * fabs(Bt[kBlockCos + k]) * fk * 1.01;
            }
            if (k < 2) {   // turn the TM output row (q, s) by e^{i lut_TIR[t]}
                const int t = k == 0 ? ta : tb;
                const double c = rot[2 * t], sn = rot[2 * t + 1];
                for (int j = 2; j <= 6; j += 4) {
                    const double re = rec[j], im = rec[j + 1];
                    rec[j] = re * c - im * sn;
                    rec[j + 1] = re * sn + im * c;
                }
            }
            O[kJBlockW + k] = w;
            sum += w;
            // the estimate's single-precision Hermitian form H = M^H M (M = [[p, r], [q, s]]; the TIR
            // turn of the TM row does not change it)
            const double pr = rec[0], pi = rec[1], qr = rec[2], qi = rec[3];
            const double rr = rec[4], ri = rec[5], sr = rec[6], si = rec[7];
            float *h = (float *)(O + kJBlockHerm) + 4 * k;
            h[0] = (float)((pr * pr + pi * pi) + (qr * qr + qi * qi));
            h[1] = (float)((rr * rr + ri * ri) + (sr * sr + si * si));
            h[2] = (float)((pr * rr + pi * ri) + (qr * sr + qi * si));   // Re(conj(p) r + conj(q) s)
            h[3] = (float)((pr * ri - pi * rr) + (qr * si - qi * sr));   // Im(conj(p) r + conj(q) s)
            if (k < 2) {
                // kappa^2 = s1^2 / s2^2 of H (s1^2 - s2^2 = sqrt((h11 - h22)^2 + 4 |h12|^2), no cancellation):
                // not scaled-unitary once kappa^2 > 1 + 1e-6 (the Jones lane's amplification step, wgrt_device.h)
                const double h11 = (pr * pr + pi * pi) + (qr * qr + qi * qi), h22 = (rr * rr + ri * ri) + (sr * sr + si * si);
                const double g_re = (pr * rr + pi * ri) + (qr * sr + qi * si), g_im = (pr * ri - pi * rr) + (qr * si - qi * sr);
                const double dif = sqrt((h11 - h22) * (h11 - h22) + 4.0 * (g_re * g_re + g_im * g_im));
                const double s2 = 0.5 * ((h11 + h22) - dif);
                if (h11 + h22 > 0.0 && !(dif <= 1e-6 * s2)) nonunitary = true;
            }
        }
        f32[0] = (float)(sum * 1.01);   // 1.01: covers this bound's own rounding to float
        if (nonunitary) f32[0] = -f32[0];   // the sign bit flags the block (block_cw)
        // the phase-growth bound with the block's line-0 loads (it only ever scales a tolerance up, so
        // rounded up); block 0 also carries the in-coupling event's denominator cos(ic1) as the bits
        // of a double, in place of the cosA_2 it does not have
        const float growth = (float)(J[kJGrowth] * 1.000001);
        if (b == 0) {
            f32[1] = growth;
            O[kJBlockF32 + 1] = J[kJCosIc1];
        } else {
            f32[1] = (float)Bt[kBlockCos + 2];
            f32[2] = growth;
            f32[3] = 0.0f;
        }
    }
}

}  // namespace wgrt
