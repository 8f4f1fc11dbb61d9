// wgrt_scene_build.cpp -- host-side scene preparation (one-shot, C++).
//
// Turns the reference's 19 scene arrays (couplers_coor_full_color outputs + the seven
// RCWA LUTs, gpu_ray_tracing_pro_fullColor.py:19-57) into the two device structures
// the bounce kernel reads:
//
//  1. Packed LUT tiles, one per (lambda, m, n): the channels the kernel gathers
//      re-ordered into per-FSM-state "interaction blocks" in the
//     exact (p, q, r, s) argument order of each E_field_cal call, plus the cosines of
//     the LUT polar angles.  The cosines are computed here with the host libm cos --
//     the same function Python's math.cos calls in the reference (GRTF:868-1200), so
//     they are bit-identical to the reference's values.
//
//  2. An exact polygon locator: a uniform grid over all coupler / region polygons in
//     which every cell stores, per polygon, 2 bits: OUT, IN, or EDGE.  A cell is IN/OUT
//     only when no point of the cell (expanded by kPad) lies within kPad of any edge of
//     the polygon; the answer is then taken from the reference predicate
//     (is_inside_or_on_edge, GRTF:63-71) evaluated at the cell centre.  For such a cell
//     every point gives the same answer as the centre, bit for bit: the on-edge test
//     fails on its bounding-box pre-check or on |cross| > tol (|edge| * kPad >> tol),
//     and each crossing comparison is at least kPad from its rounding-sensitive point.
//     EDGE cells fall back to the exact reference predicate in the kernel, restricted to
//     the polygon's edges whose (padded) y-range meets the cell's row: every other edge
//     fails on_segment's y bounding-box check and cannot straddle the point's y, so
//     dropping it changes neither the "any on-edge" nor the crossing parity.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "wgrt_common.h"
#include "wgrt_scene_build.h"
#include "../../include/wgrt.h"

namespace wgrt {

namespace {

constexpr double kPad = 1e-6;          // mm; >> tol (1e-12) and >> float64 rounding at |x| ~ 60 mm
constexpr double kShortEdge = 1e-4;    // mm; shorter edges use the bbox criterion

struct Poly {
    const double *xy;
    int64_t nv;
};

// Does the segment (ax,ay)-(bx,by) intersect the closed rectangle [x0,x1]x[y0,y1]?
// Liang-Barsky clipping.
bool segment_hits_rect(double ax, double ay, double bx, double by, double x0, double x1, double y0,
                       double y1) {
    double t0 = 0.0, t1 = 1.0;
    const double dx = bx - ax, dy = by - ay;
    const double p[4] = {-dx, dx, -dy, dy};
    const double q[4] = {ax - x0, x1 - ax, ay - y0, y1 - ay};
    for (int k = 0; k < 4; ++k) {
        if (p[k] == 0.0) {
            if (q[k] < 0.0) return false;
        } else {
            const double t = q[k] / p[k];
            if (p[k] < 0.0) {
                if (t > t1) return false;
                if (t > t0) t0 = t;
            } else {
                if (t < t0) return false;
                if (t < t1) t1 = t;
            }
        }
    }
    return t0 <= t1;
}

void check(bool ok, const std::string &msg) {
    if (!ok) throw std::invalid_argument(msg);
}

}  // namespace

void build_locator(const std::vector<const double *> &polys, const std::vector<int64_t> &nverts,
                   double cell_mm, LocatorHost &out) {
    const int np = (int)polys.size();
    check(np <= 32, "at most 32 polygons (eff_reg1, eff_reg2, IC, FC and OC slices) are supported");
    double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
    out.poly_off.assign(np + 1, 0);
    out.verts.clear();
    for (int k = 0; k < np; ++k) {
        for (int64_t v = 0; v < nverts[k]; ++v) {
            const double x = polys[k][2 * v], y = polys[k][2 * v + 1];
            check(std::isfinite(x) && std::isfinite(y), "polygon vertex is not finite");
            xmin = std::min(xmin, x);
            xmax = std::max(xmax, x);
            ymin = std::min(ymin, y);
            ymax = std::max(ymax, y);
            out.verts.push_back(x);
            out.verts.push_back(y);
        }
        out.poly_off[k + 1] = out.poly_off[k] + (int32_t)nverts[k];
    }
    if (!(xmin <= xmax)) {  // no vertices at all
        xmin = ymin = 0.0;
        xmax = ymax = 1.0;
    }
    double h = cell_mm;
    // keep the grid below ~32M cells (256 MB of 64-bit host words) whatever the coordinate range
    while (((xmax - xmin) / h + 5) * ((ymax - ymin) / h + 5) > 3.2e7) h *= 2.0;
    const double x0 = std::floor(xmin / h) * h - 2 * h;
    const double y0 = std::floor(ymin / h) * h - 2 * h;
    const int ncx = (int)std::ceil((xmax - x0) / h) + 3;
    const int ncy = (int)std::ceil((ymax - y0) / h) + 3;
    out.x0 = x0;
    out.y0 = y0;
    out.h = h;
    out.inv_h = 1.0 / h;
    out.ncx = ncx;
    out.ncy = ncy;
    out.cells.assign((size_t)ncx * ncy, 0ull);
    out.edge_cells = 0;

    std::vector<uint8_t> edge((size_t)ncx * ncy);
    out.row_off.assign((size_t)np * ncy + 1, 0);
    out.row_edges.clear();
    for (int k = 0; k < np; ++k) {
        const double *xy = polys[k];
        const int64_t nv = nverts[k];
        for (int cy = 0; cy < ncy; ++cy) {
            const double by0 = y0 + cy * h - 2 * kPad, by1 = y0 + (cy + 1) * h + 2 * kPad;
            for (int64_t i = 0, j = nv - 1; i < nv; j = i++) {
                const double ey0 = std::min(xy[2 * j + 1], xy[2 * i + 1]) - 2 * kPad;
                const double ey1 = std::max(xy[2 * j + 1], xy[2 * i + 1]) + 2 * kPad;
                if (!(ey1 < by0 || ey0 > by1)) out.row_edges.push_back((int32_t)i);
            }
            out.row_off[(size_t)k * ncy + cy + 1] = (int32_t)out.row_edges.size();
        }
    }
    out.bands.assign((size_t)np * ncy * 4 * kBandSegs, NAN);
    for (int k = 0; k < np; ++k) {
        const double *xy = polys[k];
        const int64_t nv = nverts[k];
        for (int cy = 0; cy < ncy; ++cy) {
            const size_t r = (size_t)k * ncy + cy;
            double *rec = out.bands.data() + r * 4 * kBandSegs;
            const int e0 = out.row_off[r], e1 = out.row_off[r + 1];
            if (e1 - e0 > kBandSegs) {
                rec[0] = INFINITY;
                continue;
            }
            for (int e = e0; e < e1; ++e) {
                const int64_t i = out.row_edges[e], j = (i == 0) ? nv - 1 : i - 1;
                double *sg = rec + 4 * (e - e0);
                sg[0] = xy[2 * j];
                sg[1] = xy[2 * j + 1];
                sg[2] = xy[2 * i];
                sg[3] = xy[2 * i + 1];
            }
        }
    }
    std::vector<double> xs;
    for (int k = 0; k < np; ++k) {
        std::fill(edge.begin(), edge.end(), 0);
        const double *xy = polys[k];
        const int64_t nv = nverts[k];
        const double pad2 = 2 * kPad;
        // (1) EDGE cells, row by row: the cells of row cy (expanded by pad2) that the edge's
        //     part inside the row's y-range (expanded by pad2) can reach, widened by pad2.
        for (int64_t i = 0, j = nv - 1; i < nv; j = i++) {
            const double ax = xy[2 * j], ay = xy[2 * j + 1], bx = xy[2 * i], by = xy[2 * i + 1];
            const double len = std::hypot(bx - ax, by - ay);
            const double ey0 = std::min(ay, by) - pad2, ey1 = std::max(ay, by) + pad2;
            const int cy0 = std::max(0, (int)std::floor((ey0 - y0) / h) - 1);
            const int cy1 = std::min(ncy - 1, (int)std::floor((ey1 - y0) / h) + 1);
            for (int cy = cy0; cy <= cy1; ++cy) {
                const double ry0 = y0 + cy * h - pad2, ry1 = y0 + (cy + 1) * h + pad2;
                double lo, hi;
                if (len < kShortEdge || std::fabs(by - ay) < 1e-300) {
                    if (ey1 < ry0 || ey0 > ry1) continue;
                    lo = std::min(ax, bx);
                    hi = std::max(ax, bx);
                } else {
                    // parameter range of the segment inside [ry0, ry1]
                    double t0 = (ry0 - ay) / (by - ay), t1 = (ry1 - ay) / (by - ay);
                    if (t0 > t1) std::swap(t0, t1);
                    t0 = std::max(t0, 0.0);
                    t1 = std::min(t1, 1.0);
                    if (t0 > t1 + 1e-12) continue;
                    const double xa = ax + t0 * (bx - ax), xb = ax + t1 * (bx - ax);
                    lo = std::min(xa, xb);
                    hi = std::max(xa, xb);
                }
                lo -= pad2 + 1e-9;
                hi += pad2 + 1e-9;
                const int cx0 = std::max(0, (int)std::floor((lo - x0) / h));
                const int cx1 = std::min(ncx - 1, (int)std::floor((hi - x0) / h));
                for (int cx = cx0; cx <= cx1; ++cx) edge[(size_t)cy * ncx + cx] = 1;
            }
        }
        // (2) IN / OUT of the other cells: the reference predicate at the cell centre,
        //     evaluated for a whole row at once.  At a non-EDGE centre no edge is on-edge
        //     (bounding box), so the predicate is the crossing parity; the crossings of the
        //     row-centre line are computed with the reference's own expression (GRTF:47) and
        //     counted against the centres in one sweep.
        for (int cy = 0; cy < ncy; ++cy) {
            const double py = y0 + (cy + 0.5) * h;
            xs.clear();
            for (int64_t i = 0, j = nv - 1; i < nv; j = i++) {
                const double xi = xy[2 * i], yi = xy[2 * i + 1], xj = xy[2 * j], yj = xy[2 * j + 1];
                if ((yi > py) != (yj > py)) xs.push_back((xj - xi) * (py - yi) / (yj - yi + 1e-20) + xi);
            }
            std::sort(xs.begin(), xs.end());
            size_t le = 0;   // crossings with xint <= px
            for (int cx = 0; cx < ncx; ++cx) {
                const size_t c = (size_t)cy * ncx + cx;
                const double px = x0 + (cx + 0.5) * h;
                while (le < xs.size() && !(px < xs[le])) ++le;
                uint64_t cls;
                if (edge[c]) {
                    cls = 2;
                    ++out.edge_cells;
                } else {
                    cls = ((xs.size() - le) & 1u) ? 1 : 0;   // parity of crossings with px < xint
                }
                out.cells[c] |= cls << (2 * k);
            }
        }
    }
}

namespace {

struct LutView {
    const double *p;  // complex interleaved
    int64_t slices, L, nx, ny, ch;
    const double *at(int64_t s, int64_t l, int64_t m, int64_t n, int64_t c) const {
        return p + 2 * ((((s * L + l) * nx + m) * ny + n) * ch + c);
    }
};

void put_rec(double *dst, const LutView &v, int64_t s, int64_t l, int64_t m, int64_t n, int p, int q,
             int r, int t) {
    const int ch[4] = {p, q, r, t};
    for (int k = 0; k < 4; ++k) {
        const double *c = v.at(s, l, m, n, ch[k]);
        dst[2 * k] = c[0];
        dst[2 * k + 1] = c[1];
    }
}

}  // namespace

void pack_tiles(const wgrt_scene_desc &d, std::vector<double> &tiles) {
    const int64_t L = d.num_lmd, NX = d.nx, NY = d.ny;
    const int nfc = (int)d.n_fc_slices, noc = (int)d.n_oc_slices;
    const int TD = tile_doubles(nfc, noc);
    tiles.assign((size_t)(L * NX * NY) * TD, 0.0);
    const LutView ic1{d.lut_ic1, 1, L, NX, NY, d.ch5}, ic2{d.lut_ic2, 1, L, NX, NY, d.ch5},
        ic3{d.lut_ic3, 1, L, NX, NY, d.ch5};
    const LutView fc1{d.lut_fc1, nfc, L, NX, NY, d.ch3}, fc2{d.lut_fc2, nfc, L, NX, NY, d.ch3};
    const LutView oc1{d.lut_oc1, noc, L, NX, NY, d.ch5}, oc2{d.lut_oc2, noc, L, NX, NY, d.ch5};
    for (int64_t l = 0; l < L; ++l)
        for (int64_t m = 0; m < NX; ++m)
            for (int64_t n = 0; n < NY; ++n) {
                double *T = tiles.data() + (size_t)((l * NX + m) * NY + n) * TD;
                const int64_t g = (l * NX + m) * NY + n;
                for (int k = 0; k < 4; ++k) {
                    T[kTileTir + k] = d.lut_TIR[4 * g + k];
                    T[kTileTirRot + 2 * k] = std::cos(d.lut_TIR[4 * g + k]);
                    T[kTileTirRot + 2 * k + 1] = std::sin(d.lut_TIR[4 * g + k]);
                }
                for (int k = 0; k < 2; ++k) {
                    T[kTileHopRot + 2 * k] = std::cos(2 * d.lut_TIR[4 * g + k]);
                    T[kTileHopRot + 2 * k + 1] = std::sin(2 * d.lut_TIR[4 * g + k]);
                }
                for (int k = 0; k < 8; ++k) T[kTileGap + k] = d.lut_gap[8 * g + k];
                const int64_t f = m * NY + n;
                for (int k = 0; k < 4; ++k) T[kTileEbRange + k] = d.eff_reg_FOV_range[4 * f + k];
                for (int k = 0; k < 8; ++k) T[kTileEbRect + k] = d.eff_reg_FOV[8 * f + k];
                const double c_ic1 = std::cos(ic1.at(0, l, m, n, 0)[0]);
                const double c_ic2 = std::cos(ic2.at(0, l, m, n, 0)[0]);
                const double c_ic3 = std::cos(ic3.at(0, l, m, n, 0)[0]);
                T[kTileCosIc1] = c_ic1;
                auto block = [&](int b) { return T + kTileHeader + kBlock * b; };
                // in-coupling event (GRTF:860-869)
                double *B = block(0);
                B[0] = c_ic2, B[1] = c_ic3;
                put_rec(B + kBlockRec, ic1, 0, l, m, n, 13, 18, 33, 38);
                put_rec(B + kBlockRec + 8, ic1, 0, l, m, n, 15, 20, 35, 40);
                // R0 (GRTF:909-918)
                B = block(1);
                B[0] = c_ic2, B[1] = c_ic3;
                put_rec(B + kBlockRec, ic2, 0, l, m, n, 4, 9, 24, 29);
                put_rec(B + kBlockRec + 8, ic2, 0, l, m, n, 6, 11, 26, 31);
                // R1 (GRTF:955-964) -- the reference's (2, 22, 7, 27) argument order kept
                B = block(2);
                B[0] = c_ic2, B[1] = c_ic3;
                put_rec(B + kBlockRec, ic3, 0, l, m, n, 2, 22, 7, 27);
                put_rec(B + kBlockRec + 8, ic3, 0, l, m, n, 4, 9, 24, 29);
                for (int k = 0; k < nfc; ++k) {
                    const double cf1 = std::cos(fc1.at(k, l, m, n, 0)[0]);
                    const double cf2 = std::cos(fc2.at(k, l, m, n, 0)[0]);
                    B = block(3 + k);  // R2 (GRTF:1007-1016)
                    B[0] = cf1, B[1] = cf2;
                    put_rec(B + kBlockRec, fc1, k, l, m, n, 3, 6, 15, 18);
                    put_rec(B + kBlockRec + 8, fc1, k, l, m, n, 2, 5, 14, 17);
                    B = block(3 + nfc + k);  // R3 (GRTF:1060-1069)
                    B[0] = cf1, B[1] = cf2;
                    put_rec(B + kBlockRec, fc2, k, l, m, n, 4, 7, 16, 19);
                    put_rec(B + kBlockRec + 8, fc2, k, l, m, n, 3, 6, 15, 18);
                }
                for (int k = 0; k < noc; ++k) {
                    const double co1 = std::cos(oc1.at(k, l, m, n, 0)[0]);
                    const double co2 = std::cos(oc2.at(k, l, m, n, 0)[0]);
                    B = block(3 + 2 * nfc + k);  // R4 (GRTF:1117-1131)
                    B[0] = co1, B[1] = co2, B[2] = c_ic1;
                    put_rec(B + kBlockRec, oc1, k, l, m, n, 4, 9, 24, 29);
                    put_rec(B + kBlockRec + 8, oc1, k, l, m, n, 2, 7, 22, 27);
                    put_rec(B + kBlockRec + 16, oc1, k, l, m, n, 13, 18, 33, 38);
                    B = block(3 + 2 * nfc + noc + k);  // R5 (GRTF:1186-1200)
                    B[0] = co1, B[1] = co2, B[2] = c_ic1;
                    put_rec(B + kBlockRec, oc2, k, l, m, n, 6, 11, 26, 31);
                    put_rec(B + kBlockRec + 8, oc2, k, l, m, n, 4, 9, 24, 29);
                    put_rec(B + kBlockRec + 16, oc2, k, l, m, n, 15, 20, 35, 40);
                }
            }
}

void pack_jtiles(const wgrt_scene_desc &d, const std::vector<double> &tiles, std::vector<double> &jt) {
    const int64_t L = d.num_lmd, NX = d.nx, NY = d.ny;
    const int nfc = (int)d.n_fc_slices, noc = (int)d.n_oc_slices;
    const int TD = tile_doubles(nfc, noc), JD = jtile_doubles(nfc, noc);
    const int nblk = 3 + 2 * nfc + 2 * noc;
    jt.assign((size_t)(L * NX * NY) * JD, 0.0);
    for (int64_t g = 0; g < L * NX * NY; ++g) {
        const double *T = tiles.data() + (size_t)g * TD;
        double *J = jt.data() + (size_t)g * JD;
        const double *tir = d.lut_TIR + 4 * g;
        for (int k = 0; k < 8; ++k) J[kJGap + k] = T[kTileGap + k];
        for (int k = 0; k < 4; ++k) J[kJHop + k] = T[kTileHopRot + k];
        J[kJCosIc1] = T[kTileCosIc1];
        double tir_max = 0.0;
        for (int k = 0; k < 4; ++k) tir_max = std::max(tir_max, std::fabs(tir[k]));
        J[kJGrowth] = std::max(1.0, tir_max / kPi);
        for (int b = 0; b < nblk; ++b) {
            const double *B = T + kTileHeader + kBlock * b;
            double *O = J + kJHeader + kJBlock * b;
            const bool three = b >= 3 + 2 * nfc;
            // TIR step of the taken branches (GRTF:877, 926, 942, 1026, 1039, ...): block 0-2 (IC
            // states) TIR[0] / TIR[2], FC blocks TIR[0] / TIR[1], OC blocks TIR[1] / TIR[3]
            const int ta = b < 3 ? 0 : (three ? 1 : 0), tb = b < 3 ? 2 : (three ? 3 : 1);
            double sum = 0.0;
            for (int k = 0; k < 3; ++k) {
                O[kJBlockCos + k] = B[kBlockCos + k];
                double *rec = O + kJBlockRec + 8 * k;
                for (int j = 0; j < 8; ++j) rec[j] = B[kBlockRec + 8 * k + j];
                double w = 0.0;
                if (k < 2 || three) {
                    const double p = std::hypot(rec[0], rec[1]), q = std::hypot(rec[2], rec[3]);
                    const double r = std::hypot(rec[4], rec[5]), s = std::hypot(rec[6], rec[7]);
                    const double f = (b == 0) ? d.n_g : (k == 2 ? 1.0 / d.n_g : 1.0);
                    // 1.01: covers the rounding of this bound itself
                    w = ((p + r) * (p + r) + (q + s) * (q + s)) * std::fabs(B[kBlockCos + k]) * f * 1.01;
                }
                if (k < 2) {   // turn the TM output row (q, s) by e^{i lut_TIR[t]}
                    const double th = tir[k == 0 ? ta : tb], c = std::cos(th), sn = std::sin(th);
                    for (int j : {2, 6}) {
                        const double re = rec[j], im = rec[j + 1];
                        rec[j] = re * c - im * sn;
                        rec[j + 1] = re * sn + im * c;
                    }
                }
                O[kJBlockW + k] = w;
                sum += w;
                float *r32 = (float *)(O + kJBlockRec32) + 8 * k;   // the estimate's single-precision copy
                for (int j = 0; j < 8; ++j) r32[j] = (float)rec[j];
            }
            O[kJBlockWsum] = sum * 1.01;
        }
    }
}

void validate_desc(const wgrt_scene_desc &d) {
    check(d.num_lmd > 0 && d.nx > 0 && d.ny > 0, "num_lmd, nx, ny must be positive");
    check(d.n_fc_slices >= 0 && d.n_oc_slices >= 0, "slice counts must be >= 0");
    check(3 + d.n_fc_slices + d.n_oc_slices <= 32, "too many coupler slices (max 29 in total)");
    check(d.ch5 >= 41, "5-order LUTs need >= 41 channels (kernel reads channel 40)");
    check(d.ch3 >= 20, "3-order LUTs need >= 20 channels (kernel reads channel 19)");
    check(d.IC && d.eff_reg1 && d.eff_reg2 && d.eff_reg_FOV && d.eff_reg_FOV_range && d.lut_TIR &&
              d.lut_gap && d.lut_ic1 && d.lut_ic2 && d.lut_ic3,
          "NULL scene array");
    check(d.n_fc_slices == 0 || (d.FC && d.FC_offset && d.lut_fc1 && d.lut_fc2), "NULL FC array");
    check(d.n_oc_slices == 0 || (d.OC && d.OC_offset && d.lut_oc1 && d.lut_oc2), "NULL OC array");
    for (int64_t k = 0; k < d.n_fc_slices; ++k)
        check(d.FC_offset[k + 1] >= d.FC_offset[k], "FC_offset must be non-decreasing");
    for (int64_t k = 0; k < d.n_oc_slices; ++k)
        check(d.OC_offset[k + 1] >= d.OC_offset[k], "OC_offset must be non-decreasing");
    check(d.n_fc_slices == 0 || d.FC_offset[0] >= 0, "FC_offset[0] < 0");
    check(d.n_oc_slices == 0 || d.OC_offset[0] >= 0, "OC_offset[0] < 0");
}

void build_scene_host(const wgrt_scene_desc &d, double cell_mm, SceneHost &out) {
    validate_desc(d);
    std::vector<const double *> polys;
    std::vector<int64_t> nv;
    polys.push_back(d.eff_reg1);
    nv.push_back(d.n_eff_reg1);
    polys.push_back(d.eff_reg2);
    nv.push_back(d.n_eff_reg2);
    polys.push_back(d.IC);
    nv.push_back(d.n_ic);
    for (int64_t k = 0; k < d.n_fc_slices; ++k) {
        polys.push_back(d.FC + 2 * d.FC_offset[k]);
        nv.push_back(d.FC_offset[k + 1] - d.FC_offset[k]);
    }
    for (int64_t k = 0; k < d.n_oc_slices; ++k) {
        polys.push_back(d.OC + 2 * d.OC_offset[k]);
        nv.push_back(d.OC_offset[k + 1] - d.OC_offset[k]);
    }
    build_locator(polys, nv, cell_mm, out.loc);
    pack_tiles(d, out.tiles);
    pack_jtiles(d, out.tiles, out.jtiles);
    // The kernels' cheap branch estimates assume finite tables (an inf / NaN coefficient would
    // make the reference's efficiencies NaN); such LUTs are rejected instead.
    for (const double v : out.tiles) check(std::isfinite(v), "non-finite value in the LUTs / lut_TIR / lut_gap / eyebox tables");
    out.tile_doubles = tile_doubles((int)d.n_fc_slices, (int)d.n_oc_slices);
    out.jtile_doubles = jtile_doubles((int)d.n_fc_slices, (int)d.n_oc_slices);
}

}  // namespace wgrt
