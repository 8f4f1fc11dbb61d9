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
#include <map>
#include <vector>

#include "wgrt_common.h"
#include "wgrt_pack.h"
#include "wgrt_scene_build.h"
#include "../../include/wgrt.h"

namespace wgrt {

namespace {

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

void build_locator_geometry(const std::vector<const double *> &polys, const std::vector<int64_t> &nverts,
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
    out.cells.clear();
    out.edge_cells = 0;
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
}

void classify_cells_host(const std::vector<const double *> &polys, const std::vector<int64_t> &nverts,
                         LocatorHost &out) {
    const int np = (int)polys.size();
    const int ncx = out.ncx, ncy = out.ncy;
    const double x0 = out.x0, y0 = out.y0, h = out.h;
    out.cells.assign((size_t)ncx * ncy, 0ull);
    out.edge_cells = 0;
    std::vector<uint8_t> edge((size_t)ncx * ncy);
    std::vector<double> xs;
    for (int k = 0; k < np; ++k) {
        std::fill(edge.begin(), edge.end(), 0);
        const double *xy = polys[k];
        const int64_t nv = nverts[k];
        // (1) EDGE cells, row by row: the cells of row cy (expanded by 2 kPad) that the edge's
        //     part inside the row's y-range (expanded by 2 kPad) can reach, widened by 2 kPad
        //     (wgrt_pack.h edge_row_span, shared with the device build).
        for (int64_t i = 0, j = nv - 1; i < nv; j = i++) {
            const double ax = xy[2 * j], ay = xy[2 * j + 1], bx = xy[2 * i], by = xy[2 * i + 1];
            int cy0, cy1;
            edge_rows(ay, by, y0, h, ncy, cy0, cy1);
            for (int cy = cy0; cy <= cy1; ++cy) {
                int cx0, cx1;
                if (!edge_row_span(ax, ay, bx, by, cy, x0, y0, h, ncx, cx0, cx1)) continue;
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

void build_locator(const std::vector<const double *> &polys, const std::vector<int64_t> &nverts,
                   double cell_mm, LocatorHost &out) {
    build_locator_geometry(polys, nverts, cell_mm, out);
    classify_cells_host(polys, nverts, out);
}

PackView pack_view(const wgrt_scene_desc &d, const double *trig) {
    PackView v;
    v.ic1 = d.lut_ic1, v.ic2 = d.lut_ic2, v.ic3 = d.lut_ic3;
    v.fc1 = d.lut_fc1, v.fc2 = d.lut_fc2, v.oc1 = d.lut_oc1, v.oc2 = d.lut_oc2;
    v.tir = d.lut_TIR, v.gap = d.lut_gap, v.fov = d.eff_reg_FOV, v.fovr = d.eff_reg_FOV_range;
    v.trig = trig;
    v.L = d.num_lmd, v.NX = d.nx, v.NY = d.ny;
    v.ch5 = (int)d.ch5, v.ch3 = (int)d.ch3, v.nfc = (int)d.n_fc_slices, v.noc = (int)d.n_oc_slices;
    v.n_g = d.n_g;
    return v;
}

void build_trig(const wgrt_scene_desc &d, std::vector<double> &trig, int lut_f32_angles) {
    const int nfc = (int)d.n_fc_slices, noc = (int)d.n_oc_slices;
    const int TG = trig_doubles(nfc, noc);
    const int64_t ntiles = (int64_t)d.num_lmd * d.nx * d.ny;
    trig.assign((size_t)ntiles * TG, 0.0);
    const PackView v = pack_view(d, nullptr);
    // math.cos of table k's angle: libm cos, or cosf of the float32 angle for a complex64 table
    auto lcos = [&](int k, double th) -> double {
        return ((lut_f32_angles >> k) & 1) ? (double)std::cos((float)th) : std::cos(th);
    };
    for (int64_t g = 0; g < ntiles; ++g) {
        const int64_t n = g % d.ny, m = g / d.ny % d.nx, l = g / ((int64_t)d.ny * d.nx);
        double *t = trig.data() + (size_t)g * TG;
        // math.cos of each LUT's polar angle (channel 0, real part; GRTF:868-1200)
        t[0] = lcos(0, lut_at(d.lut_ic1, 0, l, m, n, 0, v, v.ch5)[0]);
        t[1] = lcos(1, lut_at(d.lut_ic2, 0, l, m, n, 0, v, v.ch5)[0]);
        t[2] = lcos(2, lut_at(d.lut_ic3, 0, l, m, n, 0, v, v.ch5)[0]);
        for (int k = 0; k < nfc; ++k) {
            t[3 + k] = lcos(3, lut_at(d.lut_fc1, k, l, m, n, 0, v, v.ch3)[0]);
            t[3 + nfc + k] = lcos(4, lut_at(d.lut_fc2, k, l, m, n, 0, v, v.ch3)[0]);
        }
        for (int k = 0; k < noc; ++k) {
            t[3 + 2 * nfc + k] = lcos(5, lut_at(d.lut_oc1, k, l, m, n, 0, v, v.ch5)[0]);
            t[3 + 2 * nfc + noc + k] = lcos(6, lut_at(d.lut_oc2, k, l, m, n, 0, v, v.ch5)[0]);
        }
        double *rot = t + 3 + 2 * nfc + 2 * noc;
        for (int k = 0; k < 4; ++k) {
            rot[2 * k] = std::cos(d.lut_TIR[4 * g + k]);
            rot[2 * k + 1] = std::sin(d.lut_TIR[4 * g + k]);
        }
        for (int k = 0; k < 2; ++k) {
            rot[8 + 2 * k] = std::cos(2 * d.lut_TIR[4 * g + k]);
            rot[8 + 2 * k + 1] = std::sin(2 * d.lut_TIR[4 * g + k]);
        }
    }
}

void pack_tiles_host(const wgrt_scene_desc &d, const std::vector<double> &trig, std::vector<double> &tiles,
                     std::vector<double> &jtiles) {
    const int nfc = (int)d.n_fc_slices, noc = (int)d.n_oc_slices;
    const int TD = tile_doubles(nfc, noc), JD = jtile_doubles(nfc, noc);
    const int64_t ntiles = (int64_t)d.num_lmd * d.nx * d.ny;
    tiles.assign((size_t)ntiles * TD, 0.0);
    jtiles.assign((size_t)ntiles * JD, 0.0);
    const PackView v = pack_view(d, trig.data());
    for (int64_t g = 0; g < ntiles; ++g) pack_tile(v, g, tiles.data() + (size_t)g * TD, jtiles.data() + (size_t)g * JD);
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

void scene_polygons(const wgrt_scene_desc &d, std::vector<const double *> &polys, std::vector<int64_t> &nv) {
    polys.clear();
    nv.clear();
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
}

void build_scene_host(const wgrt_scene_desc &d, double cell_mm, SceneHost &out, bool cells, bool pack,
                      int lut_f32_angles) {
    validate_desc(d);
    std::vector<const double *> polys;
    std::vector<int64_t> nv;
    scene_polygons(d, polys, nv);
    if (cells)
        build_locator(polys, nv, cell_mm, out.loc);
    else
        build_locator_geometry(polys, nv, cell_mm, out.loc);
    build_trig(d, out.trig, lut_f32_angles);
    if (pack) {
        pack_tiles_host(d, out.trig, out.tiles, out.jtiles);
        // The kernels' cheap branch estimates assume finite tables (an inf / NaN coefficient would
        // make the reference's efficiencies NaN); such LUTs are rejected instead.
        for (const double v : out.tiles)
            check(std::isfinite(v), "non-finite value in the LUTs / lut_TIR / lut_gap / eyebox tables");
    }
    out.tile_doubles = tile_doubles((int)d.n_fc_slices, (int)d.n_oc_slices);
    out.jtile_doubles = jtile_doubles((int)d.n_fc_slices, (int)d.n_oc_slices);
}

}  // namespace wgrt
