// wgrt_scene_build.h -- host-side scene preparation (see wgrt_scene_build.cpp).
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/wgrt.h"
#include "wgrt_pack.h"

namespace wgrt {

constexpr int kBandSegs = 4;

struct LocatorHost {
    std::vector<uint64_t> cells;   // [ncy][ncx], 2 bits per polygon: 0 OUT, 1 IN, 2 EDGE
    std::vector<double> verts;     // all polygon vertices, [V][2]
    std::vector<int32_t> poly_off; // polygon k = verts[poly_off[k] .. poly_off[k+1])
    // row-band edge lists (CSR): the edges of polygon k whose y-range, padded, meets cell
    // row cy are row_edges[row_off[k * ncy + cy] .. row_off[k * ncy + cy + 1]), each given
    // as the index i (within polygon k) of its end vertex; its start vertex is i - 1 (mod nv)
    std::vector<int32_t> row_off;
    std::vector<int32_t> row_edges;
    // the same row bands as fixed 128-B records (Jones-vector kernels): up to kBandSegs
    // segments (x_start, y_start, x_end, y_end) of polygon k's edges meeting row cy, unused
    // slots NaN (inert in the predicate); a band with more edges starts with +inf and is
    // resolved through row_off / row_edges instead
    std::vector<double> bands;
    double x0 = 0, y0 = 0, h = 0, inv_h = 0;
    int ncx = 0, ncy = 0;
    int64_t edge_cells = 0;
};

struct SceneHost {
    LocatorHost loc;
    std::vector<double> tiles;     // [num_lmd * nx * ny][tile_doubles]
    int tile_doubles = 0;
    std::vector<double> jtiles;    // [num_lmd * nx * ny][jtile_doubles] (Jones-vector variants)
    int jtile_doubles = 0;
    std::vector<double> trig;      // [num_lmd * nx * ny][trig_doubles]: host-libm cos / sin (build_trig)
};

// grid extent, vertices, row-band edge lists and band records (everything but the cell words)
void build_locator_geometry(const std::vector<const double *> &polys, const std::vector<int64_t> &nverts,
                            double cell_mm, LocatorHost &out);
// the cell words on the host (the device builds them with the same edge_row_span / parity rules)
void classify_cells_host(const std::vector<const double *> &polys, const std::vector<int64_t> &nverts,
                         LocatorHost &out);
void build_locator(const std::vector<const double *> &polys, const std::vector<int64_t> &nverts,
                   double cell_mm, LocatorHost &out);
PackView pack_view(const wgrt_scene_desc &d, const double *trig);
// lut_f32_angles: wgrt_scene_opts bit mask of complex64 tables (cosf of their float32 angles)
void build_trig(const wgrt_scene_desc &d, std::vector<double> &trig, int lut_f32_angles = 0);
void pack_tiles_host(const wgrt_scene_desc &d, const std::vector<double> &trig, std::vector<double> &tiles,
                     std::vector<double> &jtiles);
void validate_desc(const wgrt_scene_desc &d);
// cells: classify the grid on the host; pack: pack the tiles on the host
void build_scene_host(const wgrt_scene_desc &d, double cell_mm, SceneHost &out, bool cells = true, bool pack = true,
                      int lut_f32_angles = 0);
// the polygon list the locator covers: eff_reg1, eff_reg2, IC, FC slices, OC slices
void scene_polygons(const wgrt_scene_desc &d, std::vector<const double *> &polys, std::vector<int64_t> &nv);


}  // namespace wgrt
