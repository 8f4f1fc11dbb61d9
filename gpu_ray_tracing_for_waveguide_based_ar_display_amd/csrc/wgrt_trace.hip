// wgrt_trace.hip -- CDNA4 (gfx950) kernels of the waveguide Monte-Carlo bounce loop
// and the C ABI declared in include/wgrt.h.
//
// Restates the reference's full-colour kernel process_rays_kernel_pro_fullColor
// (GPU_ray_tracing_functions.py = GRTF:833-1246, call at gpu_ray_tracing_pro_fullColor.py:170).
// One ray per lane (wave64); the ray record lives in VGPRs for its whole life; the
// only global writes are the final RNG state, optional per-ray bounce counts, one
// float atomic per eyebox hit (GRTF:164) and one set of 64-bit stats atomics per
// workgroup.
//
// Arithmetic is float64 throughout, like the reference (its state is promoted to
// float64 on first use, GRTF:846-882), compiled with -ffp-contract=off and in the
// reference's expression order, so results match the reference bit for bit except
// where the device libm's cos/sin/atan2 differ from glibc's in the last ulp -- which
// changes a Monte-Carlo decision only if a uniform draw lands within ~1e-16 of a
// branch threshold.
//
// Kernel structure: the reference's six-state machine (R0..R5)
// is driven by data.  Every coupler interaction, whatever its state, runs the same
// instruction stream: fetch one "interaction block" of the per-(lambda, FoV) LUT tile
// (2 or 3 Jones matrices + cosines), evaluate the branch efficiencies, draw, pick the
// branch, and only then evaluate the atan2 phase of the chosen branch.  The six states
// therefore diverge only in the short polygon-scan / hop code, not in the fp64 math.
// Polygon membership goes through the exact grid locator (wgrt_scene_build.cpp).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wgrt.h"
#include "wgrt_common.h"
#include "wgrt_scene_build.h"

using namespace wgrt;

namespace {

thread_local std::string g_last_error;

wgrt_status fail(wgrt_status s, const std::string &msg) {
    g_last_error = msg;
    return s;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(WGRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

// ----------------------------------------------------------------------------
// device-side scene view
// ----------------------------------------------------------------------------
struct Locator {
    const uint64_t *cells;
    const double *verts;
    const int32_t *poly_off;
    double x0, y0, inv_h;
    int ncx, ncy;
};

struct TraceArgs {
    const float *x, *y, *m, *n, *l, *te, *tm, *dph;
    uint32_t *rng;
    float *eb;
    wgrt_trace_stats *stats;
    uint32_t *per_ray;
    int64_t n_rays, gid_offset;
    const double *tiles;
    Locator loc;
    int tile_d, nfc, noc, nx, ny, nl;
    double n_g;
};

constexpr int kPolyEff1 = 0;
constexpr int kPolyEff2 = 1;
constexpr int kPolyIC = 2;
constexpr int kPolyFC0 = 3;

__device__ __forceinline__ uint64_t cell_word(const Locator &L, double x, double y) {
    const double fx = floor((x - L.x0) * L.inv_h);
    const double fy = floor((y - L.y0) * L.inv_h);
    // NaN / out-of-grid points are outside every polygon (cell word 0 = all OUT)
    if (!(fx >= 0.0 && fy >= 0.0 && fx < (double)L.ncx && fy < (double)L.ncy)) return 0ull;
    return L.cells[(int)fy * L.ncx + (int)fx];
}

__device__ __forceinline__ bool in_poly(const Locator &L, uint64_t w, int k, double x, double y) {
    const unsigned c = (unsigned)(w >> (2 * k)) & 3u;
    if (c != 2u) return c == 1u;
    const int a = L.poly_off[k], b = L.poly_off[k + 1];
    return inside_or_on_edge(x, y, L.verts + 2 * a, b - a);
}

// First slice s in [first, first + count) containing (x, y), -1 if none (GRTF:1002-1005).
__device__ __forceinline__ int first_slice(const Locator &L, uint64_t w, int first, int count,
                                           double x, double y) {
    for (int s = 0; s < count; ++s)
        if (in_poly(L, w, first + s, x, y)) return s;
    return -1;
}

struct Amp {
    double te_re, te_im, tm_re, tm_im, te, tm;
};

// E_field_cal (GRTF:132-152) up to the magnitudes.  rec = (p, q, r, s) complex, the
// reference call's argument order: Ete' = p*te_in + r*tm_in, Etm' = q*te_in + s*tm_in.
// The multiplications by 0.0 are Python's real->complex promotions; they are kept so
// signed zeros propagate exactly as in the reference.
__device__ __forceinline__ void efield_amp(double Ete, double Etm, double cd, double sd,
                                           const double *rec, Amp &o) {
    const double pr = rec[0], pi = rec[1], qr = rec[2], qi = rec[3];
    const double rr = rec[4], ri = rec[5], sr = rec[6], si = rec[7];
    const double ti_re = cd * Etm - sd * 0.0, ti_im = cd * 0.0 + sd * Etm;
    const double a_re = pr * Ete - pi * 0.0, a_im = pr * 0.0 + pi * Ete;
    const double b_re = rr * ti_re - ri * ti_im, b_im = rr * ti_im + ri * ti_re;
    const double c_re = qr * Ete - qi * 0.0, c_im = qr * 0.0 + qi * Ete;
    const double d_re = sr * ti_re - si * ti_im, d_im = sr * ti_im + si * ti_re;
    o.te_re = a_re + b_re;
    o.te_im = a_im + b_im;
    o.tm_re = c_re + d_re;
    o.tm_im = c_im + d_im;
    o.te = hypot_cr(o.te_re, o.te_im);
    o.tm = hypot_cr(o.tm_re, o.tm_im);
}

__device__ __forceinline__ double efield_phase(const Amp &o) {
    const double pte = (o.te >= 1e-20) ? atan2(o.te_im, o.te_re) : 0.0;
    const double ptm = (o.tm >= 1e-20) ? atan2(o.tm_im, o.tm_re) : 0.0;
    return wrap_pi(ptm - pte);
}

struct Ray {
    double x, y, te, tm, dph, cos_t, ener;
    uint32_t s;
    int region;
};

enum : int { kDie = -1 };

// kind: 0 in-coupler states (entry event, R0, R1), 1 R2, 2 R3, 3 R4, 4 R5.
// Returns the next region or kDie; *eb_hit set when the ray is out-coupled into the eyebox.
__device__ __forceinline__ int interact(const TraceArgs &A, Ray &r, const double *T, const double *B,
                                        int kind, bool entry, int64_t gid, int l, int m, int n,
                                        bool &eb_hit) {
    double sd, cd;
    sincos(r.dph, &sd, &cd);
    const bool three = kind >= 3;
    Amp a0, a1, a2;
    efield_amp(r.te, r.tm, cd, sd, B + kBlockRec, a0);
    efield_amp(r.te, r.tm, cd, sd, B + kBlockRec + 8, a1);
    if (three) efield_amp(r.te, r.tm, cd, sd, B + kBlockRec + 16, a2);
    const double denom = entry ? T[kTileCosIc1] : r.cos_t;
    double e0 = (a0.te * a0.te + a0.tm * a0.tm) * B[0] / denom;
    double e1 = (a1.te * a1.te + a1.tm * a1.tm) * B[1] / denom;
    if (entry) {
        e0 = e0 * A.n_g;
        e1 = e1 * A.n_g;
    }
    double e2 = 0.0;
    if (three) e2 = (a2.te * a2.te + a2.tm * a2.tm) * B[2] / denom / A.n_g;
    const double u = rng_draw(r.s, gid);
    const bool thr = kind >= 1;  // the ener > threshold guard exists only in R2..R5
    int b;
    if (u <= e0 && (!thr || r.ener * e0 > 0.0)) b = 0;
    else if (u <= e0 + e1 && (!thr || r.ener * e1 > 0.0)) b = 1;
    else if (three && u <= e0 + e1 + e2 && r.ener * e2 > 0.0) b = 2;
    else return kDie;

    if (b == 2) {  // out-coupling (GRTF:1162-1171, 1231-1240)
        if (inside_or_on_edge(r.x, r.y, T + kTileEbRect, 4)) {
            const double xmin = T[kTileEbRange], xmax = T[kTileEbRange + 1];
            const double ymin = T[kTileEbRange + 2], ymax = T[kTileEbRange + 3];
            const double dx = (xmax - xmin) / kEbNx, dy = (ymax - ymin) / kEbNy;
            int64_t ix = (int64_t)floor((r.x - xmin) / dx);
            int64_t iy = (int64_t)floor((r.y - ymin) / dy);
            // compiled-numba addressing (GRTF:164): a negative index wraps once, an index
            // equal to the axis length aliases into the next row; guarded to the buffer
            if (ix < 0) ix += kEbNx;
            if (iy < 0) iy += kEbNy;
            const int64_t off = ((((int64_t)l * A.ny + n) * A.nx + m) * kEbNy + iy) * kEbNx + ix;
            const int64_t total = (int64_t)A.nl * A.ny * A.nx * kEbNy * kEbNx;
            if (off >= 0 && off < total) {
                unsafeAtomicAdd(A.eb + off, 1.0f);
                eb_hit = true;
            }
        }
        return kDie;
    }
    const Amp &c = b == 0 ? a0 : a1;
    const double e = b == 0 ? e0 : e1;
    // take the branch (GRTF:872-882 and every branch body after it)
    const double norm = sqrt(c.te * c.te + c.tm * c.tm);
    const double ph = efield_phase(c);
    int tir, gap;
    if (kind == 0) { tir = b == 0 ? 0 : 2; gap = b == 0 ? 0 : 4; }
    else if (kind <= 2) { tir = b == 0 ? 0 : 1; gap = b == 0 ? 0 : 2; }
    else { tir = b == 0 ? 1 : 3; gap = b == 0 ? 2 : 6; }
    r.cos_t = B[b];
    r.te = c.te / norm;
    r.tm = c.tm / norm;
    r.dph = ph + T[kTileTir + tir];
    r.x += T[kTileGap + gap];
    r.y += T[kTileGap + gap + 1];
    r.ener = r.ener * e;
    if (kind == 0) {
        const bool in_ic = in_poly(A.loc, cell_word(A.loc, r.x, r.y), kPolyIC, r.x, r.y);
        if (b == 0) return in_ic ? 0 : 2;
        return in_ic ? 1 : kDie;
    }
    if (kind <= 2) return b == 0 ? 2 : 3;
    return b == 0 ? 4 : 5;
}

struct RayOutcome {
    uint32_t bounces;
    bool eb_hit;
    bool bad;
};

__device__ __forceinline__ RayOutcome trace_one(const TraceArgs &A, int64_t i) {
    RayOutcome out{0u, false, false};
    const int m = (int)A.m[i], n = (int)A.n[i], l = (int)A.l[i];
    if (!(m >= 0 && m < A.nx && n >= 0 && n < A.ny && l >= 0 && l < A.nl)) {
        out.bad = true;
        return out;
    }
    const int64_t gid = A.gid_offset + i;
    const double *T = A.tiles + (int64_t)((l * A.nx + m) * A.ny + n) * A.tile_d;
    const double *blocks = T + kTileHeader;
    Ray r;
    r.x = (double)A.x[i];
    r.y = (double)A.y[i];
    r.te = (double)A.te[i];
    r.tm = (double)A.tm[i];
    r.dph = (double)A.dph[i];
    r.cos_t = 1.0;
    r.ener = 1.0;
    r.s = A.rng[i];
    uint32_t bounces = 1;
    bool hit = false;
    int region = interact(A, r, T, blocks, 0, true, gid, l, m, n, hit);
    const int nfc = A.nfc, noc = A.noc;
    for (int64_t it = 0; region >= 0 && it < kMaxLoop; ++it) {
        ++bounces;
        const uint64_t w = cell_word(A.loc, r.x, r.y);
        if (!in_poly(A.loc, w, kPolyEff1, r.x, r.y)) break;  // GRTF:906
        int blk;
        int kind;
        if (region <= 1) {
            blk = 1 + region;
            kind = 0;
        } else if (region <= 3) {
            const int s = first_slice(A.loc, w, kPolyFC0, nfc, r.x, r.y);
            if (s < 0) {  // GRTF:1049-1052, 1102-1108
                if (region == 2) {
                    r.x += T[kTileGap + 0];
                    r.y += T[kTileGap + 1];
                    r.dph += 2 * T[kTileTir + 0];
                } else if (!in_poly(A.loc, w, kPolyEff2, r.x, r.y)) {
                    region = 4;
                } else {
                    r.x += T[kTileGap + 2];
                    r.y += T[kTileGap + 3];
                    r.dph += 2 * T[kTileTir + 1];
                }
                continue;
            }
            blk = 3 + (region - 2) * nfc + s;
            kind = region - 1;
        } else {
            const int s = first_slice(A.loc, w, kPolyFC0 + nfc, noc, r.x, r.y);
            if (s < 0) {  // GRTF:1175-1178, 1244-1246
                if (region == 5) break;
                r.x += T[kTileGap + 2];
                r.y += T[kTileGap + 3];
                r.dph += 2 * T[kTileTir + 1];
                continue;
            }
            blk = 3 + 2 * nfc + (region - 4) * noc + s;
            kind = region - 1;
        }
        region = interact(A, r, T, blocks + kBlock * blk, kind, false, gid, l, m, n, hit);
    }
    A.rng[i] = r.s;
    out.bounces = bounces;
    out.eb_hit = hit;
    return out;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ void add_stats(wgrt_trace_stats *stats, uint64_t bounces, uint64_t hits, uint64_t bad) {
    __shared__ unsigned long long red[3];
    if (threadIdx.x == 0) red[0] = red[1] = red[2] = 0ull;
    __syncthreads();
    bounces = wave_sum(bounces);
    hits = wave_sum(hits);
    bad = wave_sum(bad);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&red[0], (unsigned long long)bounces);
        atomicAdd(&red[1], (unsigned long long)hits);
        atomicAdd(&red[2], (unsigned long long)bad);
    }
    __syncthreads();
    if (threadIdx.x == 0 && stats) {
        atomicAdd((unsigned long long *)&stats->bounces, red[0]);
        atomicAdd((unsigned long long *)&stats->eyebox_hits, red[1]);
        atomicAdd((unsigned long long *)&stats->bad_rays, red[2]);
    }
}

// Variant 1: one ray per lane over a 1-D grid (the reference's launch shape, MAIN:167).
__global__ __launch_bounds__(256) void trace_grid_kernel(TraceArgs A) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t b = 0, h = 0, bad = 0;
    if (i < A.n_rays) {
        const RayOutcome o = trace_one(A, i);
        b = o.bounces;
        h = o.eb_hit;
        bad = o.bad;
        if (A.per_ray) A.per_ray[i] = o.bounces;
    }
    add_stats(A.stats, b, h, bad);
}

__global__ __launch_bounds__(256) void classify_kernel(Locator L, int npoly, const double *xy, int64_t n,
                                                       uint64_t *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = xy[2 * i], y = xy[2 * i + 1];
    const uint64_t w = cell_word(L, x, y);
    uint64_t mask = 0;
    for (int k = 0; k < npoly; ++k)
        if (in_poly(L, w, k, x, y)) mask |= 1ull << k;
    out[i] = mask;
}

__global__ __launch_bounds__(256) void selftest_math_kernel(const double *a, const double *b, int64_t n,
                                                            double *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i], y = b[i];
    out[0 * n + i] = sqrt(x);
    out[1 * n + i] = x / y;
    out[2 * n + i] = hypot_cr(x, y);
    out[3 * n + i] = atan2(x, y);
    double s, c;
    sincos(x, &s, &c);
    out[4 * n + i] = s;
    out[5 * n + i] = c;
    out[6 * n + i] = wrap_pi(x);
}

}  // namespace

struct wgrt_scene {
    int device = 0;
    int nx = 0, ny = 0, nl = 0, nfc = 0, noc = 0, tile_d = 0, npoly = 0;
    double n_g = 0;
    double *d_tiles = nullptr;
    uint64_t *d_cells = nullptr;
    double *d_verts = nullptr;
    int32_t *d_poly_off = nullptr;
    LocatorHost loc_host;  // grid parameters (cells / verts vectors released after upload)
    int64_t tiles = 0;
};

namespace {

Locator make_locator(const wgrt_scene *s) {
    Locator L;
    L.cells = s->d_cells;
    L.verts = s->d_verts;
    L.poly_off = s->d_poly_off;
    L.x0 = s->loc_host.x0;
    L.y0 = s->loc_host.y0;
    L.inv_h = s->loc_host.inv_h;
    L.ncx = s->loc_host.ncx;
    L.ncy = s->loc_host.ncy;
    return L;
}

template <class T>
wgrt_status upload(const std::vector<T> &v, T **dst) {
    const size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(T);
    hipError_t e = hipMalloc((void **)dst, bytes);
    if (e == hipErrorOutOfMemory) return fail(WGRT_ERR_OUT_OF_MEMORY, "hipMalloc: out of memory");
    if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return WGRT_OK;
}

}  // namespace

extern "C" {

wgrt_status wgrt_scene_create(const wgrt_scene_desc *desc, int device, wgrt_scene **out) {
    if (!desc || !out) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL desc / out");
    *out = nullptr;
    SceneHost host;
    try {
        build_scene_host(*desc, 0.25, host);
    } catch (const std::exception &e) {
        return fail(WGRT_ERR_INVALID_ARGUMENT, e.what());
    }
    HIP_TRY(hipSetDevice(device));
    auto *s = new wgrt_scene();
    s->device = device;
    s->nx = desc->nx;
    s->ny = desc->ny;
    s->nl = desc->num_lmd;
    s->nfc = (int)desc->n_fc_slices;
    s->noc = (int)desc->n_oc_slices;
    s->tile_d = host.tile_doubles;
    s->npoly = 3 + s->nfc + s->noc;
    s->n_g = desc->n_g;
    s->tiles = (int64_t)s->nl * s->nx * s->ny;
    wgrt_status st;
    if ((st = upload(host.tiles, &s->d_tiles)) != WGRT_OK || (st = upload(host.loc.cells, &s->d_cells)) != WGRT_OK ||
        (st = upload(host.loc.verts, &s->d_verts)) != WGRT_OK ||
        (st = upload(host.loc.poly_off, &s->d_poly_off)) != WGRT_OK) {
        wgrt_scene_destroy(s);
        return st;
    }
    s->loc_host = host.loc;
    s->loc_host.cells.clear();
    s->loc_host.cells.shrink_to_fit();
    *out = s;
    return WGRT_OK;
}

wgrt_status wgrt_scene_destroy(wgrt_scene *s) {
    if (!s) return WGRT_OK;
    hipSetDevice(s->device);
    hipFree(s->d_tiles);
    hipFree(s->d_cells);
    hipFree(s->d_verts);
    hipFree(s->d_poly_off);
    delete s;
    return WGRT_OK;
}

wgrt_status wgrt_scene_get_info(const wgrt_scene *s, wgrt_scene_info *info) {
    if (!s || !info) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL scene / info");
    info->tile_bytes = (int64_t)s->tile_d * 8;
    info->tiles = s->tiles;
    info->grid_cells_x = s->loc_host.ncx;
    info->grid_cells_y = s->loc_host.ncy;
    info->grid_cell_mm = s->loc_host.h;
    info->grid_edge_cells = s->loc_host.edge_cells;
    info->n_polygons = s->npoly;
    info->device = s->device;
    return WGRT_OK;
}

wgrt_status wgrt_trace_fullcolor_ex(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays,
                                    int64_t gid_offset, uint32_t *rng_states, float *matrix_EB,
                                    wgrt_trace_stats *stats, uint32_t *per_ray_bounces, void *stream,
                                    int variant, int workgroups) {
    if (!s || !rays) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL scene / rays");
    if (n_rays < 0 || gid_offset < 0) return fail(WGRT_ERR_INVALID_ARGUMENT, "negative n_rays / gid_offset");
    if (n_rays == 0) return WGRT_OK;
    if (!rays->x || !rays->y || !rays->m || !rays->n || !rays->lmd_num || !rays->te || !rays->tm ||
        !rays->delta_phase || !rng_states || !matrix_EB)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL ray column / rng_states / matrix_EB");
    if (variant < 0 || variant > 2) return fail(WGRT_ERR_INVALID_ARGUMENT, "unknown kernel variant");
    (void)workgroups;
    TraceArgs A;
    A.x = rays->x;
    A.y = rays->y;
    A.m = rays->m;
    A.n = rays->n;
    A.l = rays->lmd_num;
    A.te = rays->te;
    A.tm = rays->tm;
    A.dph = rays->delta_phase;
    A.rng = rng_states;
    A.eb = matrix_EB;
    A.stats = stats;
    A.per_ray = per_ray_bounces;
    A.n_rays = n_rays;
    A.gid_offset = gid_offset;
    A.tiles = s->d_tiles;
    A.loc = make_locator(s);
    A.tile_d = s->tile_d;
    A.nfc = s->nfc;
    A.noc = s->noc;
    A.nx = s->nx;
    A.ny = s->ny;
    A.nl = s->nl;
    A.n_g = s->n_g;
    hipStream_t st = (hipStream_t)stream;
    const int64_t blocks = (n_rays + 255) / 256;
    if (blocks > 0x7fffffff) return fail(WGRT_ERR_INVALID_ARGUMENT, "too many rays for one launch");
    hipLaunchKernelGGL(trace_grid_kernel, dim3((unsigned)blocks), dim3(256), 0, st, A);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

wgrt_status wgrt_trace_fullcolor(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays,
                                 int64_t gid_offset, uint32_t *rng_states, float *matrix_EB,
                                 wgrt_trace_stats *stats, uint32_t *per_ray_bounces, void *stream) {
    return wgrt_trace_fullcolor_ex(s, rays, n_rays, gid_offset, rng_states, matrix_EB, stats,
                                   per_ray_bounces, stream, 0, 0);
}

wgrt_status wgrt_scene_classify(const wgrt_scene *s, const double *xy, int64_t n, uint64_t *out_mask,
                                void *stream) {
    if (!s || (n > 0 && (!xy || !out_mask))) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n <= 0) return WGRT_OK;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(classify_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       make_locator(s), s->npoly, xy, n, out_mask);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

wgrt_status wgrt_selftest_math(const double *a, const double *b, int64_t n, double *out, void *stream) {
    if (n > 0 && (!a || !b || !out)) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n <= 0) return WGRT_OK;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(selftest_math_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, b,
                       n, out);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

const char *wgrt_status_string(wgrt_status s) {
    switch (s) {
        case WGRT_OK: return "ok";
        case WGRT_ERR_INVALID_ARGUMENT: return "invalid argument";
        case WGRT_ERR_HIP: return "HIP runtime error";
        case WGRT_ERR_OUT_OF_MEMORY: return "out of device memory";
        case WGRT_ERR_UNSUPPORTED: return "unsupported";
    }
    return "unknown status";
}

const char *wgrt_last_error(void) { return g_last_error.c_str(); }

int wgrt_abi_version(void) { return WGRT_ABI_VERSION; }

}  // extern "C"
