// wgrt_device.h -- device-side pieces shared by the bounce kernels (wgrt_trace.hip) and the
// certification shadow (wgrt_shadow.hip): the launch arguments, the exact polygon locator, the
// exact-arithmetic lane and the Jones-vector lane of the reference's per-ray state machine
// (GPU_ray_tracing_functions.py = GRTF:833-1246).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/wgrt.h"
#include "wgrt_common.h"
#include "wgrt_scene_build.h"

namespace wgrt {

// s_waitcnt vmcnt(0) with expcnt / lgkmcnt left at their maxima, in the gfx9 simm16 encoding (vmcnt bits
// 3:0 and 15:14, expcnt 6:4 = 7, lgkmcnt 11:8 = 15): through __builtin_amdgcn_s_waitcnt, so the compiler's
// wait insertion knows that every vector-memory access issued before it has completed
constexpr int kWaitVmcnt0 = 0x0F70;

// ----------------------------------------------------------------------------
// device-side scene view
// ----------------------------------------------------------------------------
// The exact polygon locator (wgrt_scene_build.cpp).  CellT = uint64_t cell words (up to 32
// polygons), uint32_t (up to 16 polygons: half the grid's cache footprint).
template <class CellT>
struct LocatorT {
    using Word = CellT;
    const CellT *cells;
    const double *verts;
    const int32_t *poly_off;
    const int32_t *row_off;
    const int32_t *row_edges;
    double x0, y0, inv_h;
    int ncx, ncy;
    const double *bands;    // 128-B band records (LocatorHost::bands); NULL: CSR lists only
};
using Locator = LocatorT<uint64_t>;

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
    double n_g, inv_n_g;
    double threshold;   // ener * efficiency > threshold guard of R2..R5: 0 full colour, 1e-15 single lambda
    const int32_t *order;   // Jones-vector variants: issue order of the 64-ray chunks (NULL: ascending)
    const double *jtiles;   // Jones-vector tiles (wgrt_common.h kJ*)
    int jtile_d;
    // Jones-vector variants: out-couplings appended as (position, tile index) and binned into
    // matrix_EB by the epilogue kernel after the launch
    double2 *q_xy;
    uint32_t *q_i;
    unsigned long long *q_count;
    double cert_tol;   // Jones-vector variants: base of the double-precision certification bound
    double cert_tol32; // ... and of the single-precision estimate's bound
    unsigned long long *replay_count;   // Jones-vector variants: abandoned rays (local indices)
    uint32_t *replay_list;
    // Jones-vector variants: per-workgroup counter partials {bounces, bad_rays, eyebox_hits, interactions, ...} of
    // the trace kernel, summed into *stats by the epilogue -- no contended atomics on the stats
    unsigned long long *part;
    int n_trace_waves;                  // partial slots of the trace kernel (one per workgroup)
    unsigned long long *heads0;         // this launch's counter set (kScratchCtr words)
    unsigned long long *other_ctr;      // the next launch's counter set, zeroed by this launch's epilogue
    uint32_t *full_list;                // out-coupling queue blocks the trace waves filled (block numbers); with the
                                        // in-kernel epilogue: per block, the link to the block its wave filled before
    unsigned long long *full_count;
    unsigned long long *epi_acc;        // in-kernel epilogue: {bounces, bad_rays, eyebox_hits, interactions} totals ...
    unsigned long long *epi_done;       // ... and the count of trace workgroups that have added theirs
    unsigned long long *timeline;       // debug: per-wave timeline (wgrt_debug_opts), timeline kernels only
    int64_t timeline_waves;
    // fused launches (variants 7 / 9, n_iter > 1): n_iter chained traces of every ray in one
    // launch; rng64[i] = (state << 32) | iter_tag(iter_epoch, traces completed, broken)
    int n_iter;
    uint64_t *rng64;
    uint32_t iter_epoch;
    unsigned long long handoff_wait_ticks;   // fused: s_memrealtime ticks a lane may wait for a hand-off ...
    uint32_t handoff_min_passes;             // ... once its wave has also run this many passes waiting
    // global ray ids of an interleaved shard (wgrt_launch_opts.gid_blocks): NULL = gid_offset + i
    const int64_t *gid_blocks;
    int64_t gid_block_rays;
};

constexpr int kPartWords = 8;   // counter partial slot of a trace workgroup (64-bit words)

// TraceArgs fields re-read from the kernarg segment where they are used (a volatile scalar load,
// a scalar-cache hit) instead of being held in SGPRs for the whole kernel: the Jones loop keeps
// only its per-pass operands in SGPRs; the ray columns and the rare-path pointers (refill,
// retire, replay, out-coupling) are fetched when those run.
//
// KArgs is the handle those reads go through: the base of the kernarg segment as the KERNEL BODY
// saw it.  Only kernel_kargs<Kernel>() makes one, and it refuses to compile unless Kernel's first
// parameter is a TraceArgs (which then lies at offset 0 of the segment).  A function that reads a
// field takes the handle as a parameter, so it reads the right segment whether or not the
// compiler inlines it; __builtin_amdgcn_kernarg_segment_ptr() evaluated inside a called function
// instead reads whatever the caller's registers hold (round 4's out-of-line EDGE build faulted
// with hipErrorIllegalAddress that way).
typedef const char __attribute__((address_space(4))) KSeg;

template <class F>
struct first_param;
template <class A0, class... R>
struct first_param<void(A0, R...)> {
    using type = A0;
};
template <class X, class Y>
struct same_type {
    static constexpr bool value = false;
};
template <class X>
struct same_type<X, X> {
    static constexpr bool value = true;
};

class KArgs {
    KSeg *base_;
    __device__ explicit KArgs(KSeg *b) : base_(b) {}
    template <class Kernel>
    friend __device__ KArgs kernel_kargs();

public:
    template <class T>
    __device__ __forceinline__ T get(size_t off) const {
        return *(volatile const T __attribute__((address_space(4))) *)(base_ + off);
    }
};

// Call in the body of the __global__ function Kernel itself: kernel_kargs<decltype(my_kernel<...>)>().
template <class Kernel>
__device__ __forceinline__ KArgs kernel_kargs() {
    static_assert(same_type<typename first_param<Kernel>::type, TraceArgs>::value,
                  "KArgs reads TraceArgs fields at their offsets in the kernarg segment: the kernel's first "
                  "parameter must be the TraceArgs");
    return KArgs((KSeg *)__builtin_amdgcn_kernarg_segment_ptr());
}

// A TraceArgs field through the handle K in scope.
#define KA(f) K.template get<decltype(TraceArgs::f)>(offsetof(TraceArgs, f))
// the same for the locator's exact-test arrays (TraceArgs::loc holds them for every variant)
#define KLOCP(Kp, f) (Kp)->template get<decltype(Locator::f)>(offsetof(TraceArgs, loc) + offsetof(Locator, f))
#define KLOC(f) KLOCP(&K, f)

// Global id of local ray i (wgrt_launch_opts.gid_blocks): only the zero-state RNG fix-up reads it.
__device__ __forceinline__ int64_t ray_gid(const TraceArgs &A, int64_t i) {
    return A.gid_blocks ? A.gid_blocks[i / A.gid_block_rays] + i % A.gid_block_rays : A.gid_offset + i;
}
// The same from the kernarg segment.
__device__ __forceinline__ int64_t ray_gid_ka(const KArgs &K, int64_t i) {
    const int64_t *gb = KA(gid_blocks);
    if (gb) {
        const int64_t r = KA(gid_block_rays);
        return gb[i / r] + i % r;
    }
    return KA(gid_offset) + i;
}


constexpr int kPolyEff1 = 0;
constexpr int kPolyEff2 = 1;
constexpr int kPolyIC = 2;
constexpr int kPolyFC0 = 3;


// A point's cell of the locator grid: the per-polygon class word and the cell row.
struct Cell {
    uint64_t w;
    int cy;
};

template <class Loc>
__device__ __forceinline__ Cell locate(const Loc &L, double x, double y) {
    const double fx = floor((x - L.x0) * L.inv_h);
    const double fy = floor((y - L.y0) * L.inv_h);
    // NaN / out-of-grid points are outside every polygon (cell word 0 = all OUT)
    if (!(fx >= 0.0 && fy >= 0.0 && fx < (double)L.ncx && fy < (double)L.ncy)) return Cell{0ull, 0};
    const int cx = (int)fx, cy = (int)fy;
    return Cell{(uint64_t)L.cells[cy * L.ncx + cx], cy};
}

// is_inside_or_on_edge(x, y, polygon k) (GRTF:63-71): the cell class when the cell is IN or
// OUT, else the reference predicate over the polygon's edges that meet the cell's row.
template <class Loc>
__device__ __forceinline__ bool in_poly(const Loc &L, const Cell &c, int k, double x, double y) {
    const unsigned cls = (unsigned)(c.w >> (2 * k)) & 3u;
    if (__builtin_expect(cls != 2u, 1)) return cls == 1u;   // IN / OUT; EDGE cells are rare (0.34 % of C3 lane-passes)
    const int a = L.poly_off[k], nv = L.poly_off[k + 1] - a;
    const int r = k * L.ncy + c.cy;
    const int e0 = L.row_off[r], e1 = L.row_off[r + 1];
    return inside_or_on_edge_subset(x, y, L.verts + 2 * a, nv, L.row_edges + e0, e1 - e0);
}

// First slice s in [0, count) of polygons first .. first + count - 1 containing (x, y),
// -1 if none (the slice scans of GRTF:1002-1005 and GRTF:1112-1115, which stop at the
// first hit).  Candidates come straight from the cell word: a slice is tested exactly only
// when its class is EDGE; an IN slice is a hit; OUT slices are skipped.
template <class Loc>
__device__ __forceinline__ int first_slice(const Loc &L, const Cell &c, int first, int count,
                                           double x, double y) {
    uint64_t f = c.w >> (2 * first);
    if (count < 32) f &= (1ull << (2 * count)) - 1ull;
    const uint64_t in = f & 0x5555555555555555ull;           // class 01
    uint64_t cand = in | ((f >> 1) & 0x5555555555555555ull);  // class 01 or 10
    while (cand != 0ull) {
        const int p = __builtin_ctzll(cand);
        const int s = p >> 1;
        if ((in >> p) & 1ull) return s;
        if (in_poly(L, c, first + s, x, y)) return s;
        cand &= cand - 1ull;
    }
    return -1;
}

// Word-only forms for the Jones-vector lane: a cell is just its class word (the row of an
// EDGE cell is recomputed from y on the rare exact test), which keeps prefetched cells in one
// register each.
template <class Loc>
__device__ __forceinline__ typename Loc::Word locate_w(const Loc &L, double x, double y) {
    const double fx = floor((x - L.x0) * L.inv_h);
    const double fy = floor((y - L.y0) * L.inv_h);
    if (!(fx >= 0.0 && fy >= 0.0 && fx < (double)L.ncx && fy < (double)L.ncy)) return 0;
    return L.cells[(int)fy * L.ncx + (int)fx];
}

// The exact test of an EDGE class.  Kp: the launch's kernarg handle -- the locator's array pointers
// are then read from the kernarg segment (not held in SGPRs across the Jones loop); NULL: from L.
template <class Loc>
#ifdef WGRT_EDGE_NOINLINE
__device__ __attribute__((noinline))   // A/B and contract check: the exact tests as a real call
#else
__device__ __forceinline__
#endif
bool in_poly_w(const Loc &L, typename Loc::Word w, int k, double x, double y, const KArgs *Kp = nullptr) {
    const unsigned cls = (unsigned)(w >> (2 * k)) & 3u;
    if (__builtin_expect(cls != 2u, 1)) return cls == 1u;   // IN / OUT; EDGE cells are rare (0.34 % of C3 lane-passes)
    const int cy = (int)floor((y - L.y0) * L.inv_h);   // an EDGE cell is inside the grid
    const int r = k * L.ncy + cy;
    const bool KARG = Kp != nullptr;
    // one 128-B record: the (at most kBandSegs) edges of polygon k meeting this cell row,
    // evaluated with the reference predicate's operations (GRTF:36-71); NaN slots are inert
    const double *const bands = KARG ? KLOCP(Kp, bands) : L.bands;
    const double4 *rec = (const double4 *)(bands + (size_t)r * 4 * kBandSegs);
    const double4 s0 = rec[0], s1 = rec[1], s2 = rec[2], s3 = rec[3];
    if (__builtin_expect(s0.x != INFINITY, 1)) {   // else: a row with more edges than a band record holds
        bool inside = false;
        const double4 sg[kBandSegs] = {s0, s1, s2, s3};
#pragma unroll
        for (int e = 0; e < kBandSegs; ++e) {
            const double xj = sg[e].x, yj = sg[e].y, xi = sg[e].z, yi = sg[e].w;
            if (on_segment(x, y, xj, yj, xi, yi)) return true;
            if (((yi > y) != (yj > y)) && (x < (xj - xi) * (y - yi) / (yj - yi + 1e-20) + xi)) inside = !inside;
        }
        return inside;
    }
    const int32_t *const po = KARG ? KLOCP(Kp, poly_off) : L.poly_off;
    const int32_t *const ro = KARG ? KLOCP(Kp, row_off) : L.row_off;
    const int a = po[k], nv = po[k + 1] - a;
    const int e0 = ro[r], e1 = ro[r + 1];
    return inside_or_on_edge_subset(x, y, (KARG ? KLOCP(Kp, verts) : L.verts) + 2 * a, nv,
                                    (KARG ? KLOCP(Kp, row_edges) : L.row_edges) + e0, e1 - e0);
}

// E_field_cal (GRTF:132-152).  rec = (p, q, r, s) complex in the reference call's argument
// order: Ete' = p*te_in + r*tm_in, Etm' = q*te_in + s*tm_in.  The multiplications by 0.0 are
// Python's real->complex promotions; they are kept so signed zeros propagate exactly.
struct Field {
    double te_re, te_im, tm_re, tm_im;
};

__device__ __forceinline__ Field efield(double Ete, double Etm, double cd, double sd, const double *rec) {
    const double pr = rec[0], pi = rec[1], qr = rec[2], qi = rec[3];
    const double rr = rec[4], ri = rec[5], sr = rec[6], si = rec[7];
    const double ti_re = cd * Etm - sd * 0.0, ti_im = cd * 0.0 + sd * Etm;
    const double a_re = pr * Ete - pi * 0.0, a_im = pr * 0.0 + pi * Ete;
    const double b_re = rr * ti_re - ri * ti_im, b_im = rr * ti_im + ri * ti_re;
    const double c_re = qr * Ete - qi * 0.0, c_im = qr * 0.0 + qi * Ete;
    const double d_re = sr * ti_re - si * ti_im, d_im = sr * ti_im + si * ti_re;
    return Field{a_re + b_re, a_im + b_im, c_re + d_re, c_im + d_im};
}

// |Ete'|^2 + |Etm'|^2 of efield() without the "* 0.0" promotion terms: for finite inputs
// (LUTs are checked at scene creation, ray state stays finite) those terms only change the
// sign of zero components, so every component has the same magnitude as efield()'s and the
// sum of squares is identical.  Used for the branch estimates only.
__device__ __forceinline__ double efield_sq(double Ete, double Etm, double cd, double sd, const double *rec) {
    const double pr = rec[0], pi = rec[1], qr = rec[2], qi = rec[3];
    const double rr = rec[4], ri = rec[5], sr = rec[6], si = rec[7];
    const double ti_re = cd * Etm, ti_im = sd * Etm;
    const double a_re = pr * Ete + (rr * ti_re - ri * ti_im), a_im = pi * Ete + (rr * ti_im + ri * ti_re);
    const double c_re = qr * Ete + (sr * ti_re - si * ti_im), c_im = qi * Ete + (sr * ti_im + si * ti_re);
    return (a_re * a_re + a_im * a_im) + (c_re * c_re + c_im * c_im);
}

// The exact lane carries the ray's delta_phase as the reference does (GRTF:857): a taken branch
// sets it to E_field_cal's wrapped phase difference plus lut_TIR (GRTF:145-150, 877, 926, ...), a
// miss hop adds 2 lut_TIR without a wrap (GRTF:1052, 1108, 1178), and every E_field_cal takes
// cos / sin of the accumulated, unwrapped value (GRTF:135).  The rounding of that accumulation is
// part of the reference's result: with lut_TIR near +-pi and runs of hundreds of hops the phase
// reaches thousands of radians, and a rotation carried as a product of hop phasors instead (round
// 4's lane) drifted from it far enough to change decisions (the adversarial_lossless LUTs of
// tests/test_gpu_certification.py: 33 of 96,768 rays).  This lane differs from the reference only by
// the device's cos / sin / atan2 against glibc's (ulps of the result).
struct Ray {
    double x, y, te, tm, cos_t, ener;
    double dph;   // delta_phase (GRTF:857), unwrapped as the reference carries it
    uint32_t s;
    int region;
};

// One ray in flight on a lane.
struct Lane {
    Ray r;
    const double *T;   // this ray's (lambda, m, n) tile
    int64_t i;         // local ray index
    int l, m, n;
    uint32_t bounces;  // 1 in-coupling event + loop iterations (GRTF:905)
    bool hit;          // accumulated into matrix_EB
    bool libm;         // a guard product ener * e_k fell below 2^-1000 (wgrt_trace_stats.libm_rays)
};

// Load ray i (GRTF:846-859).  Returns false (and leaves the lane empty) for a ray whose
// FoV / wavelength indices fall outside the scene.
__device__ __forceinline__ bool lane_load(const TraceArgs &A, int64_t i, Lane &L) {
    const int64_t ld = i;
    const int m = (int)A.m[ld], n = (int)A.n[ld], l = A.l ? (int)A.l[ld] : 0;
    if (!(m >= 0 && m < A.nx && n >= 0 && n < A.ny && l >= 0 && l < A.nl)) return false;
    L.i = i;
    L.l = l;
    L.m = m;
    L.n = n;
    L.T = A.tiles + (int64_t)((l * A.nx + m) * A.ny + n) * A.tile_d;
    L.r.x = (double)A.x[ld];
    L.r.y = (double)A.y[ld];
    L.r.te = (double)A.te[ld];
    L.r.tm = (double)A.tm[ld];
    L.r.dph = (double)A.dph[ld];
    L.r.cos_t = 1.0;
    L.r.ener = 1.0;
    L.r.s = A.rng[ld];
    L.r.region = 0;
    L.bounces = 1;
    L.hit = false;
    L.libm = false;
    return true;
}

enum : int { kDie = -1, kTransit = -2 };
constexpr int kChunk = 64;   // rays per work-queue chunk of the Jones-vector variants (chunk_order unit)



// A coupler interaction: `blk` of the lane's tile, `kind` 0 in-coupler states (entry event,
// R0, R1), 1 R2, 2 R3, 3 R4, 4 R5.  Evaluates every branch's efficiency (GRTF:860-869,
// 909-918, ..., 1186-1200), draws, and applies the chosen branch.  Returns the next region
// or kDie.  Only the chosen branch's phase (two atan2) is evaluated; its field is recomputed
// by the same operations rather than kept in registers for every branch.
template <class Loc>
__device__ __forceinline__ int interact(const TraceArgs &A, const Loc &loc, Lane &L, int blk, int kind,
                                        bool entry) {
    Ray &r = L.r;
    const double *T = L.T;
    const double *B = T + kTileHeader + kBlock * blk;
    // phase = complex(math.cos(delta), math.sin(delta)) (GRTF:135), once for every E_field_cal call of
    // this interaction (they all take the same delta)
    const double cd = cos(r.dph), sd = sin(r.dph);
    const bool three = kind >= 3;
    const bool thr = kind >= 1;  // the ener > threshold guard exists only in R2..R5
    const double denom = entry ? T[kTileCosIc1] : r.cos_t;
    const double u = rng_draw_lazy(r.s, [&]() { return ray_gid(A, L.i); });

    // Decide the branch.  The reference compares u with cumulative branch efficiencies
    // e_k = (hypot(Ete')^2 + hypot(Etm')^2) * cosA_k / cos(theta) [* or / n_g].  Here the
    // comparisons are first made with cheap estimates (squared moduli instead of the
    // correctly rounded hypot, one reciprocal instead of three divisions), whose relative
    // error is below 1e-14; a decision is accepted only when every threshold it depends on
    // is farther than 1e-12 (relative) from u and no product can underflow, which makes it
    // provably the reference's decision.  Otherwise -- about once in 1e12 draws -- the lane
    // recomputes every e_k exactly as the reference does.  The chosen branch's magnitudes
    // and efficiency are always computed exactly.
    // one branch at a time (a rolled loop keeps the register peak down)
    double q[3] = {0.0, 0.0, 0.0};
    const int nbr = three ? 3 : 2;
#pragma unroll 1
    for (int k = 0; k < nbr; ++k) {
        const double v = efield_sq(r.te, r.tm, cd, sd, B + kBlockRec + 8 * k);
        q[0] = k == 0 ? v : q[0];
        q[1] = k == 1 ? v : q[1];
        q[2] = k == 2 ? v : q[2];
    }
    // 1 / denom to ~1e-16 relative (estimates only): hardware reciprocal + two Newton steps
    double inv = __builtin_amdgcn_rcp(denom);
    inv = fma(inv, fma(-denom, inv, 1.0), inv);
    inv = fma(inv, fma(-denom, inv, 1.0), inv);
    double a0 = q[0] * B[0] * inv, a1 = q[1] * B[1] * inv;
    if (entry) {
        a0 *= A.n_g;
        a1 *= A.n_g;
    }
    const double a2 = three ? q[2] * B[2] * inv * A.inv_n_g : 0.0;
    const double c0 = a0, c1 = a0 + a1, c2 = c1 + a2;
    const double scale = fabs(a0) + fabs(a1) + fabs(a2);   // bounds every partial sum
    const double tol = 1e-12 * scale;
    const bool tiny = thr && !(r.ener > 1e-200 && (a0 == 0.0 || a0 > 1e-100) && (a1 == 0.0 || a1 > 1e-100) &&
                               (!three || a2 == 0.0 || a2 > 1e-100));
    // ener * e_k > threshold (GRTF:606 single-lambda: 1e-15; GRTF:1020 full colour: 0).  With
    // threshold 0 and no underflow it is e_k > 0, i.e. a_k > 0; otherwise the estimate
    // ener * a_k must clear the threshold by a relative margin far above its error.
    const double t = A.threshold;
    const double p0 = r.ener * a0, p1 = r.ener * a1, p2 = r.ener * a2;
    const double tmar = 1e-12 * t;
    const bool tsure = !thr || t == 0.0 ||
                       (fabs(p0 - t) > tmar && fabs(p1 - t) > tmar && (!three || fabs(p2 - t) > tmar));
    const bool pass0 = !thr || (t == 0.0 ? a0 > 0.0 : p0 > t);
    const bool pass1 = !thr || (t == 0.0 ? a1 > 0.0 : p1 > t);
    const bool pass2 = t == 0.0 ? a2 > 0.0 : p2 > t;
    const bool sure = scale > 1e-290 && !tiny && tsure && fabs(u - c0) > tol && fabs(u - c1) > tol &&
                      (!three || fabs(u - c2) > tol);
    int b;
    if (sure) {
        if (u <= c0 && pass0) b = 0;
        else if (u <= c1 && pass1) b = 1;
        else if (three && u <= c2 && pass2) b = 2;
        else return kDie;
    } else {
        double te[3], tm[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            te[k] = tm[k] = 0.0;
            if (k < 2 || three) {
                const Field f = efield(r.te, r.tm, cd, sd, B + kBlockRec + 8 * k);
                te[k] = hypot_cr(f.te_re, f.te_im);
                tm[k] = hypot_cr(f.tm_re, f.tm_im);
            }
        }
        double e0 = (te[0] * te[0] + tm[0] * tm[0]) * B[0] / denom;
        double e1 = (te[1] * te[1] + tm[1] * tm[1]) * B[1] / denom;
        if (entry) {
            e0 = e0 * A.n_g;
            e1 = e1 * A.n_g;
        }
        double e2 = 0.0;
        if (three) e2 = (te[2] * te[2] + tm[2] * tm[2]) * B[2] / denom / A.n_g;
        // the ener-underflow regime: a guard product ener * e_k (GRTF:1020, 1073, 1136,
        // ...) of a nonzero efficiency below 2^-1000, next to the subnormal range, where whether it rounds
        // to zero -- and so the decision -- hangs on the last bits of the libm's cos / sin / atan2.  The
        // certain path above never gets here with such a product (it needs ener > 1e-200 and every
        // nonzero a_k > 1e-100), so checking this path sees every one.
        if (thr)
            L.libm |= ((e0 > 0.0) & (r.ener * e0 < 0x1p-1000)) | ((e1 > 0.0) & (r.ener * e1 < 0x1p-1000)) |
                      (three & (e2 > 0.0) & (r.ener * e2 < 0x1p-1000));
        if (u <= e0 && (!thr || r.ener * e0 > t)) b = 0;
        else if (u <= e0 + e1 && (!thr || r.ener * e1 > t)) b = 1;
        else if (three && u <= e0 + e1 + e2 && r.ener * e2 > t) b = 2;
        else return kDie;
    }

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
            const int64_t off = ((((int64_t)L.l * A.ny + L.n) * A.nx + L.m) * kEbNy + iy) * kEbNx + ix;
            const int64_t total = (int64_t)A.nl * A.ny * A.nx * kEbNy * kEbNx;
            if (off >= 0 && off < total) {
                unsafeAtomicAdd(A.eb + off, 1.0f);
                L.hit = true;
            }
        }
        return kDie;
    }
    const Field f = efield(r.te, r.tm, cd, sd, B + kBlockRec + 8 * b);
    const double cte = hypot_cr(f.te_re, f.te_im);
    const double ctm = hypot_cr(f.tm_re, f.tm_im);
    double e = (cte * cte + ctm * ctm) * B[b] / denom;   // exact e_b (GRTF:868-869, 917-918, ...)
    if (entry) e = e * A.n_g;
    // take the branch (GRTF:872-882 and every branch body after it)
    const double norm = sqrt(cte * cte + ctm * ctm);
    // E_field_cal's output phase (GRTF:145-150): 0 for a component below 1e-20, wrapped difference
    const double pte = cte >= 1e-20 ? atan2(f.te_im, f.te_re) : 0.0;
    const double ptm = ctm >= 1e-20 ? atan2(f.tm_im, f.tm_re) : 0.0;
    int tir, gap;
    if (kind == 0) { tir = b == 0 ? 0 : 2; gap = b == 0 ? 0 : 4; }
    else if (kind <= 2) { tir = b == 0 ? 0 : 1; gap = b == 0 ? 0 : 2; }
    else { tir = b == 0 ? 1 : 3; gap = b == 0 ? 2 : 6; }
    r.cos_t = B[b];
    r.te = cte / norm;
    r.tm = ctm / norm;
    r.dph = wrap_pi(ptm - pte) + T[kTileTir + tir];   // delta_phase = delta_phase_b + lut_TIR[...] (GRTF:877, ...)
    r.x += T[kTileGap + gap];
    r.y += T[kTileGap + gap + 1];
    r.ener = r.ener * e;
    if (kind == 0) {
        const bool in_ic = in_poly(loc, locate(loc, r.x, r.y), kPolyIC, r.x, r.y);
        if (b == 0) return in_ic ? 0 : 2;
        return in_ic ? 1 : kDie;
    }
    if (kind <= 2) return b == 0 ? 2 : 3;
    return b == 0 ? 4 : 5;
}

// Run a ray through the loop iterations that need no Monte-Carlo interaction -- hops that
// miss every coupler slice (GRTF:1049-1052, 1102-1108, 1175-1178) and the R3 -> R4 switch
// -- until the next interaction is due.  Returns that interaction's block index, or kDie
// when the ray terminated (left eff_reg1 at GRTF:906, R5 miss at GRTF:1244-1246, or
// range(1e5) exhausted).  Each iteration counts one bounce.
template <class Loc>
__device__ __forceinline__ int advance(const TraceArgs &A, const Loc &loc, Lane &L, int &kind) {
    Ray &r = L.r;
    const double *T = L.T;
    // A miss hop's step is fixed by the region: R2 moves by gap[0:2] and adds 2*TIR[0],
    // R3 and R4 move by gap[2:4] and add 2*TIR[1] (R5 misses die).  Fetch it once.
    const int g = (r.region == 2) ? 0 : 2;
    const double gx = T[kTileGap + g], gy = T[kTileGap + g + 1];
    const double tir2 = 2 * T[kTileTir + g / 2];   // 2*lut_TIR[...] (exact doubling)
    for (;;) {
        if (L.bounces > (uint32_t)kMaxLoop) return kDie;
        ++L.bounces;
        const Cell c = locate(loc, r.x, r.y);
        if (!in_poly(loc, c, kPolyEff1, r.x, r.y)) return kDie;
        const int region = r.region;
        if (region <= 1) {
            kind = 0;
            return 1 + region;
        }
        int s;
        if (region <= 3) {
            s = first_slice(loc, c, kPolyFC0, A.nfc, r.x, r.y);
            if (s >= 0) {
                kind = region - 1;
                return 3 + (region - 2) * A.nfc + s;
            }
            if (region == 3 && !in_poly(loc, c, kPolyEff2, r.x, r.y)) {
                r.region = 4;   // GRTF:1103-1104: switch to the out-coupler state without moving
                continue;
            }
        } else {
            s = first_slice(loc, c, kPolyFC0 + A.nfc, A.noc, r.x, r.y);
            if (s >= 0) {
                kind = region - 1;
                return 3 + 2 * A.nfc + (region - 4) * A.noc + s;
            }
            if (region == 5) return kDie;
        }
        r.x += gx;
        r.y += gy;
        r.dph += tir2;   // delta_phase += 2*lut_TIR[...] (GRTF:1052, 1108, 1178)
    }
}

// Eyebox accumulation of an out-coupling (GRTF:1162-1171, 1231-1240): the per-FoV
// eyebox rectangle test, the bin, and the atomic; compiled-numba addressing as in interact().
__device__ __forceinline__ bool eyebox_add(const TraceArgs &A, int l, int m, int n, double x, double y) {
    const double *T = A.tiles + (int64_t)((l * A.nx + m) * A.ny + n) * A.tile_d;
    if (!inside_or_on_edge(x, y, T + kTileEbRect, 4)) return false;
    const double xmin = T[kTileEbRange], xmax = T[kTileEbRange + 1];
    const double ymin = T[kTileEbRange + 2], ymax = T[kTileEbRange + 3];
    const double dx = (xmax - xmin) / kEbNx, dy = (ymax - ymin) / kEbNy;
    int64_t ix = (int64_t)floor((x - xmin) / dx);
    int64_t iy = (int64_t)floor((y - ymin) / dy);
    if (ix < 0) ix += kEbNx;
    if (iy < 0) iy += kEbNy;
    const int64_t off = ((((int64_t)l * A.ny + n) * A.nx + m) * kEbNy + iy) * kEbNx + ix;
    const int64_t total = (int64_t)A.nl * A.ny * A.nx * kEbNy * kEbNx;
    if (off < 0 || off >= total) return false;
    unsafeAtomicAdd(A.eb + off, 1.0f);
    return true;
}

// ----------------------------------------------------------------------------
// Jones-vector path (variants 7-9): certified decisions, side-effect-free abandon + replay
// ----------------------------------------------------------------------------
// The reference carries a ray's polarisation as (|Ete|, |Etm|, delta_phase) and re-derives it
// at every taken branch through hypot, atan2 and a wrap (E_field_cal, GRTF:132-152; the
// branch bodies GRTF:872-882, ...).  Up to a global phase that triple is the Jones vector
// E = (|Ete|, |Etm| e^{i delta}): E_field_cal applies a 2x2 complex matrix to it, the branch
// efficiencies are |M E|^2 times a cosine ratio, and taking a branch normalises M E and turns
// its TM component by e^{i lut_TIR} (a miss hop by e^{2 i lut_TIR}).  These variants carry E
// itself -- no hypot, atan2, wrap, sin or cos per interaction, one reciprocal square root for
// the normalisation -- and keep every Monte-Carlo decision the reference's by certifying it:
// a decision is taken only when the draw lies farther from every branch threshold than a bound
// on the difference between this arithmetic and the reference's,
//     tol = D * |1 / cos(theta)| * max(|E|^2, 1) * sum_k W[k]     (W[k]: wgrt_common.h kBlockW),
//     D   = cert_tol * (1 + G (bounces / 100)^2),
// where cert_tol (1e-10) covers the per-step rounding of both evaluations with a wide margin and
// the quadratic term the reference's phase, which grows without a wrap over miss hops (G: the
// tile's max |lut_TIR| / pi).  A ray whose decision cannot be certified (about one in 1e9
// decisions) is abandoned with no side effect -- its RNG state, counters and eyebox cells are
// written only when it terminates -- and re-traced from its launch-start state by the
// reference-arithmetic path (the epilogue kernel).  Positions, hop counts and eyebox indices are the
// reference's exact float64 operations, as in every other variant.
//
// Latency and traffic: a ray's bounces form one dependent chain (cell word -> block -> math ->
// next position).  An interaction loads its block's single-precision part (the TIR step of each
// taken branch is pre-folded into the block's TM rows, wgrt_common.h kJ*), decides, then loads
// the taken branch's double-precision matrix and issues the cell-word load of the new position;
// a miss hop moves the ray, turns Etm by its region's hop phasor (carried in JRay::hr, hi) and
// issues the cell load of its new position.  Either cell word is read in the next pass
// (JLane::pf), so its latency overlaps the rest of the pass and the other waves'.  Out-coupled
// rays are queued (position + ray index) and binned into matrix_EB by the epilogue kernel, so
// the eyebox predicate and its divisions stay out of the wave loop.
struct JRay {
    double x, y;
    double er, ei, mr, mi;   // Jones vector (Ete, Etm), up to a global phase
    double cos_t, ener;
    double eerr;             // relative error bound of ener (threshold > 0 kernels only)
    double gx, gy;           // miss-hop move of the current region
    double hr, hi;           // miss-hop phase step e^{2 i lut_TIR} of the current region, applied at each hop
    float amp;               // bound on the amplification of the lanes' state discrepancy so far (>= 1; §2.4)
    uint32_t s;
    int region;
};

struct JLane {
    JRay r;
    uint32_t tix;            // this ray's (lambda, m, n) tile index (its Jones tile: jtiles + tix * jtile_d)
    uint32_t i;              // local ray index (variants 7 / 9: < 2^32)
    uint32_t bounces;
    uint32_t inter;          // interactions of this trace after the in-coupling event (wgrt_trace_stats.interactions)
    uint32_t k;              // fused launches: the iteration (chained launch) this trace belongs to
    uint32_t s0;             // RNG state at the start of this trace (fused launches: replay point)
    uint64_t pf;             // locator cell word of (x, y), loaded a step ahead
};

enum : int { kUncertain = -3, kOut = -4 };

// Default bases of the certification bounds (wgrt_debug_opts overrides them per call): the
// double-precision evaluation's, and the single-precision estimate's -- 8e-6 covers the rounding
// of |M E|^2 from float matrices and vector (about 26 ulp(1) of the bound's W scale) five times
// over; wgrt_shadow.hip measures the margin.
constexpr double kCertTol = 1e-10;
constexpr double kCertTol32 = 8e-6;


// The Jones-vector lane combines per-lane predicates with & and | on purpose: no short-circuit,
// so the decision is straight-line code instead of nested divergent branches.
#pragma clang diagnostic ignored "-Wbitwise-instead-of-logical"

// Ray columns staged in LDS a work-queue chunk at a time: the wave that dequeues a chunk of
// at most 64 rays copies their nine columns (wgrt_rays order below; lmd_num 0 when absent)
// into its LDS buffer with one direct-to-LDS load per column (lane j <- ray base + j: no
// VGPR destinations, every lane of the wave busy); once they have landed, lane j turns slot j
// into the ray's start state (prep_staged), and the lanes it refills from that chunk later
// read their ray from there.  A refill then costs LDS reads instead of nine per-lane gathers,
// a memory round trip and the start phase's sincos (a refill runs in almost every bulk pass:
// the sincos on the refilled lanes alone was ~15 % of a pass's instructions; per chunk, all
// 64 lanes compute it once).
constexpr int kStageCols = 9;   // x, y, m, n, lmd_num, te, tm, delta_phase, rng
// ... and the prepared slot: x, y, tile index (kBadTix: FoV / wavelength index out of range),
// Etm's real part (lo, hi), te, Etm's imaginary part (lo, hi), rng
constexpr uint32_t kBadTix = 0xffffffffu;
typedef uint32_t __attribute__((address_space(3))) LdsU32;

__device__ __forceinline__ void glds4(const void *g, LdsU32 *dst) {
    __builtin_amdgcn_global_load_lds(g, (void __attribute__((address_space(3))) *)dst, 4, 0, 0);
}

// Issued by the lanes j < n of a wave (exec-masked): column c of ray base + j -> S[c * 64 + j].
__device__ __forceinline__ void stage_chunk(const KArgs &K, LdsU32 *S, int64_t ray) {
    glds4(KA(x) + ray, S + 0 * 64);
    glds4(KA(y) + ray, S + 1 * 64);
    glds4(KA(m) + ray, S + 2 * 64);
    glds4(KA(n) + ray, S + 3 * 64);
    const float *const cl = KA(l);
    if (cl) glds4(cl + ray, S + 4 * 64);
    glds4(KA(te) + ray, S + 5 * 64);
    glds4(KA(tm) + ray, S + 6 * 64);
    glds4(KA(dph) + ray, S + 7 * 64);
    glds4(KA(rng) + ray, S + 8 * 64);
}

// Slot j of a staged chunk (its loads have landed) -> the ray's start state, in place: lane j
// of the wave that dequeued the chunk, for every ray of it at once.
__device__ __forceinline__ void prep_staged(const TraceArgs &A, const KArgs &K, LdsU32 *S, int j) {
    const int m = (int)__uint_as_float(S[2 * 64 + j]), n = (int)__uint_as_float(S[3 * 64 + j]);
    const int l = KA(l) ? (int)__uint_as_float(S[4 * 64 + j]) : 0;
    const float ftm = __uint_as_float(S[6 * 64 + j]), d = __uint_as_float(S[7 * 64 + j]);
    const bool ok = m >= 0 && m < A.nx && n >= 0 && n < A.ny && l >= 0 && l < A.nl;
    const double tm = (double)ftm;
    double sd = 0.0, cd = 1.0;
    if (d != 0.0f) sincos((double)d, &sd, &cd);   // phase = cos + i sin (GRTF:136), exact at 0
    // te_in = Ete, tm_in = phase * Etm (GRTF:137-138)
    const double mr = cd * tm, mi = sd * tm;
    S[2 * 64 + j] = ok ? (uint32_t)((l * A.nx + m) * A.ny + n) : kBadTix;
    S[3 * 64 + j] = (uint32_t)__double_as_longlong(mr);
    S[4 * 64 + j] = (uint32_t)((uint64_t)__double_as_longlong(mr) >> 32);
    S[6 * 64 + j] = (uint32_t)__double_as_longlong(mi);
    S[7 * 64 + j] = (uint32_t)((uint64_t)__double_as_longlong(mi) >> 32);
}

// A lane's ray from slot j of a prepared chunk.  Fused launches pass the ray's hand-off granule
// address: it is loaded with the slot.  False: a bad ray (not traced).
__device__ __forceinline__ bool lane_load_staged(const LdsU32 *S, int j, int64_t i, JLane &L,
                                                 const uint64_t *granule = nullptr, uint64_t *gword = nullptr) {
    const uint32_t tix = S[2 * 64 + j];
    L.i = (uint32_t)i;
    L.tix = tix == kBadTix ? 0u : tix;
    L.r.x = (double)__uint_as_float(S[0 * 64 + j]);
    L.r.y = (double)__uint_as_float(S[1 * 64 + j]);
    L.r.er = (double)__uint_as_float(S[5 * 64 + j]);
    L.r.ei = 0.0;
    L.r.mr = __longlong_as_double((long long)(((uint64_t)S[4 * 64 + j] << 32) | S[3 * 64 + j]));
    L.r.mi = __longlong_as_double((long long)(((uint64_t)S[7 * 64 + j] << 32) | S[6 * 64 + j]));
    L.r.s = S[8 * 64 + j];
    if (granule) *gword = __hip_atomic_load(granule, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    L.r.cos_t = 1.0;
    L.r.ener = 1.0;
    L.r.eerr = 0.0;
    L.r.amp = 1.0f;
    L.r.gx = L.r.gy = 0.0;
    L.r.hr = 1.0;
    L.r.hi = 0.0;
    L.r.region = 0;
    L.bounces = 1;
    L.inter = 0;
    // L.pf is not set: the first pass runs the in-coupling interaction, which loads it (and a
    // write here would wait for the cell loads other lanes' miss hops have in flight)
    return tix != kBadTix;
}

struct JField {
    double er, ei, mr, mi;
};

// Diagnostic segment stamps of a launch-tail pass (tools/segments.py).  Only a build with
// -DWGRT_SEG (an experimental library, never the product) executes any of this: s_memtime at fixed
// points of the pass, each segment's shader cycles summed per wave in scalar registers, and forced
// vmcnt(0) waits at the ends of the two load segments, which separate a load's wait from the arithmetic
// that overlaps it in the real kernel -- so the build's SHARES are read, not its length.
// s[0] advance, s[1] retire / ballots, s[2] line-0 loads + the draw and bound arithmetic until they have
// landed, s[3] estimate + decision, s[4] the taken branch's cell word, hop and matrix until landed,
// s[5] field update, s[6] the rest of the pass (in-coupler test, outcome, out-coupling queue), s[7] passes.
// The sums live in the wave's own LDS words (p[0..7], p[8] = the last stamp), updated by the wave's first
// active lane: a mark inside exec-masked code then still adds to the wave's sums (register sums there
// become per-lane vector values).  32-bit sums of 32-bit differences: a tail is < 2^32 cycles.
struct SegAcc {
    uint32_t __attribute__((address_space(3))) *p;
};
#ifdef WGRT_SEG
__device__ __forceinline__ uint32_t seg_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return (uint32_t)t;
}
#define SEG_WAITVM(sg)                                        \
    do {                                                      \
        if (sg) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    } while (0)
// dep: a value the segment computes; the stamp takes it as an operand, so the compiler cannot sink
// that arithmetic past the stamp (IR passes move arithmetic across an asm statement otherwise)
__device__ __forceinline__ uint32_t seg_stamp_dep(double dep) {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    return (uint32_t)t;
}
__device__ __forceinline__ bool seg_first_lane() {
    return (threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63);
}
#define SEG_MARK_DEP(sg, k, dep)                              \
    do {                                                      \
        if (sg) {                                             \
            const uint32_t t_ = seg_stamp_dep((double)(dep)); \
            if (seg_first_lane()) {                           \
                (sg)->p[k] += t_ - (sg)->p[8];                \
                (sg)->p[8] = t_;                              \
            }                                                 \
        }                                                     \
    } while (0)
#define SEG_MARK(sg, k) SEG_MARK_DEP(sg, k, 0.0)
#if WGRT_SEG == 2
// -DWGRT_SEG=2: wave-uniform marks only (the top level of a pass, jones_body); the interior marks below
// sit in exec-masked code, whose stamps run only when a lane is there and whose sums the compiler merges
// in vector registers
#define SEG_IWAITVM(sg) ((void)0)
#define SEG_IMARK_DEP(sg, k, dep) ((void)0)
#else
#define SEG_IWAITVM(sg) SEG_WAITVM(sg)
#define SEG_IMARK_DEP(sg, k, dep) SEG_MARK_DEP(sg, k, dep)
#endif
#else
#define SEG_IWAITVM(sg) ((void)0)
#define SEG_IMARK_DEP(sg, k, dep) ((void)0)
#define SEG_WAITVM(sg) ((void)0)
#define SEG_MARK(sg, k) ((void)0)
#define SEG_MARK_DEP(sg, k, dep) ((void)0)
#endif

struct Rec {
    double pr, pi, qr, qi, rr, ri, sr, si;
};

__device__ __forceinline__ Rec load_rec(const double *p) {
    const double2 a = *(const double2 *)p, b = *(const double2 *)(p + 2);
    const double2 c = *(const double2 *)(p + 4), d = *(const double2 *)(p + 6);
    return Rec{a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
}

// M E for the coefficients (p, q, r, s) of one E_field_cal call (GRTF:139-144):
// Ete' = p Ete + r Etm, Etm' = q Ete + s Etm.
__device__ __forceinline__ JField jones(const Rec &c, const JRay &r) {
    JField f;
    f.er = fma(c.pr, r.er, fma(-c.pi, r.ei, fma(c.rr, r.mr, -c.ri * r.mi)));
    f.ei = fma(c.pr, r.ei, fma(c.pi, r.er, fma(c.rr, r.mi, c.ri * r.mr)));
    f.mr = fma(c.qr, r.er, fma(-c.qi, r.ei, fma(c.sr, r.mr, -c.si * r.mi)));
    f.mi = fma(c.qr, r.ei, fma(c.qi, r.er, fma(c.sr, r.mi, c.si * r.mr)));
    return f;
}

__device__ __forceinline__ double norm2(const JField &f) {
    return fma(f.er, f.er, fma(f.ei, f.ei, fma(f.mr, f.mr, f.mi * f.mi)));
}

// 1 / d and 1 / sqrt(v) to ~1 ulp: hardware estimate + two Newton steps.
__device__ __forceinline__ double rcp_nr(double d) {
    double y = __builtin_amdgcn_rcp(d);
    y = fma(y, fma(-d, y, 1.0), y);
    return fma(y, fma(-d, y, 1.0), y);
}

__device__ __forceinline__ double rsq_nr(double v) {
    double y = __builtin_amdgcn_rsq(v);
    const double h = 0.5 * v;
    y = y * fma(-h * y, y, 1.5);
    return y * fma(-h * y, y, 1.5);
}

// Cell word of (x, y): the grid has a border of all-OUT cells, so clamping is exact for points
// outside it (and for NaN, which converts to 0).
template <class Loc>
__device__ __forceinline__ typename Loc::Word locate_c(const Loc &L, double x, double y) {
    int ix = (int)((x - L.x0) * L.inv_h), iy = (int)((y - L.y0) * L.inv_h);
    ix = min(max(ix, 0), L.ncx - 1);
    iy = min(max(iy, 0), L.ncy - 1);
    return L.cells[iy * L.ncx + ix];
}

// |M E|^2 in single precision from the block's Hermitian form H = M^H M (the certified estimate
// of a branch efficiency's numerator): h11 |Ete|^2 + h22 |Etm|^2 + 2 Re(h12 conj(Ete) Etm),
// with a = |Ete|^2, b = |Etm|^2, (cr, ci) = conj(Ete) Etm shared by every branch.
__device__ __forceinline__ float herm_form(const float4 &h, float a, float b, float cr, float ci) {
    return fmaf(h.x, a, fmaf(h.y, b, 2.0f * fmaf(h.z, cr, -h.w * ci)));
}

// A Monte-Carlo decision of the Jones-vector lane: the branch efficiencies a_k (estimates of the
// reference's e_k), the draw u, and whether the decision is certified at bound scale `scl`
// (tol = scl * sum_k W[k]; the single-wavelength guard margins use scl * W[k]).
struct JDecision {
    double a0, a1, a2;
    bool ok, s0, s1, s2;
};

__device__ __forceinline__ void jones_decide(JDecision &d, double u, double scl, const double *B, double Wsum,
                                             bool three, bool thr, double t, double ener, double eerr) {
    const double c0 = d.a0, c1 = d.a0 + d.a1, c2 = c1 + d.a2;
    const double tol = scl * Wsum;
    // NaN anywhere fails these comparisons: such a ray is replayed by the reference arithmetic.
    // Non-short-circuit (&, |) throughout: one straight-line evaluation per lane.
    bool ok = (tol > 1e-250) & (fabs(u - c0) > tol) & (fabs(u - c1) > tol) & (!three | (fabs(u - c2) > tol));
    bool p0 = true, p1 = true, p2 = true;
    if (t == 0.0) {   // full colour (uniform branch)
        // a branch the certified draw selects has e_k > tol (it lies between two thresholds more
        // than tol from the draw), so ener * e_k > 0 holds for the reference too unless that
        // product could underflow
        ok = ok & (!thr | (ener * tol > 1e-290));
    } else if (thr) {
        // ener * e_k > threshold (GRTF:606): certified with ener's tracked relative error
        const double g0 = ener * d.a0, g1 = ener * d.a1, g2 = ener * d.a2;
        const double re = eerr + 1e-15;
        const double m0 = re * fabs(g0) + ener * scl * B[kJBlockW] * 1.01;
        const double m1 = re * fabs(g1) + ener * scl * B[kJBlockW + 1] * 1.01;
        const double m2 = re * fabs(g2) + ener * scl * B[kJBlockW + 2] * 1.01;
        p0 = g0 > t;
        p1 = g1 > t;
        p2 = g2 > t;
        ok = ok & ((u > c0) | (fabs(g0 - t) > m0)) & ((u > c1) | (fabs(g1 - t) > m1)) &
             (!three | (u > c2) | (fabs(g2 - t) > m2));
    }
    d.s0 = (u <= c0) & p0;
    d.s1 = !d.s0 & (u <= c1) & p1;
    d.s2 = !d.s0 & !d.s1 & three & (u <= c2) & p2;   // out-coupling (GRTF:1162-1171, 1231-1240)
    d.ok = ok;
}

// A block's {cosA_0, cosA_1, cosA_2, Wsum} for the estimate: cosA_0 and cosA_1 in double (the
// taken branch's efficiency uses them), cosA_2 and Wsum from their floats (the exact cosA_2 is
// read only by the rare double-precision re-evaluation, estimate64).
// The same loads also bring what the tile header would otherwise be loaded for: the phase-growth bound,
// and for block 0 (entry: the in-coupling event) the event's denominator cos(ic1) (kJBlockF32; block 0's
// cosA_2 slot holds the growth bound, and a two-branch block never reads cosA_2).
// Wsum's sign bit flags a block with a branch matrix that is not scaled-unitary (amp_blk: the
// amplification step runs there; wgrt_pack.h).
__device__ __forceinline__ double4 block_cw(const double *B, bool entry, double &growth, double &cos_ic1,
                                            bool &amp_blk) {
    const double2 c01 = *(const double2 *)(B + kJBlockCos);
    const float4 fw = *(const float4 *)(B + kJBlockF32);
    growth = (double)(entry ? fw.y : fw.z);
    cos_ic1 = __hiloint2double(__float_as_int(fw.w), __float_as_int(fw.z));
    amp_blk = __float_as_uint(fw.x) >> 31;
    return double4{c01.x, c01.y, (double)fw.y, (double)fabsf(fw.x)};
}

// The efficiencies from the single-precision Hermitian forms (the estimate every decision starts
// with).  cw = {cosA_0, cosA_1, cosA_2, Wsum}.
__device__ __forceinline__ void estimate32(JDecision &d, const double *B, const JRay &r, bool three, double inv,
                                           double f01, double inv_n_g, const double4 &cw, SegAcc *sg = nullptr,
                                           float4 *h01 = nullptr) {
    const float4 *H = (const float4 *)(B + kJBlockHerm);
    const float4 h0 = H[0], h1 = H[1];
    if (h01) {
        h01[0] = h0;
        h01[1] = h1;
    }
    SEG_IWAITVM(sg);   // (the third branch's form is loaded after the mark: its wait counts in s[3])
    SEG_IMARK_DEP(sg, 2, h0.x + h1.x);
    const float er = (float)r.er, ei = (float)r.ei, mr = (float)r.mr, mi = (float)r.mi;
    const float a = fmaf(er, er, ei * ei), b = fmaf(mr, mr, mi * mi);
    const float cr = fmaf(er, mr, ei * mi), ci = fmaf(er, mi, -ei * mr);
    const double q0 = (double)herm_form(h0, a, b, cr, ci), q1 = (double)herm_form(h1, a, b, cr, ci);
    double q2 = 0.0;
    if (three) q2 = (double)herm_form(H[2], a, b, cr, ci);
    d.a0 = q0 * cw.x * inv * f01;
    d.a1 = q1 * cw.y * inv * f01;
    d.a2 = three ? q2 * cw.z * inv * inv_n_g : 0.0;
}

// The same in double precision, one matrix at a time (the rare re-evaluation of a decision the
// single-precision estimate could not certify; register-light rather than fast).
__device__ __forceinline__ void estimate64(JDecision &d, const double *B, const JRay &r, bool three, double inv,
                                           double f01, double inv_n_g, const double4 &cw) {
    double q[3] = {0.0, 0.0, 0.0};
#pragma unroll 1
    for (int k = 0; k < (three ? 3 : 2); ++k) {
        const double v = norm2(jones(load_rec(B + kJBlockRec + 8 * k), r));
        q[0] = k == 0 ? v : q[0];
        q[1] = k == 1 ? v : q[1];
        q[2] = k == 2 ? v : q[2];
    }
    d.a0 = q[0] * cw.x * inv * f01;
    d.a1 = q[1] * cw.y * inv * f01;
    d.a2 = three ? q[2] * B[kJBlockCos2] * inv * inv_n_g : 0.0;
}

// Amplification of the lanes' state discrepancy ("The bound, stated").  Both lanes apply
// the same Jones matrix M to states that differ, up to a global phase, by a chordal distance eps; after the
// normalisation the distance is at most a eps / (1 - eps / rho) (first order exact: a = |det M| |E|^2 /
// |M E|^2, the stretch of the direction orthogonal to E over that of E; rho = |M E| / (sigma_max |E|)).
// For a scaled-unitary M, a = 1; a singular one contracts (a = 0); a = kappa at worst, for the least
// transmitted polarisation -- the branch the Monte-Carlo draw takes least often.  The Jones lane carries
// A = prod max(1, a_k) (JRay::amp, times 1.006 per step for the second-order term and this evaluation's
// rounding) and scales its certification bound by it; a branch with rho < 1e3 x the discrepancy bound is
// abandoned (kUncertain).  The step runs only in blocks whose branch matrices are not scaled-unitary to
// within kappa^2 <= 1 + 1e-6 (the sign bit of the block's float Wsum, wgrt_pack.h): a unitary branch has
// a <= kappa <= 1 + 5e-7 for every state, so those blocks' factors multiply to at most exp(5e-7 n), 1.05
// at the 1e5-bounce cap, which the bound's margin covers (§2.4).  It lives in the AMP instantiations of
// the trace kernel, which a launch runs when its scene has such a block (wgrt_scene::nonunitary_blocks):
// on scaled-unitary LUTs the kernel carries none of it (compiled into every launch it cost 2-4 %).
// WGRT_AMPLIFY=0 never selects them (the round-5 bound, proven for scaled-unitary matrices only).
#ifndef WGRT_AMPLIFY
#define WGRT_AMPLIFY 1
#endif
constexpr bool kAmplify = WGRT_AMPLIFY != 0;

// |det M|^2 = det H, bounded from above from the tile's single-precision H = M^H M: the float products
// are exact in double and the float entries carry 2^-24 relative rounding, so det H lies within
// 7 2^-24 h11 h22 of this evaluation (|h12|^2 <= h11 h22).
__device__ __forceinline__ double det2_ub(const float4 &h) {
    const double hx = h.x, hy = h.y, hz = h.z, hw = h.w;
    const double d = hx * hy - (hz * hz + hw * hw);
    return fmax(d, 0.0) + 0x1p-21 * (hx * hy);
}

// The decision's half of a taken branch's amplification step, from the branch's H (single precision),
// e2 = |E|^2 and q = the discrepancy bound the decision used (cert_tol (1 + G (n / 100)^2) amp):
// pa = |det M|^2 |E|^4 (so a^2 = pa / |M E|^4), and nmin = 1e6 q^2 trace(H) |E|^2, the least |M E|^2 with
// rho >= 1e3 q (sigma_max^2 <= trace H); both rounded up into floats.
__device__ __forceinline__ void amp_prepare(const float4 &hb, double e2, double q, float &pa, float &nmin) {
    pa = (float)(det2_ub(hb) * e2 * e2 * (1.0 + 0x1p-20));
    nmin = (float)(1e6 * q * q * ((double)hb.x + (double)hb.y) * e2 * (1.0 + 0x1p-20));
}

// The take's half: amp times max(1, a) (rn = 1 / |M E| to ~1 ulp), or a negative value when |M E|^2 = n2
// is below nmin (the first-order step is not certain there: the ray is abandoned).
__device__ __forceinline__ float amp_step(float amp, float pa, float nmin, double n2, double rn) {
    const double r2 = rn * rn;
    const double a2 = (double)pa * r2 * r2;
    float out = amp;
    if (__builtin_expect(a2 > 1.0, 0)) out = (float)((double)amp * sqrt(a2) * 1.006);
    return n2 < (double)nmin ? -1.0f : out;
}

// Same contract as interact() (GRTF:860-904 and the branch bodies of GRTF:905-1246), plus
// kUncertain: the decision could not be certified; the lane's ray must be abandoned (nothing
// of it has been written) and replayed.
//
// A decision is first taken from single-precision efficiencies, certified against the bound
// scaled by A.cert_tol32 (which covers single-precision rounding of |M E|^2 with a wide margin,
// wgrt_shadow.hip measures it); the rare decision that bound leaves open is re-evaluated in
// double precision against the A.cert_tol bound, and only if that fails too is the ray
// abandoned.  The taken branch's field is always computed in double precision from its
// double-precision matrix (loaded after the decision), so the carried Jones vector and ener
// are the same values the all-double evaluation gives.
template <bool SINGLE, bool AMP, class Loc>
__device__ __forceinline__ int interact(const TraceArgs &A, const KArgs &K, const Loc &loc, JLane &L, int blk,
                                        int kind, bool entry, SegAcc *sg = nullptr) {
    JRay &r = L.r;
    const double *T = KA(jtiles) + (size_t)L.tix * (size_t)A.jtile_d;
    const double *B = T + kJHeader + kJBlock * blk;
    const bool three = kind >= 3;
    const bool thr = kind >= 1;   // the ener > threshold guard exists only in R2..R5
    const double t = SINGLE ? A.threshold : 0.0;
    // the moves of branch a (index 0) and b (index 1) of this state (GRTF:878, 894, 1027, 1040,
    // 1134, 1147, ...); each is also the miss hop of the region it leads to (R5 never hops)
    const int ga = kind >= 3 ? 2 : 0;
    const int gb = kind == 0 ? 4 : (kind >= 3 ? 6 : 2);
    double growth, cos_ic1;
    bool amp_blk;
    const double4 cw = block_cw(B, entry, growth, cos_ic1, amp_blk);
    // both branches' moves with the estimate's loads: the taken branch's new cell word can then be
    // issued together with its matrix, one memory round trip per interaction less
    const double2 mva = *(const double2 *)(T + kJGap + ga);
    const double2 mvb = *(const double2 *)(T + kJGap + gb);
    const double denom = entry ? cos_ic1 : r.cos_t;
    const double u = rng_draw_lazy(r.s, [&]() { return ray_gid_ka(K, (int64_t)L.i); });
    const double inv = rcp_nr(denom);
    const double f01 = entry ? A.n_g : 1.0;
    const double nb = (double)L.bounces * 0.01;
    const double e2 = fma(r.er, r.er, fma(r.ei, r.ei, fma(r.mr, r.mr, r.mi * r.mi)));
    const double grow = AMP ? fma(nb * nb, growth, 1.0) * (double)r.amp : fma(nb * nb, growth, 1.0);
    const double base = grow * fabs(inv) * fmax(e2, 1.0);
    JDecision d;
    estimate32(d, B, r, three, inv, f01, A.inv_n_g, cw, sg);
    jones_decide(d, u, A.cert_tol32 * base, B, cw.w, three, thr, t, r.ener, SINGLE ? r.eerr : 0.0);
    if (__builtin_expect(!d.ok, 0)) {   // rare: the double-precision evaluation
        estimate64(d, B, r, three, inv, f01, A.inv_n_g, cw);
        jones_decide(d, u, A.cert_tol * base, B, cw.w, three, thr, t, r.ener, SINGLE ? r.eerr : 0.0);
    }
    SEG_IMARK_DEP(sg, 3, d.a0 + d.a1 + d.a2 + (d.ok ? 1.0 : 0.0) + (d.s0 ? 2.0 : 0.0) + (d.s1 ? 4.0 : 0.0));
    // one exit for every outcome but a taken branch; an out-coupling is appended to the
    // out-coupling queue by the caller (at (r.x, r.y))
    const int code = !d.ok ? kUncertain : d.s2 ? kOut : !(d.s0 | d.s1) ? kDie : 0;
    if (code != 0) return code;
    const bool ba = d.s0;
    const int b = ba ? 0 : 1;
    // the taken branch's new position and its cell word (read by the next pass's advance(); kind
    // 0: below), issued together with the load of its double-precision matrix.  Only the taken
    // branch's cell word: loading both candidates' before the decision hid no more latency and
    // doubled the cell-word gathers (random 4-B reads of a 71 MB grid): 9-12 % slower on C3
    const double2 mv = ba ? mva : mvb;
    r.x = r.x + mv.x;
    r.y = r.y + mv.y;
    L.pf = locate_c(loc, r.x, r.y);
    // the phase step of the new region's miss hops (R2: 2 lut_TIR[0]; R3, R4: 2 lut_TIR[1]; the
    // in-coupler states and R5 never hop), loaded with the taken branch's matrix
    const double2 hop = *(const double2 *)(T + kJHop + ((kind == 0 || (kind <= 2 && ba)) ? 0 : 2));
#ifdef WGRT_SEG
    const Rec rec_b = load_rec(B + kJBlockRec + 8 * b);
    SEG_IWAITVM(sg);
    SEG_IMARK_DEP(sg, 4, rec_b.pr + rec_b.si + hop.x);
    const JField f = jones(rec_b, r);
#else
    const JField f = jones(load_rec(B + kJBlockRec + 8 * b), r);
#endif
    // Ete = Ete1 / norm, Etm = Etm1 / norm (GRTF:874-876); the TIR step is in the TM row
    const double n2 = norm2(f);
    if (!(n2 > 1e-300)) return kUncertain;
    const double rn = rsq_nr(n2);
    if (AMP && __builtin_expect(amp_blk, 0)) {
        // a non-unitary branch matrix: the amplification step (its inputs re-read here, off the common path)
        const float4 hb = ((const float4 *)(B + kJBlockHerm))[b];
        const double e2b = fma(r.er, r.er, fma(r.ei, r.ei, fma(r.mr, r.mr, r.mi * r.mi)));
        float pa, nmin;
        amp_prepare(hb, e2b, A.cert_tol * grow, pa, nmin);
        const float a = amp_step(r.amp, pa, nmin, n2, rn);
        if (a < 0.0f) return kUncertain;
        r.amp = a;
    }
    r.er = f.er * rn;
    r.ei = f.ei * rn;
    r.mr = f.mr * rn;
    r.mi = f.mi * rn;
    const double ab = n2 * (ba ? cw.x : cw.y) * inv * f01;   // the taken branch's efficiency, double precision
    // ener accumulates every taken branch's relative error, the in-coupler states' too (no guard there,
    // but their factors are part of ener at every later guard)
    if (SINGLE) r.eerr += A.cert_tol * base * B[kJBlockW + b] * 1.01 * rcp_nr(ab) + 1e-15;
    r.ener = r.ener * ab;
    r.cos_t = ba ? cw.x : cw.y;
    r.gx = mv.x;
    r.gy = mv.y;
    r.hr = hop.x;
    r.hi = hop.y;
    SEG_IMARK_DEP(sg, 5, r.er + r.ei + r.mr + r.mi + r.ener);
    if (kind == 0) {
        const bool in_ic = in_poly_w(loc, (typename Loc::Word)L.pf, kPolyIC, r.x, r.y, &K);
        if (ba) return in_ic ? 0 : 2;
        return in_ic ? 1 : kDie;
    }
    if (kind <= 2) return ba ? 2 : 3;
    return ba ? 4 : 5;
}

// The EDGE classes a lane's loop iteration consults -- eff_reg1's, the region's slices' up to the
// first IN one, eff_reg2's in R3 -- replaced by the exact predicate's verdict (IN 1 / OUT 0) through
// the 128-B band records (in_poly_w).  Rare: 0.34 % of C3 lane-passes meet an EDGE cell.
#ifndef WGRT_EDGE_WAIT
#define WGRT_EDGE_WAIT 1
#endif
template <class Loc>
__device__ __forceinline__ typename Loc::Word resolve_edges(const KArgs &K, const Loc &loc, typename Loc::Word w,
                                                            int region, int first, int count, double x, double y) {
    using W = typename Loc::Word;
    auto fix = [&](int k) {
        if (((w >> (2 * k)) & 3u) == 2u) {
            const bool in = in_poly_w(loc, w, k, x, y, &K);
            w = (W)((w & ~((W)3 << (2 * k))) | ((W)(in ? 1u : 0u) << (2 * k)));
        }
    };
    fix(kPolyEff1);
    if (region >= 2) {
        for (int sl = 0; sl < count; ++sl) {
            fix(first + sl);
            if (((w >> (2 * (first + sl))) & 3u) == 1u) break;
        }
        if (region == 3) fix(kPolyEff2);
    }
    return w;
}

// lowest set bit of a cell word (undefined for 0: callers guard)
__device__ __forceinline__ int low_bit(uint32_t v) { return __builtin_ctz(v); }
__device__ __forceinline__ int low_bit(uint64_t v) { return __builtin_ctzll(v); }

// Same contract as advance() for the Jones-vector lane: one loop iteration of GRTF:905-1246 that
// needs no Monte-Carlo interaction (a miss hop or the R3 -> R4 switch: kTransit), or the next
// interaction's block index, or kDie.  It tests the cell word loaded a pass earlier (JLane::pf);
// a miss hop issues the load of the next one.  The outcome is computed as selects from the cell
// word's class bits (in the word's own width: 32 bits for variant 7) -- one straight-line
// evaluation per lane -- and only lanes whose outcome hinges on an EDGE class take the (rare)
// exact path first: the earlier nested per-slice tests cost every wave-pass the exec-mask
// bookkeeping of every slice's exact test (SALU per bounce).
template <class Loc>
__device__ __forceinline__ int advance(const TraceArgs &A, const KArgs &K, const Loc &loc, JLane &L, int &kind) {
    using W = typename Loc::Word;
    constexpr int kBits = 8 * (int)sizeof(W);
    constexpr W kLow = (W)0x5555555555555555ull;
    constexpr W kTop = (W)1 << (kBits - 1);
    JRay &r = L.r;
    W c = (W)L.pf;
    const int region = r.region;
    const int nfc = A.nfc, noc = A.noc;
    // the coupler slices this region scans (GRTF:1002-1005, 1112-1115) and its blocks
    const bool fc = region <= 3;
    const int first = fc ? kPolyFC0 : kPolyFC0 + nfc, count = fc ? nfc : noc;
    const W gmask = 2 * count < kBits ? ((W)1 << (2 * count)) - (W)1 : (W)~(W)0;
    W f = (c >> (2 * first)) & gmask;
    W in = f & kLow, cand = in | ((f >> 1) & kLow);
    const bool e1edge = ((c >> (2 * kPolyEff1)) & 3u) == 2u;
    const bool sedge = region >= 2 && cand != 0 && !((in >> low_bit((W)(cand | kTop))) & 1u);
    const bool e2edge = region == 3 && cand == 0 && ((c >> (2 * kPolyEff2)) & 3u) == 2u;
    if (__builtin_expect(e1edge | sedge | e2edge, 0)) {
        c = resolve_edges(K, loc, c, region, first, count, r.x, r.y);
        // the band records' loads have all landed (a compiler-visible vmcnt(0), gfx9 encoding): an exit of the
        // exact test that leaves some in flight would otherwise make the wait insertion assume them pending
        // on every path after this rare one, and wait for every load in flight before the interaction's
        // line-0 loads -- the pass's miss-hop gathers among them
#if WGRT_EDGE_WAIT
        __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
#endif
        f = (c >> (2 * first)) & gmask;
        in = f & kLow;
        cand = in | ((f >> 1) & kLow);
    }
    const bool over = L.bounces > (uint32_t)kMaxLoop;   // range(1e5) exhausted (GRTF:905)
    const bool eff1 = ((c >> (2 * kPolyEff1)) & 3u) == 1u;   // GRTF:906
    const bool eff2 = ((c >> (2 * kPolyEff2)) & 3u) == 1u;
    const bool ic = region <= 1;
    const bool hit = !ic & (cand != 0);
    const int sl = low_bit((W)(cand | kTop)) >> 1;
    const bool die = over | !eff1 | (!ic & !hit & (region == 5));           // GRTF:1244-1246
    const bool sw = !die & !ic & !hit & (region == 3) & !eff2;              // GRTF:1103-1104: R3 -> R4, no move
    const bool hop = !die & !ic & !hit & !sw;                               // miss hop
    // the region's first block: FC regions 2-3 follow the 3 in-coupler states, OC regions 4-5 both FC
    // regions (one multiply of selected operands: no divergent branch)
    const int blkbase = 3 + (fc ? 0 : 2 * nfc) + (region - (fc ? 2 : 4)) * count;
    L.bounces += over ? 0u : 1u;
    kind = ic ? 0 : region - 1;
    r.region = sw ? 4 : region;
    if (hop) {
        // miss hop (GRTF:1049-1052, 1105-1108, 1175-1178)
        r.x = r.x + r.gx;
        r.y = r.y + r.gy;
        // delta_phase += 2 lut_TIR (GRTF:1052, 1108, 1178) as a turn of Etm at the hop itself: a
        // deferred per-interaction loop ran max(hops) iterations over a wave's lanes (+3 % single
        // launch, +5 % fused on C3, +10 % on C5's short hops)
        const double mr = r.mr;
        r.mr = fma(mr, r.hr, -r.mi * r.hi);
        r.mi = fma(mr, r.hi, r.mi * r.hr);
        L.pf = locate_c(loc, r.x, r.y);   // read by the next pass
    }
    const int step = hit ? blkbase + sl : kTransit;
    const int next = ic ? 1 + region : step;
    return die ? kDie : next;
}

template <class LaneT>
__device__ __forceinline__ void lane_retire(const TraceArgs &A, const LaneT &L) {
    A.rng[L.i] = L.r.s;
    if (A.per_ray) A.per_ray[L.i] = L.bounces;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Per-wave reduction of the ray counters, then one 64-bit atomic per counter per wave.
__device__ __forceinline__ void add_stats(wgrt_trace_stats *stats, uint64_t bounces, uint64_t hits,
                                          uint64_t bad, uint64_t inter, uint64_t libm = 0) {
    bounces = wave_sum(bounces);
    hits = wave_sum(hits);
    bad = wave_sum(bad);
    inter = wave_sum(inter);
    libm = wave_sum(libm);
    if ((threadIdx.x & 63) == 0 && stats) {
        if (libm) atomicAdd((unsigned long long *)&stats->libm_rays, (unsigned long long)libm);
        if (inter) atomicAdd((unsigned long long *)&stats->interactions, (unsigned long long)inter);
        if (bounces) atomicAdd((unsigned long long *)&stats->bounces, (unsigned long long)bounces);
        if (hits) atomicAdd((unsigned long long *)&stats->eyebox_hits, (unsigned long long)hits);
        if (bad) atomicAdd((unsigned long long *)&stats->bad_rays, (unsigned long long)bad);
    }
}

// Trace ray i to termination with the reference arithmetic (variant 1's lane; replays).  With
// s_io, the trace starts from *s_io instead of rng_states[i] and leaves its final state there
// (rng_states untouched).  ni (optional) counts the interactions after the in-coupling event.
__device__ __forceinline__ void trace_one(const TraceArgs &A, int64_t i, uint64_t &b, uint64_t &h, uint64_t &bad,
                                          uint32_t *s_io = nullptr, uint64_t *ni = nullptr, uint64_t *lm = nullptr) {
    Lane L;
    if (!lane_load(A, i, L)) {
        ++bad;
        return;
    }
    if (s_io) L.r.s = *s_io;
    int blk = 0, kind = 0;
    bool entry = true;
    for (;;) {
        const int next = interact(A, A.loc, L, blk, kind, entry);
        if (next < 0) break;
        L.r.region = next;
        entry = false;
        blk = advance(A, A.loc, L, kind);
        if (blk < 0) break;
        if (ni) ++*ni;
    }
    if (s_io) *s_io = L.r.s;
    else lane_retire(A, L);
    b += L.bounces;
    h += L.hit;
    if (lm) *lm += L.libm ? 1u : 0u;
}

}  // namespace wgrt
