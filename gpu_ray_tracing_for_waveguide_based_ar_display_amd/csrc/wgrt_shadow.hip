// wgrt_shadow.hip -- certification shadow of the Jones-vector lane (diagnostic entry point
// wgrt_debug_shadow, include/wgrt.h).
//
// The Jones-vector kernels (variants 7 / 9) take a Monte-Carlo decision only when the draw lies
// farther than a bound `tol` from every branch threshold (wgrt_device.h, "Jones-vector path").
// This kernel measures how much of that bound the arithmetic actually uses.  One lane per ray
// traces the ray with the reference's own arithmetic, literally (GPU_ray_tracing_functions.py =
// GRTF):
//   * E_field_cal (GRTF:132-152): phase = cos / sin of the UNWRAPPED delta_phase, the Jones
//     products with Python's real->complex promotions, correctly rounded hypot, atan2 of both
//     components (0 below 1e-20), wrap to [-pi, pi);
//   * a taken branch sets delta_phase = phase + lut_TIR[k] (GRTF:877, 926, ...), a miss hop adds
//     2 * lut_TIR[k] without a wrap (GRTF:1052, 1108, 1178), so |delta_phase| grows with depth;
//   * the branch efficiencies and their cumulative thresholds in the reference's expression
//     order (GRTF:868-869, 917-918, ..., 1196-1200), the draw (GRTF:25-34) and the decision.
// Alongside, the lane carries the Jones-vector state exactly as the product lane does (the
// block's Jones matrices with the TIR step folded in, miss-hop phase steps applied as a power at
// the next interaction, rsq normalisation) and, at every decision, evaluates the product lane's
// thresholds c_k^J and its bounds tol -- for its single-precision estimate (tol32, the bound
// every decision is first certified against) and its double-precision re-evaluation (tol64).
// It records
//     ratio = max_k |c_k^J - c_k^ref| / tol
// for both (max overall; for tol32 also by bounce depth and as a log10 histogram), the decisions
// the single-precision estimate leaves to the double-precision one (fallbacks), the decisions
// the product lane would leave uncertain (replayed), and "silent flips": decisions the product
// lane would certify although they differ from the reference's -- which must never happen.  The ray always
// follows the reference's decision, so its final RNG state and bounce count are the reference's
// (tests compare them with the CPU oracle).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "../../include/wgrt.h"
#include "../../include/wgrt_debug.h"
#include "wgrt_common.h"
#include "wgrt_device.h"
#include "wgrt_scene.h"

using namespace wgrt;

namespace {

constexpr int kDepthBuckets = 6;   // bounce depth [1,10) [10,30) [30,100) [100,300) [300,1000) [1000,inf)
constexpr int kHistBuckets = 20;   // log10 ratio: bucket b = [1e(b-18), 1e(b-17)); 0 also below, 19 also above

struct ShadowArgs {
    TraceArgs A;
    wgrt_shadow_stats *out;
};

__device__ __forceinline__ int depth_bucket(uint32_t b) {
    return b < 10 ? 0 : b < 30 ? 1 : b < 100 ? 2 : b < 300 ? 3 : b < 1000 ? 4 : 5;
}

__device__ __forceinline__ int hist_bucket(double r) {
    if (!(r > 0.0)) return 0;
    const int b = (int)floor(log10(r)) + 18;
    return b < 0 ? 0 : (b >= kHistBuckets ? kHistBuckets - 1 : b);
}

__device__ __forceinline__ void atomic_max_pos(double *p, double v) {
    if (v > 0.0) atomicMax((unsigned long long *)p, (unsigned long long)__double_as_longlong(v));
}

// Per-lane accumulators, flushed once per lane at the end.
struct ShadowAcc {
    uint64_t decisions = 0, uncertain = 0, flips = 0, bounces = 0, fallbacks = 0;
    double max_ratio = 0.0, max_ratio32 = 0.0, max_ener = 0.0, max_amp = 1.0;
    double max_depth[kDepthBuckets] = {0, 0, 0, 0, 0, 0};
    uint64_t n_depth[kDepthBuckets] = {0, 0, 0, 0, 0, 0};
    uint64_t hist[kHistBuckets] = {};
};

// E_field_cal's magnitudes and wrapped phase difference (GRTF:132-152), literal.
struct RefField {
    double te, tm, dphi;
};

__device__ __forceinline__ RefField ref_efield(double Ete, double Etm, double dph, const double *rec) {
    const double cd = cos(dph), sd = sin(dph);
    const Field f = efield(Ete, Etm, cd, sd, rec);   // Python-promotion complex products (wgrt_device.h)
    RefField o;
    o.te = hypot_cr(f.te_re, f.te_im);
    o.tm = hypot_cr(f.tm_re, f.tm_im);
    const double pte = (o.te >= 1e-20) ? atan2(f.te_im, f.te_re) : 0.0;
    const double ptm = (o.tm >= 1e-20) ? atan2(f.tm_im, f.tm_re) : 0.0;
    o.dphi = wrap_pi(ptm - pte);
    return o;
}

template <class Loc>
__device__ void shadow_trace(const TraceArgs &A, const Loc &loc, int64_t i, ShadowAcc &acc) {
    // ---- load (GRTF:842-859) ----
    const int m = (int)A.m[i], n = (int)A.n[i], l = A.l ? (int)A.l[i] : 0;
    if (!(m >= 0 && m < A.nx && n >= 0 && n < A.ny && l >= 0 && l < A.nl)) return;
    const int64_t g = (int64_t)((l * A.nx + m) * A.ny + n);
    const double *T = A.tiles + g * A.tile_d;     // exact tile (reference arithmetic)
    const double *J = A.jtiles + g * A.jtile_d;   // Jones tile (product lane)
    const int64_t gid = A.gid_offset + i;
    double x = (double)A.x[i], y = (double)A.y[i];
    double Ete = (double)A.te[i], Etm = (double)A.tm[i], dph = (double)A.dph[i];
    double cos_th = 1.0, ener = 1.0;
    uint32_t s = A.rng[i];
    uint32_t bounces = 1;
    int region = 0;
    // Jones-vector state (te_in = Ete, tm_in = phase * Etm, GRTF:136-138)
    JRay jr{};
    {
        double sd = 0.0, cd = 1.0;
        if (A.dph[i] != 0.0f) sincos(dph, &sd, &cd);
        jr.er = Ete;
        jr.ei = 0.0;
        jr.mr = cd * Etm;
        jr.mi = sd * Etm;
        jr.amp = 1.0f;
    }
    double jener = 1.0, eerr = 0.0;
    uint32_t hops = 0;
    const double t = A.threshold;
    int blk = 0, kind = 0;
    bool entry = true;
    for (;;) {
        // ---- one interaction: block blk of state `kind` ----
        const double *B = T + kTileHeader + kBlock * blk;
        const double *JB = J + kJHeader + kJBlock * blk;
        const bool three = kind >= 3, thr = kind >= 1;
        const double denom = entry ? T[kTileCosIc1] : cos_th;
        RefField E[3];
        E[2] = RefField{0.0, 0.0, 0.0};
        for (int k = 0; k < (three ? 3 : 2); ++k) E[k] = ref_efield(Ete, Etm, dph, B + kBlockRec + 8 * k);
        double e0 = (E[0].te * E[0].te + E[0].tm * E[0].tm) * B[0] / denom;
        double e1 = (E[1].te * E[1].te + E[1].tm * E[1].tm) * B[1] / denom;
        if (entry) {
            e0 = e0 * A.n_g;
            e1 = e1 * A.n_g;
        }
        const double e2 = three ? (E[2].te * E[2].te + E[2].tm * E[2].tm) * B[2] / denom / A.n_g : 0.0;
        const double u = rng_draw(s, gid);
        int b;   // the reference's decision: 0, 1, 2 (out-coupling) or -1 (dies)
        if (u <= e0 && (!thr || ener * e0 > t)) b = 0;
        else if (u <= e0 + e1 && (!thr || ener * e1 > t)) b = 1;
        else if (three && u <= e0 + e1 + e2 && ener * e2 > t) b = 2;
        else b = -1;

        // ---- the product lane's view of the same decision (wgrt_device.h Jones interact) ----
        {
            const double2 hp = *(const double2 *)(J + kJHop + (region == 2 ? 0 : 2));
            for (uint32_t h = 0; h < hops; ++h) {
                const double mr = jr.mr;
                jr.mr = fma(mr, hp.x, -jr.mi * hp.y);
                jr.mi = fma(mr, hp.y, jr.mi * hp.x);
            }
            hops = 0;
            double growth, cos_ic1;
            bool amp_blk;
            const double4 cw = block_cw(JB, entry, growth, cos_ic1, amp_blk);
            const double jden = entry ? cos_ic1 : cos_th;
            const double inv = rcp_nr(jden);
            const double f01 = entry ? A.n_g : 1.0;
            const double nb = (double)bounces * 0.01;
            const double en2 = fma(jr.er, jr.er, fma(jr.ei, jr.ei, fma(jr.mr, jr.mr, jr.mi * jr.mi)));
            const double grow = kAmplify ? fma(nb * nb, growth, 1.0) * (double)jr.amp : fma(nb * nb, growth, 1.0);
            const double base = grow * fabs(inv) * fmax(en2, 1.0);
            const double c_ref[3] = {e0, e0 + e1, e0 + e1 + e2};
            // how much of each bound the arithmetic uses against the reference's thresholds
            auto ratio = [&](const JDecision &d, double scl) {
                const double tol = scl * cw.w;
                if (!(tol > 1e-250)) return 0.0;
                const double c0 = d.a0, c1 = d.a0 + d.a1, c2 = c1 + d.a2;
                const double r0 = fabs(c0 - c_ref[0]) / tol, r1 = fabs(c1 - c_ref[1]) / tol;
                const double r2 = three ? fabs(c2 - c_ref[2]) / tol : 0.0;
                return fmax(r0, fmax(r1, r2));
            };
            JDecision d32, d64;
            estimate32(d32, JB, jr, three, inv, f01, A.inv_n_g, cw);
            jones_decide(d32, u, A.cert_tol32 * base, JB, cw.w, three, thr, t, jener, eerr);
            estimate64(d64, JB, jr, three, inv, f01, A.inv_n_g, cw);
            jones_decide(d64, u, A.cert_tol * base, JB, cw.w, three, thr, t, jener, eerr);
            const double r32 = ratio(d32, A.cert_tol32 * base), r64 = ratio(d64, A.cert_tol * base);
            if (thr && t != 0.0) {   // the ener guard's tracked relative error against the reference's ener
                const double er = fabs(jener / ener - 1.0) / (eerr + 1e-15);
                acc.max_ener = fmax(acc.max_ener, er);
            }
            // the product lane's decision: the single-precision one, else the double-precision one
            const JDecision &dd = d32.ok ? d32 : d64;
            const int bj = dd.s0 ? 0 : dd.s1 ? 1 : dd.s2 ? 2 : -1;
            ++acc.decisions;
            if (!d32.ok) ++acc.fallbacks;
            if (!dd.ok) ++acc.uncertain;
            else if (bj != b) ++acc.flips;
            acc.max_ratio = fmax(acc.max_ratio, r64);
            acc.max_ratio32 = fmax(acc.max_ratio32, r32);
            const int db = depth_bucket(bounces);
            acc.max_depth[db] = fmax(acc.max_depth[db], r32);
            ++acc.n_depth[db];
            ++acc.hist[hist_bucket(r32)];
            // the product lane's state follows the reference's branch (its double-precision take)
            if (b == 0 || b == 1) {
                const JField f = jones(load_rec(JB + kJBlockRec + 8 * b), jr);
                const double n2 = norm2(f);
                const double rn = rsq_nr(n2);
                if (kAmplify && amp_blk) {   // the product lane's amplification step (wgrt_device.h interact)
                    const float4 hb = ((const float4 *)(JB + kJBlockHerm))[b];
                    float pa, nmin;
                    amp_prepare(hb, en2, A.cert_tol * grow, pa, nmin);
                    const float a = amp_step(jr.amp, pa, nmin, n2, rn);
                    if (a < 0.0f) ++acc.uncertain;   // the product lane abandons the ray here
                    else jr.amp = a;
                    acc.max_amp = fmax(acc.max_amp, (double)jr.amp);
                }
                jr.er = f.er * rn;
                jr.ei = f.ei * rn;
                jr.mr = f.mr * rn;
                jr.mi = f.mi * rn;
                const double ab = n2 * (b == 0 ? cw.x : cw.y) * inv * f01;
                if (t != 0.0) eerr += A.cert_tol * base * JB[kJBlockW + b] * 1.01 * rcp_nr(ab) + 1e-15;
                jener = jener * ab;
            }
        }
        if (b < 0 || b == 2) break;   // dies, or out-couples (GRTF:1162-1171, 1231-1240): the trace ends

        // ---- take branch b (GRTF:872-882 and every branch body after it) ----
        int tir, gap;
        if (kind == 0) { tir = b == 0 ? 0 : 2; gap = b == 0 ? 0 : 4; }
        else if (kind <= 2) { tir = b == 0 ? 0 : 1; gap = b == 0 ? 0 : 2; }
        else { tir = b == 0 ? 1 : 3; gap = b == 0 ? 2 : 6; }
        const RefField &Eb = E[b];
        cos_th = B[b];
        const double norm = sqrt(Eb.te * Eb.te + Eb.tm * Eb.tm);
        Ete = Eb.te / norm;
        Etm = Eb.tm / norm;
        dph = Eb.dphi + T[kTileTir + tir];
        x += T[kTileGap + gap];
        y += T[kTileGap + gap + 1];
        ener *= b == 0 ? e0 : e1;
        int next;
        if (kind == 0) {
            const bool in_ic = in_poly(loc, locate(loc, x, y), kPolyIC, x, y);
            next = b == 0 ? (in_ic ? 0 : 2) : (in_ic ? 1 : kDie);
        } else if (kind <= 2) {
            next = b == 0 ? 2 : 3;
        } else {
            next = b == 0 ? 4 : 5;
        }
        if (next < 0) break;
        region = next;
        entry = false;

        // ---- loop iterations up to the next interaction (GRTF:905-1246) ----
        const int hg = region == 2 ? 0 : 2;   // miss hop: gap[0:2] + 2 TIR[0] in R2, gap[2:4] + 2 TIR[1] in R3 / R4
        blk = -1;
        for (;;) {
            if (bounces > (uint32_t)kMaxLoop) break;
            ++bounces;
            const Cell c = locate(loc, x, y);
            if (!in_poly(loc, c, kPolyEff1, x, y)) break;
            if (region <= 1) {
                kind = 0;
                blk = 1 + region;
                break;
            }
            if (region <= 3) {
                const int sl = first_slice(loc, c, kPolyFC0, A.nfc, x, y);
                if (sl >= 0) {
                    kind = region - 1;
                    blk = 3 + (region - 2) * A.nfc + sl;
                    break;
                }
                if (region == 3 && !in_poly(loc, c, kPolyEff2, x, y)) {
                    region = 4;   // GRTF:1103-1104
                    continue;
                }
            } else {
                const int sl = first_slice(loc, c, kPolyFC0 + A.nfc, A.noc, x, y);
                if (sl >= 0) {
                    kind = region - 1;
                    blk = 3 + 2 * A.nfc + (region - 4) * A.noc + sl;
                    break;
                }
                if (region == 5) break;   // GRTF:1244-1246
            }
            x += T[kTileGap + hg];
            y += T[kTileGap + hg + 1];
            dph += 2 * T[kTileTir + hg / 2];
            ++hops;
        }
        if (blk < 0) break;
    }
    A.rng[i] = s;
    if (A.per_ray) A.per_ray[i] = bounces;
    acc.bounces += bounces;
}

__device__ __forceinline__ double wave_max(double v) {
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    return v;
}

template <class Loc>
__global__ __launch_bounds__(256) void shadow_kernel(ShadowArgs S, Loc loc) {
    const TraceArgs &A = S.A;
    ShadowAcc acc;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n_rays;
         i += (int64_t)gridDim.x * blockDim.x)
        shadow_trace(A, loc, i, acc);
    wgrt_shadow_stats *o = S.out;
    const bool lead = (threadIdx.x & 63) == 0;
    const uint64_t dec = wave_sum(acc.decisions), unc = wave_sum(acc.uncertain), fl = wave_sum(acc.flips);
    const uint64_t bo = wave_sum(acc.bounces), fb = wave_sum(acc.fallbacks);
    const double mr = wave_max(acc.max_ratio), mr32 = wave_max(acc.max_ratio32), me = wave_max(acc.max_ener);
    const double ma = wave_max(acc.max_amp);
    if (lead) {
        atomicAdd((unsigned long long *)&o->decisions, (unsigned long long)dec);
        atomicAdd((unsigned long long *)&o->uncertain, (unsigned long long)unc);
        atomicAdd((unsigned long long *)&o->silent_flips, (unsigned long long)fl);
        atomicAdd((unsigned long long *)&o->bounces, (unsigned long long)bo);
        atomicAdd((unsigned long long *)&o->fallbacks, (unsigned long long)fb);
        atomic_max_pos(&o->max_ratio, mr);
        atomic_max_pos(&o->max_ratio32, mr32);
        atomic_max_pos(&o->max_ener_ratio, me);
        atomic_max_pos(&o->max_amp, ma);
    }
    for (int k = 0; k < kDepthBuckets; ++k) {
        const double v = wave_max(acc.max_depth[k]);
        const uint64_t c = wave_sum(acc.n_depth[k]);
        if (lead) {
            atomic_max_pos(&o->max_ratio_by_depth[k], v);
            if (c) atomicAdd((unsigned long long *)&o->decisions_by_depth[k], (unsigned long long)c);
        }
    }
    for (int k = 0; k < kHistBuckets; ++k) {
        const uint64_t c = wave_sum(acc.hist[k]);
        if (lead && c) atomicAdd((unsigned long long *)&o->ratio_hist[k], (unsigned long long)c);
    }
}

}  // namespace

extern "C" wgrt_status wgrt_debug_shadow(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays,
                                         int64_t gid_offset, int single, uint32_t *rng_states,
                                         uint32_t *per_ray_bounces, wgrt_shadow_stats *stats, void *stream) {
    if (!s || !rays || !stats) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL scene / rays / stats");
    if (n_rays < 0 || gid_offset < 0) return fail(WGRT_ERR_INVALID_ARGUMENT, "negative n_rays / gid_offset");
    if (single && s->nl != 1)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "single-wavelength shadow needs a scene built with num_lmd == 1");
    if (n_rays == 0) return WGRT_OK;
    if (!rays->x || !rays->y || !rays->m || !rays->n || (!single && !rays->lmd_num) || !rays->te || !rays->tm ||
        !rays->delta_phase || !rng_states)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL ray column / rng_states");
    ShadowArgs S{};
    TraceArgs &A = S.A;
    A.x = rays->x;
    A.y = rays->y;
    A.m = rays->m;
    A.n = rays->n;
    A.l = single ? nullptr : rays->lmd_num;
    A.te = rays->te;
    A.tm = rays->tm;
    A.dph = rays->delta_phase;
    A.rng = rng_states;
    A.per_ray = per_ray_bounces;
    A.n_rays = n_rays;
    A.gid_offset = gid_offset;
    A.tiles = s->d_tiles;
    A.jtiles = s->d_jtiles;
    A.tile_d = s->tile_d;
    A.jtile_d = s->jtile_d;
    A.loc = make_locator(s);
    A.nfc = s->nfc;
    A.noc = s->noc;
    A.nx = s->nx;
    A.ny = s->ny;
    A.nl = s->nl;
    A.n_g = s->n_g;
    A.inv_n_g = 1.0 / s->n_g;
    A.threshold = single ? 1e-15 : 0.0;
    A.cert_tol = kCertTol;   // the bounds the product lane uses by default
    A.cert_tol32 = std::max(kCertTol32, A.cert_tol);
    S.out = stats;
    DeviceScope dev_scope(s->device);   // launched on the scene's device; the caller's is restored
    if (dev_scope.error() != hipSuccess)
        return fail(WGRT_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(dev_scope.error()));
    const int64_t blocks = std::min<int64_t>((n_rays + 255) / 256, 16384);
    hipLaunchKernelGGL(shadow_kernel<Locator>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, S, A.loc);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("shadow_kernel: ") + hipGetErrorString(e));
    return WGRT_OK;
}
