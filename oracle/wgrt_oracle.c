/*
 * wgrt_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C, float64, CPU restatement of the reference's full-colour Monte-Carlo
 * bounce kernel `process_rays_kernel_pro_fullColor`
 * (reference GPU_ray_tracing_functions.py = GRTF:833-1246) and of every device
 * function it calls (GRTF:25-165).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.
 *
 * Semantics follow the reference executed with Python / numpy scalar semantics
 * (what the committed golden fixtures were generated with):
 *   - all state promoted to float64 on first use (GRTF:846, 872-880);
 *   - complex products in the textbook form (re = ar*br - ai*bi, im = ar*bi + ai*br)
 *     including the multiplications by 0.0 that Python performs when it promotes a
 *     real operand to complex (GRTF:136-144);
 *   - math.hypot is correctly rounded in CPython 3.10, so `hypot_cr` below is a
 *     correctly-rounded hypot (double-double square sum + one Newton correction);
 *   - cos / sin / atan2 / floor / sqrt are glibc's, exactly what Python's math
 *     module calls;
 *   - no FMA contraction (build with -ffp-contract=off);
 *   - eyebox binning uses the flat-offset addressing of compiled numba (negative
 *     index wraps once, index == axis length aliases into the next row), guarded
 *     to the buffer.
 * Parity status: pinned by the golden fixtures under tests/golden (outputs of the reference's own
 * kernel code) -- see tests/test_oracle_golden.py.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "wgrt_oracle.h"

#define PI_D 3.141592653589793

/* Analysis hook (tools/hop_runs.c includes this file with its own definition): one call per
 * bounce event -- ev 0 interaction at (x, y) before the branch moves the ray, 1 miss hop from (x, y)
 * by (gx, gy), 2 the R3 -> R4 switch, 3 termination by the loop-top eff_reg1 test or an R5 miss.
 * A no-op in the oracle library. */
#ifndef ORACLE_EV
#define ORACLE_EV(ev, region, x, y, gx, gy) ((void)0)
#endif
/* Analysis hooks (oracle/wgrt_oracle_ev.c): every value of the guard product ener * e (GRTF:1020,
 * 1073, 1136, ...) before it is compared with the threshold, and the start / end of ray i's trace.
 * No-ops in the oracle library. */
#ifndef ORACLE_ENER
#define ORACLE_ENER(en) ((void)0)
#endif
#ifndef ORACLE_RAY_BEGIN
#define ORACLE_RAY_BEGIN(i) ((void)0)
#define ORACLE_RAY_END(i) ((void)0)
#endif
#define EB_NY 80
#define EB_NX 120

/* ---- GRTF:25-34 xorshift32 ------------------------------------------------ */
static double rng_draw(uint32_t *s, int64_t gid) {
    uint32_t v = *s;
    if (v == 0u) v = 0x6D2B79F5u ^ (uint32_t)(gid + 1);
    v ^= v << 13;
    v ^= v >> 17;
    v ^= v << 5;
    *s = v;
    return (double)v * (1.0 / 4294967296.0);
}

/* ---- correctly rounded hypot (CPython 3.10 math.hypot is correctly rounded) */
static double hypot_cr(double x, double y) {
    double ax = fabs(x), ay = fabs(y);
    if (isinf(ax) || isinf(ay)) return INFINITY;
    if (isnan(ax) || isnan(ay)) return NAN;
    if (ax < ay) { double t = ax; ax = ay; ay = t; }
    if (ay == 0.0) return ax;
    int e;
    frexp(ax, &e);
    double sx = ldexp(ax, -e), sy = ldexp(ay, -e);   /* sx in [0.5, 1) */
    double h = sx * sx, hl = fma(sx, sx, -h);
    double k = sy * sy, kl = fma(sy, sy, -k);
    double s = h + k;
    double lo = ((h - s) + k) + (hl + kl);
    double r = sqrt(s);
    double rr = fma(-r, r, s);
    r = r + (rr + lo) / (2.0 * r);
    return ldexp(r, e);
}

/* ---- GRTF:124-130 -------------------------------------------------------- */
static double wrap_pi(double x) {
    const double two_pi = 2.0 * PI_D;
    x = x + PI_D;
    x = x - two_pi * floor(x / two_pi);
    return x - PI_D;
}

typedef struct { double re, im; } cplx;

/* ---- GRTF:132-152  E_field_cal(Ete, Etm, delta, p, q, r, s) ------------------
 * Ete' = p*te_in + r*tm_in ; Etm' = q*te_in + s*tm_in  (b = 3rd, c = 2nd arg). */
typedef struct { double te, tm, dphi; double te_re, te_im, tm_re, tm_im; } efield;

static void efield_amp(double Ete, double Etm, double cd, double sd,
                       const cplx *p, const cplx *q, const cplx *r, const cplx *s,
                       efield *o) {
    /* te_in = (Ete, 0); tm_in = (cd, sd) * (Etm, 0) */
    double ti_re = cd * Etm - sd * 0.0, ti_im = cd * 0.0 + sd * Etm;
    double a_re = p->re * Ete - p->im * 0.0, a_im = p->re * 0.0 + p->im * Ete;
    double b_re = r->re * ti_re - r->im * ti_im, b_im = r->re * ti_im + r->im * ti_re;
    double c_re = q->re * Ete - q->im * 0.0, c_im = q->re * 0.0 + q->im * Ete;
    double d_re = s->re * ti_re - s->im * ti_im, d_im = s->re * ti_im + s->im * ti_re;
    o->te_re = a_re + b_re; o->te_im = a_im + b_im;
    o->tm_re = c_re + d_re; o->tm_im = c_im + d_im;
    o->te = hypot_cr(o->te_re, o->te_im);
    o->tm = hypot_cr(o->tm_re, o->tm_im);
}

static double efield_phase(const efield *o) {
    double pte = (o->te >= 1e-20) ? atan2(o->te_im, o->te_re) : 0.0;
    double ptm = (o->tm >= 1e-20) ? atan2(o->tm_im, o->tm_re) : 0.0;
    return wrap_pi(ptm - pte);
}

/* ---- GRTF:36-71 polygon membership --------------------------------------- */
static int on_segment(double px, double py, double x1, double y1, double x2, double y2) {
    const double tol = 1e-12;
    if (px < fmin(x1, x2) - tol || px > fmax(x1, x2) + tol ||
        py < fmin(y1, y2) - tol || py > fmax(y1, y2) + tol)
        return 0;
    return fabs((x2 - x1) * (py - y1) - (y2 - y1) * (px - x1)) <= tol;
}

/* vertices poly[k] = (xy[2k], xy[2k+1]), k in [0, nv) */
static int inside_or_on_edge(double px, double py, const double *xy, int64_t nv) {
    if (nv <= 0) return 0;
    int64_t j = nv - 1;
    for (int64_t i = 0; i < nv; ++i) {
        if (on_segment(px, py, xy[2 * j], xy[2 * j + 1], xy[2 * i], xy[2 * i + 1])) return 1;
        j = i;
    }
    int inside = 0;
    j = nv - 1;
    for (int64_t i = 0; i < nv; ++i) {
        double xi = xy[2 * i], yi = xy[2 * i + 1], xj = xy[2 * j], yj = xy[2 * j + 1];
        if (((yi > py) != (yj > py)) && (px < (xj - xi) * (py - yi) / (yj - yi + 1e-20) + xi))
            inside = !inside;
        j = i;
    }
    return inside;
}

/* Note on min/max: Python's builtin min(x1, x2) returns x1 unless x2 < x1; for the
 * non-NaN, non-signed-zero-sensitive comparisons above fmin/fmax give the same value
 * (a signed-zero difference cannot change the result of "px < v - tol"). */

/* ---- ray record ----------------------------------------------------------- */
typedef struct {
    double x, y, Ete, Etm, dph, cos_th, ener, gx, gy;
} ray_state;

static const cplx *lut5(const wgrt_oracle_scene *sc, const double *lut, int64_t slice,
                        int l, int m, int n, int ch) {
    int64_t idx = ((((slice * sc->num_lmd + l) * sc->nx + m) * sc->ny + n) * sc->ch5) + ch;
    return (const cplx *)(lut + 2 * idx);
}
static const cplx *lut3(const wgrt_oracle_scene *sc, const double *lut, int64_t slice,
                        int l, int m, int n, int ch) {
    int64_t idx = ((((slice * sc->num_lmd + l) * sc->nx + m) * sc->ny + n) * sc->ch3) + ch;
    return (const cplx *)(lut + 2 * idx);
}

/* math.cos(lut[..., 0].real) of table k (GRTF:866-869, 917-918, ...): double cos of a complex128
 * table's angle; for a complex64 table (f32_mask bit k) compiled numba types the float32 .real's
 * cosine as float32, i.e. cosf of the float32 angle. */
enum { T_IC1, T_IC2, T_IC3, T_FC1, T_FC2, T_OC1, T_OC2 };
static double lcos(const wgrt_oracle_scene *sc, int k, double th) {
    return ((sc->f32_mask >> k) & 1) ? (double)cosf((float)th) : cos(th);
}

/* Take branch: update field, direction, position (the common block of every branch);
 * cos_theta = math.cos of the new direction's angle (lcos). */
static void take(ray_state *st, const efield *E, double cos_theta, double tir, const double *gap2) {
    st->cos_th = cos_theta;
    double norm = sqrt(E->te * E->te + E->tm * E->tm);
    double ph = efield_phase(E);
    st->Ete = E->te / norm;
    st->Etm = E->tm / norm;
    st->dph = ph + tir;
    st->gx = gap2[0];
    st->gy = gap2[1];
    st->x += st->gx;
    st->y += st->gy;
}

static void eb_add(const wgrt_oracle_scene *sc, float *eb, int l, int m, int n, double x, double y) {
    const double *rg = sc->eff_reg_fov_range + 4 * ((int64_t)m * sc->ny + n);
    double xmin = rg[0], xmax = rg[1], ymin = rg[2], ymax = rg[3];
    double dx = (xmax - xmin) / EB_NX;
    double dy = (ymax - ymin) / EB_NY;
    int64_t ix = (int64_t)floor((x - xmin) / dx);
    int64_t iy = (int64_t)floor((y - ymin) / dy);
    if (ix < 0) ix += EB_NX;
    if (iy < 0) iy += EB_NY;
    int64_t off = ((((int64_t)l * sc->ny + n) * sc->nx + m) * EB_NY + iy) * EB_NX + ix;
    int64_t total = (int64_t)sc->num_lmd * sc->ny * sc->nx * EB_NY * EB_NX;
    if (off >= 0 && off < total) {
#pragma omp atomic
        eb[off] += 1.0f;
    }
}

/* Trace one ray; returns the number of bounce events (1 + loop iterations). */
static uint32_t trace_one(const wgrt_oracle_scene *sc, const wgrt_oracle_rays *rays, int64_t i,
                          int64_t gid, uint32_t *rng, float *eb, uint8_t *fate) {
    uint8_t why = 0;   /* fate code: 10 * region + reason (region 9 = in-coupling event) */
    ray_state st;
    st.x = (double)rays->x[i];
    st.y = (double)rays->y[i];
    int m = (int)rays->m[i], n = (int)rays->n[i], l = rays->lmd ? (int)rays->lmd[i] : 0;
    st.Ete = (double)rays->te[i];
    st.Etm = (double)rays->tm[i];
    st.dph = (double)rays->dph[i];
    st.ener = 1.0;
    uint32_t s = rng[i];
    uint32_t bounces = 1;
    const double n_g = sc->n_g;
    const double *tir = sc->lut_tir + 4 * (((int64_t)l * sc->nx + m) * sc->ny + n);
    const double *gap = sc->lut_gap + 8 * (((int64_t)l * sc->nx + m) * sc->ny + n);
    const double th_ic1 = lut5(sc, sc->ic1, 0, l, m, n, 0)->re;
    const double th_ic2 = lut5(sc, sc->ic2, 0, l, m, n, 0)->re;
    const double th_ic3 = lut5(sc, sc->ic3, 0, l, m, n, 0)->re;
    int region;
    efield E1, E2, E3;

    /* ---- in-coupling (GRTF:860-904) ---- */
    {
        double cd = cos(st.dph), sd = sin(st.dph);
        efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, sc->ic1, 0, l, m, n, 13), lut5(sc, sc->ic1, 0, l, m, n, 18),
                   lut5(sc, sc->ic1, 0, l, m, n, 33), lut5(sc, sc->ic1, 0, l, m, n, 38), &E1);
        efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, sc->ic1, 0, l, m, n, 15), lut5(sc, sc->ic1, 0, l, m, n, 20),
                   lut5(sc, sc->ic1, 0, l, m, n, 35), lut5(sc, sc->ic1, 0, l, m, n, 40), &E2);
        double e1 = (E1.te * E1.te + E1.tm * E1.tm) * lcos(sc, T_IC2, th_ic2) / lcos(sc, T_IC1, th_ic1) * n_g;
        double e2 = (E2.te * E2.te + E2.tm * E2.tm) * lcos(sc, T_IC3, th_ic3) / lcos(sc, T_IC1, th_ic1) * n_g;
        double u = rng_draw(&s, gid);
        ORACLE_EV(0, 9, st.x, st.y, 0.0, 0.0);
        if (u <= e1) {
            take(&st, &E1, lcos(sc, T_IC2, th_ic2), tir[0], gap + 0);
            st.ener *= e1;
            region = inside_or_on_edge(st.x, st.y, sc->ic, sc->n_ic) ? 0 : 2;
        } else if (u <= e1 + e2) {
            take(&st, &E2, lcos(sc, T_IC3, th_ic3), tir[2], gap + 4);
            st.ener *= e2;
            if (!inside_or_on_edge(st.x, st.y, sc->ic, sc->n_ic)) { why = 96; goto done; }
            region = 1;
        } else {
            why = 92;
            goto done;
        }
    }

    for (int64_t it = 0; it < 100000; ++it) {
        ++bounces;
        if (!inside_or_on_edge(st.x, st.y, sc->eff1, sc->n_eff1)) {
            ORACLE_EV(3, region, st.x, st.y, 0.0, 0.0);
            why = (uint8_t)(10 * region + 1);
            goto done;
        }
        double cd = cos(st.dph), sd = sin(st.dph);
        if (region == 0 || region == 1) {
            /* GRTF:908-999 */
            const double *L = region == 0 ? sc->ic2 : sc->ic3;
            if (region == 0) {
                efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, 0, l, m, n, 4), lut5(sc, L, 0, l, m, n, 9),
                           lut5(sc, L, 0, l, m, n, 24), lut5(sc, L, 0, l, m, n, 29), &E1);
                efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, 0, l, m, n, 6), lut5(sc, L, 0, l, m, n, 11),
                           lut5(sc, L, 0, l, m, n, 26), lut5(sc, L, 0, l, m, n, 31), &E2);
            } else {
                efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, 0, l, m, n, 2), lut5(sc, L, 0, l, m, n, 22),
                           lut5(sc, L, 0, l, m, n, 7), lut5(sc, L, 0, l, m, n, 27), &E1);
                efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, 0, l, m, n, 4), lut5(sc, L, 0, l, m, n, 9),
                           lut5(sc, L, 0, l, m, n, 24), lut5(sc, L, 0, l, m, n, 29), &E2);
            }
            double e1 = (E1.te * E1.te + E1.tm * E1.tm) * lcos(sc, T_IC2, th_ic2) / st.cos_th;
            double e2 = (E2.te * E2.te + E2.tm * E2.tm) * lcos(sc, T_IC3, th_ic3) / st.cos_th;
            double u = rng_draw(&s, gid);
            ORACLE_EV(0, region, st.x, st.y, 0.0, 0.0);
            if (u <= e1) {
                take(&st, &E1, lcos(sc, T_IC2, th_ic2), tir[0], gap + 0);
                st.ener *= e1;
                region = inside_or_on_edge(st.x, st.y, sc->ic, sc->n_ic) ? 0 : 2;
            } else if (u <= e1 + e2) {
                take(&st, &E2, lcos(sc, T_IC3, th_ic3), tir[2], gap + 4);
                st.ener *= e2;
                if (!inside_or_on_edge(st.x, st.y, sc->ic, sc->n_ic)) { why = (uint8_t)(10 * region + 6); goto done; }
                region = 1;
            } else {
                why = (uint8_t)(10 * region + 2);
                goto done;
            }
        } else if (region == 2 || region == 3) {
            /* GRTF:1000-1108 */
            int hit = 0;
            for (int64_t k = 0; k < sc->n_fc_slices; ++k) {
                int64_t a = sc->fc_offset[k], b = sc->fc_offset[k + 1];
                if (!inside_or_on_edge(st.x, st.y, sc->fc + 2 * a, b - a)) continue;
                hit = 1;
                const double th1 = lut3(sc, sc->fc1, k, l, m, n, 0)->re;
                const double th2 = lut3(sc, sc->fc2, k, l, m, n, 0)->re;
                if (region == 2) {
                    const double *L = sc->fc1;
                    efield_amp(st.Ete, st.Etm, cd, sd, lut3(sc, L, k, l, m, n, 3), lut3(sc, L, k, l, m, n, 6),
                               lut3(sc, L, k, l, m, n, 15), lut3(sc, L, k, l, m, n, 18), &E1);
                    efield_amp(st.Ete, st.Etm, cd, sd, lut3(sc, L, k, l, m, n, 2), lut3(sc, L, k, l, m, n, 5),
                               lut3(sc, L, k, l, m, n, 14), lut3(sc, L, k, l, m, n, 17), &E2);
                } else {
                    const double *L = sc->fc2;
                    efield_amp(st.Ete, st.Etm, cd, sd, lut3(sc, L, k, l, m, n, 4), lut3(sc, L, k, l, m, n, 7),
                               lut3(sc, L, k, l, m, n, 16), lut3(sc, L, k, l, m, n, 19), &E1);
                    efield_amp(st.Ete, st.Etm, cd, sd, lut3(sc, L, k, l, m, n, 3), lut3(sc, L, k, l, m, n, 6),
                               lut3(sc, L, k, l, m, n, 15), lut3(sc, L, k, l, m, n, 18), &E2);
                }
                double e1 = (E1.te * E1.te + E1.tm * E1.tm) * lcos(sc, T_FC1, th1) / st.cos_th;
                double e2 = (E2.te * E2.te + E2.tm * E2.tm) * lcos(sc, T_FC2, th2) / st.cos_th;
                double en1 = st.ener * e1, en2 = st.ener * e2;
                ORACLE_ENER(en1);
                ORACLE_ENER(en2);
                double u = rng_draw(&s, gid);
                ORACLE_EV(0, region, st.x, st.y, 0.0, 0.0);
                if (u <= e1 && en1 > sc->threshold) {
                    take(&st, &E1, lcos(sc, T_FC1, th1), tir[0], gap + 0);
                    st.ener = en1 * 1.0;
                    region = 2;
                } else if (u <= e1 + e2 && en2 > sc->threshold) {
                    take(&st, &E2, lcos(sc, T_FC2, th2), tir[1], gap + 2);
                    st.ener = en2 * 1.0;
                    region = 3;
                } else {
                    why = (uint8_t)(10 * region + 2);
                    goto done;
                }
                break;
            }
            if (!hit) {
                if (region == 2) {
                    ORACLE_EV(1, region, st.x, st.y, st.gx, st.gy);
                    st.x += st.gx;
                    st.y += st.gy;
                    st.dph += 2 * tir[0];
                } else if (!inside_or_on_edge(st.x, st.y, sc->eff2, sc->n_eff2)) {
                    ORACLE_EV(2, region, st.x, st.y, 0.0, 0.0);
                    region = 4;
                } else {
                    ORACLE_EV(1, region, st.x, st.y, st.gx, st.gy);
                    st.x += st.gx;
                    st.y += st.gy;
                    st.dph += 2 * tir[1];
                }
            }
        } else {
            /* region 4 / 5: GRTF:1110-1246 */
            int hit = 0;
            for (int64_t k = 0; k < sc->n_oc_slices; ++k) {
                int64_t a = sc->oc_offset[k], b = sc->oc_offset[k + 1];
                if (!inside_or_on_edge(st.x, st.y, sc->oc + 2 * a, b - a)) continue;
                hit = 1;
                const double th1 = lut5(sc, sc->oc1, k, l, m, n, 0)->re;
                const double th2 = lut5(sc, sc->oc2, k, l, m, n, 0)->re;
                if (region == 4) {
                    const double *L = sc->oc1;
                    efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, k, l, m, n, 4), lut5(sc, L, k, l, m, n, 9),
                               lut5(sc, L, k, l, m, n, 24), lut5(sc, L, k, l, m, n, 29), &E1);
                    efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, k, l, m, n, 2), lut5(sc, L, k, l, m, n, 7),
                               lut5(sc, L, k, l, m, n, 22), lut5(sc, L, k, l, m, n, 27), &E2);
                    efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, k, l, m, n, 13), lut5(sc, L, k, l, m, n, 18),
                               lut5(sc, L, k, l, m, n, 33), lut5(sc, L, k, l, m, n, 38), &E3);
                } else {
                    const double *L = sc->oc2;
                    efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, k, l, m, n, 6), lut5(sc, L, k, l, m, n, 11),
                               lut5(sc, L, k, l, m, n, 26), lut5(sc, L, k, l, m, n, 31), &E1);
                    efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, k, l, m, n, 4), lut5(sc, L, k, l, m, n, 9),
                               lut5(sc, L, k, l, m, n, 24), lut5(sc, L, k, l, m, n, 29), &E2);
                    efield_amp(st.Ete, st.Etm, cd, sd, lut5(sc, L, k, l, m, n, 15), lut5(sc, L, k, l, m, n, 20),
                               lut5(sc, L, k, l, m, n, 35), lut5(sc, L, k, l, m, n, 40), &E3);
                }
                double e1 = (E1.te * E1.te + E1.tm * E1.tm) * lcos(sc, T_OC1, th1) / st.cos_th;
                double e2 = (E2.te * E2.te + E2.tm * E2.tm) * lcos(sc, T_OC2, th2) / st.cos_th;
                double e3 = (E3.te * E3.te + E3.tm * E3.tm) * lcos(sc, T_IC1, th_ic1) / st.cos_th / n_g;
                double en1 = st.ener * e1, en2 = st.ener * e2, en3 = st.ener * e3;
                ORACLE_ENER(en1);
                ORACLE_ENER(en2);
                ORACLE_ENER(en3);
                double u = rng_draw(&s, gid);
                ORACLE_EV(0, region, st.x, st.y, 0.0, 0.0);
                if (u <= e1 && en1 > sc->threshold) {
                    take(&st, &E1, lcos(sc, T_OC1, th1), tir[1], gap + 2);
                    st.ener = en1 * 1.0;
                    region = 4;
                } else if (u <= e1 + e2 && en2 > sc->threshold) {
                    take(&st, &E2, lcos(sc, T_OC2, th2), tir[3], gap + 6);
                    st.ener = en2 * 1.0;
                    region = 5;
                } else if (u <= e1 + e2 + e3 && en3 > sc->threshold) {
                    const double *rect = sc->eff_reg_fov + 8 * ((int64_t)m * sc->ny + n);
                    if (inside_or_on_edge(st.x, st.y, rect, 4)) { eb_add(sc, eb, l, m, n, st.x, st.y); why = (uint8_t)(10 * region + 3); }
                    else why = (uint8_t)(10 * region + 4);
                    goto done;
                } else {
                    why = (uint8_t)(10 * region + 2);
                    goto done;
                }
                break;
            }
            if (!hit) {
                if (region == 5) {
                    ORACLE_EV(3, region, st.x, st.y, 0.0, 0.0);
                    why = 55;
                    goto done;
                }
                ORACLE_EV(1, region, st.x, st.y, st.gx, st.gy);
                st.x += st.gx;
                st.y += st.gy;
                st.dph += 2 * tir[1];
            }
        }
    }
    why = (uint8_t)(10 * region + 7);
done:
    if (fate) fate[i] = why;
    rng[i] = s;
    return bounces;
}

int64_t wgrt_oracle_trace(const wgrt_oracle_scene *sc, const wgrt_oracle_rays *rays, int64_t n_rays,
                          int64_t gid_offset, uint32_t *rng, float *eb, uint32_t *bounces_out,
                          uint8_t *fate_out, int n_threads) {
    int64_t total = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : total)
    for (int64_t i = 0; i < n_rays; ++i) {
        ORACLE_RAY_BEGIN(i);
        uint32_t b = trace_one(sc, rays, i, gid_offset + i, rng, eb, fate_out);
        ORACLE_RAY_END(i);
        if (bounces_out) bounces_out[i] = b;
        total += b;
    }
    return total;
}

/* exported primitives, for unit tests */
double wgrt_oracle_hypot(double x, double y) { return hypot_cr(x, y); }
double wgrt_oracle_wrap(double x) { return wrap_pi(x); }
int wgrt_oracle_inside(double px, double py, const double *xy, int64_t nv) {
    return inside_or_on_edge(px, py, xy, nv);
}
uint32_t wgrt_oracle_xorshift(uint32_t s, int64_t gid, double *u) {
    *u = rng_draw(&s, gid);
    return s;
}

void wgrt_oracle_inside_many(const double *pts, int64_t n, const double *xy, int64_t nv, int32_t *out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) out[i] = inside_or_on_edge(pts[2 * i], pts[2 * i + 1], xy, nv);
}
