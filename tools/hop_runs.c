/* hop_runs.c -- analysis tool (not product code): how a ray's bounces split into interactions and
 * miss hops, and how many wave passes a ray's chain would take if runs of miss hops that stay
 * clear of every polygon edge ran inside one pass.
 *
 * It compiles the CPU oracle (oracle/wgrt_oracle.c, the reference's FSM: GRTF:833-1246) into this
 * translation unit with an event hook (ORACLE_EV) that records each bounce: an interaction, a miss
 * hop (GRTF:1049-1052, 1105-1108, 1175-1178), the R3 -> R4 switch (GRTF:1103-1104) or a
 * termination.  Per ray it then counts the passes of three pass models (the product kernel runs one
 * bounce per pass: passes == bounces):
 *   disc  -- a miss hop at p0 continues, inside the same pass, with every following miss hop whose
 *            start lies within r(p0) of p0, r(p0) the safe radius of p0's coarse cell: the distance
 *            from that cell to the nearest edge of the polygons the region tests (R2/R3: eff_reg1,
 *            eff_reg2, FC slices; R4: eff_reg1, OC slices), less a margin;
 *   exact -- the same with r(p0) the exact distance from p0 (an upper bound on what a field gives);
 *   known -- a coarse grid answers a position's whole cell word when the coarse cell is clear of
 *            every polygon edge; a pass continues through miss hops while each landing cell is
 *            answered so, and ends at an interaction, a termination or a landing that needs the
 *            global locator.
 * Built and driven by tools/hop_runs.py (ctypes).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint8_t ev, region;
    double x, y, gx, gy;
} hr_event;

#define HR_MAX_EV 200000
static __thread hr_event *hr_buf;
static __thread int hr_n;

#define ORACLE_EV(ev_, region_, x_, y_, gx_, gy_)                                                  \
    do {                                                                                           \
        if (hr_n < HR_MAX_EV) {                                                                    \
            hr_buf[hr_n].ev = (uint8_t)(ev_);                                                      \
            hr_buf[hr_n].region = (uint8_t)(region_);                                              \
            hr_buf[hr_n].x = (x_);                                                                 \
            hr_buf[hr_n].y = (y_);                                                                 \
            hr_buf[hr_n].gx = (gx_);                                                               \
            hr_buf[hr_n].gy = (gy_);                                                               \
        }                                                                                          \
        ++hr_n;                                                                                    \
    } while (0)

#include "../oracle/wgrt_oracle.c"

/* ---- coarse fields ------------------------------------------------------------------------- */
typedef struct {
    double x0, y0, h;
    int ncx, ncy;
    float *d_fc, *d_oc;   /* lower bound of the distance from the cell to the set's edges */
    uint8_t *known;       /* cell clear of every polygon's edges by more than the margin */
} hr_field;

static double seg_dist(double px, double py, double ax, double ay, double bx, double by) {
    const double dx = bx - ax, dy = by - ay, l2 = dx * dx + dy * dy;
    double t = l2 > 0.0 ? ((px - ax) * dx + (py - ay) * dy) / l2 : 0.0;
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    const double ex = ax + t * dx - px, ey = ay + t * dy - py;
    return sqrt(ex * ex + ey * ey);
}

static double ring_dist(double px, double py, const double *xy, int64_t nv) {
    double d = INFINITY;
    for (int64_t i = 0, j = nv - 1; i < nv; j = i++) {
        const double v = seg_dist(px, py, xy[2 * j], xy[2 * j + 1], xy[2 * i], xy[2 * i + 1]);
        if (v < d) d = v;
    }
    return d;
}

static double slices_dist(double px, double py, const double *xy, const int64_t *off, int64_t ns) {
    double d = INFINITY;
    for (int64_t k = 0; k < ns; ++k) {
        const double v = ring_dist(px, py, xy + 2 * off[k], off[k + 1] - off[k]);
        if (v < d) d = v;
    }
    return d;
}

static double dist_fc(const wgrt_oracle_scene *sc, double x, double y) {
    double d = ring_dist(x, y, sc->eff1, sc->n_eff1);
    d = fmin(d, ring_dist(x, y, sc->eff2, sc->n_eff2));
    return fmin(d, slices_dist(x, y, sc->fc, sc->fc_offset, sc->n_fc_slices));
}

static double dist_oc(const wgrt_oracle_scene *sc, double x, double y) {
    return fmin(ring_dist(x, y, sc->eff1, sc->n_eff1), slices_dist(x, y, sc->oc, sc->oc_offset, sc->n_oc_slices));
}

static int cell_of(const hr_field *F, double x, double y) {
    const double fx = floor((x - F->x0) / F->h), fy = floor((y - F->y0) / F->h);
    if (!(fx >= 0 && fy >= 0 && fx < F->ncx && fy < F->ncy)) return -1;
    return (int)fy * F->ncx + (int)fx;
}

/* ---- per-ray pass models -------------------------------------------------------------------- */
#define HR_HOPS_HIST 64
typedef struct {
    int64_t rays, bounces, ev[4];
    int64_t runs, run_hist[HR_HOPS_HIST];   /* maximal runs of miss hops (the switch inside a run) */
    int64_t passes[3];                      /* disc, exact, known */
    int64_t per_pass_hist[3][HR_HOPS_HIST]; /* bounces consumed by a pass */
} hr_stats;

static void count_run(hr_stats *S, int64_t len) {
    if (len <= 0) return;
    S->runs++;
    S->run_hist[len < HR_HOPS_HIST - 1 ? len : HR_HOPS_HIST - 1]++;
}

static void pass_len(hr_stats *S, int model, int64_t len) {
    S->passes[model]++;
    S->per_pass_hist[model][len < HR_HOPS_HIST - 1 ? len : HR_HOPS_HIST - 1]++;
}

/* passes of one ray's event list under model `model` (0 disc, 1 exact, 2 known) */
static int64_t ray_passes(const wgrt_oracle_scene *sc, const hr_field *F, const hr_event *E, int n, int model,
                          double margin, hr_stats *S) {
    int64_t passes = 0;
    int j = 0;
    while (j < n) {
        int64_t len = 1;
        const hr_event *e = &E[j];
        if (e->ev == 1) {
            if (model <= 1) {
                double r;
                if (model == 1) {
                    r = (e->region == 4) ? dist_oc(sc, e->x, e->y) : dist_fc(sc, e->x, e->y);
                } else {
                    const int c = cell_of(F, e->x, e->y);
                    r = c < 0 ? 0.0 : (e->region == 4 ? F->d_oc[c] : F->d_fc[c]);
                }
                r -= margin;
                int k = j + 1;
                while (k < n && E[k].ev == 1 && E[k].region == e->region) {
                    const double dx = E[k].x - e->x, dy = E[k].y - e->y;
                    if (!(sqrt(dx * dx + dy * dy) < r)) break;
                    ++k;
                    ++len;
                }
                j = k;
            } else {
                /* the landing cell of each hop answered from the coarse grid: continue */
                int k = j;
                for (;;) {
                    const hr_event *h = &E[k];
                    if (h->ev == 2) {  /* switch: same position, the same word */
                        if (k + 1 >= n) { ++k; break; }
                        ++k;
                        ++len;
                        continue;
                    }
                    if (h->ev != 1) { ++k; break; }   /* interaction / termination ends the pass */
                    const int c = cell_of(F, h->x + h->gx, h->y + h->gy);
                    ++k;
                    if (c < 0 || !F->known[c] || k >= n) break;
                    ++len;
                }
                len = k - j;
                j = k;
            }
        } else {
            ++j;
        }
        pass_len(S, model, len);
        ++passes;
    }
    return passes;
}

int hr_analyze(const wgrt_oracle_scene *sc, const wgrt_oracle_rays *rays, int64_t n_rays, int64_t gid_offset,
               uint32_t *rng, float *eb, double cell_mm, double margin, int64_t *stats_out,
               uint32_t *per_ray /* [n_rays][4]: bounces, disc, exact, known passes */, int n_threads) {
    /* coarse fields over eff_reg1's bounding box (a position outside it terminates) */
    double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
    for (int64_t i = 0; i < sc->n_eff1; ++i) {
        xmin = fmin(xmin, sc->eff1[2 * i]);
        xmax = fmax(xmax, sc->eff1[2 * i]);
        ymin = fmin(ymin, sc->eff1[2 * i + 1]);
        ymax = fmax(ymax, sc->eff1[2 * i + 1]);
    }
    hr_field F;
    F.h = cell_mm;
    F.x0 = xmin - cell_mm;
    F.y0 = ymin - cell_mm;
    F.ncx = (int)ceil((xmax - F.x0) / cell_mm) + 2;
    F.ncy = (int)ceil((ymax - F.y0) / cell_mm) + 2;
    const int64_t nc = (int64_t)F.ncx * F.ncy;
    F.d_fc = (float *)malloc(nc * sizeof(float));
    F.d_oc = (float *)malloc(nc * sizeof(float));
    F.known = (uint8_t *)malloc(nc);
    const double half_diag = cell_mm * sqrt(2.0) / 2.0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < nc; ++c) {
        const double px = F.x0 + ((double)(c % F.ncx) + 0.5) * cell_mm;
        const double py = F.y0 + ((double)(c / F.ncx) + 0.5) * cell_mm;
        const double a = dist_fc(sc, px, py), b = dist_oc(sc, px, py);
        const double ic = ring_dist(px, py, sc->ic, sc->n_ic);
        F.d_fc[c] = (float)fmax(0.0, a - half_diag);
        F.d_oc[c] = (float)fmax(0.0, b - half_diag);
        F.known[c] = fmin(fmin(a, b), ic) > half_diag + margin;
    }
    hr_stats tot;
    memset(&tot, 0, sizeof(tot));
#pragma omp parallel
    {
        hr_stats S;
        memset(&S, 0, sizeof(S));
        hr_buf = (hr_event *)malloc(HR_MAX_EV * sizeof(hr_event));
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < n_rays; ++i) {
            hr_n = 0;
            const uint32_t b = trace_one(sc, rays, i, gid_offset + i, rng, eb, NULL);
            const int n = hr_n < HR_MAX_EV ? hr_n : HR_MAX_EV;
            S.rays++;
            S.bounces += b;
            int64_t run = 0;
            for (int k = 0; k < n; ++k) {
                S.ev[hr_buf[k].ev]++;
                if (hr_buf[k].ev == 1 || hr_buf[k].ev == 2) {
                    run += hr_buf[k].ev == 1;
                } else {
                    count_run(&S, run);
                    run = 0;
                }
            }
            count_run(&S, run);
            uint32_t p[3];
            for (int m = 0; m < 3; ++m) p[m] = (uint32_t)ray_passes(sc, &F, hr_buf, n, m, margin, &S);
            if (per_ray) {
                per_ray[4 * i] = b;
                per_ray[4 * i + 1] = p[0];
                per_ray[4 * i + 2] = p[1];
                per_ray[4 * i + 3] = p[2];
            }
        }
        free(hr_buf);
#pragma omp critical
        {
            int64_t *a = (int64_t *)&tot, *s = (int64_t *)&S;
            for (size_t k = 0; k < sizeof(hr_stats) / sizeof(int64_t); ++k) a[k] += s[k];
        }
    }
    memcpy(stats_out, &tot, sizeof(tot));
    int64_t known = 0;
    for (int64_t c = 0; c < nc; ++c) known += F.known[c];
    free(F.d_fc);
    free(F.d_oc);
    free(F.known);
    return (int)(sizeof(hr_stats) / sizeof(int64_t));
}
