/* wgrt_oracle.h -- TEST INFRASTRUCTURE ONLY: CPU float64 restatement of the reference's
 * process_rays_kernel_pro_fullColor (GPU_ray_tracing_functions.py:833-1246) and, with
 * lmd == NULL and threshold 1e-15, process_rays_kernel_pro (GPU_ray_tracing_functions.py:419-831).
 * Parity pinned by the golden fixtures under tests/golden.  Never linked into the product library. */
#ifndef WGRT_ORACLE_H
#define WGRT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const double *ic;  int64_t n_ic;                          /* [n_ic, 2] */
    const double *fc;  const int64_t *fc_offset; int64_t n_fc_slices;
    const double *oc;  const int64_t *oc_offset; int64_t n_oc_slices;
    const double *eff1; int64_t n_eff1;
    const double *eff2; int64_t n_eff2;
    const double *eff_reg_fov;        /* [NX, NY, 4, 2] */
    const double *eff_reg_fov_range;  /* [NX, NY, 4]    */
    const double *lut_tir;            /* [L, NX, NY, 4] */
    const double *lut_gap;            /* [L, NX, NY, 8] */
    /* complex128 tables, interleaved (re, im) */
    const double *ic1, *ic2, *ic3;    /* [L, NX, NY, ch5] */
    const double *fc1, *fc2;          /* [nFC, L, NX, NY, ch3] */
    const double *oc1, *oc2;          /* [nOC, L, NX, NY, ch5] */
    int32_t num_lmd, nx, ny, ch5, ch3;
    double n_g;
    double threshold;   /* R2..R5 guard ener * eff > threshold: 0 full colour (GRTF:859),
                           1e-15 single wavelength (GRTF:444) */
    int32_t f32_mask;   /* bit k: table k (ic1, ic2, ic3, fc1, fc2, oc1, oc2) was complex64, so compiled
                           numba takes math.cos of its float32 .real in single precision (cosf) */
} wgrt_oracle_scene;

typedef struct {
    const float *x, *y, *m, *n, *lmd, *te, *tm, *dph;   /* lmd NULL: single wavelength, l = 0 */
} wgrt_oracle_rays;

/* Traces rays [0, n_rays) of the given shard (global ids gid_offset + i); updates rng
 * in place, accumulates into eb [L, NY, NX, 80, 120]; optional per-ray bounce counts.
 * Optional per-ray fate code (10 * region + reason; region 9 = in-coupling event; reason
 * 1 left eff_reg1, 2 Monte-Carlo loss, 3 out-coupled into the eyebox, 4 out-coupled outside
 * it, 5 R5 miss, 6 left the in-coupler, 7 loop cap).
 * Returns the total number of bounce events (1 in-coupling + loop iterations per ray). */
int64_t wgrt_oracle_trace(const wgrt_oracle_scene *sc, const wgrt_oracle_rays *rays, int64_t n_rays,
                          int64_t gid_offset, uint32_t *rng, float *eb, uint32_t *bounces_out,
                          uint8_t *fate_out, int n_threads);

double wgrt_oracle_hypot(double x, double y);
double wgrt_oracle_wrap(double x);
int wgrt_oracle_inside(double px, double py, const double *xy, int64_t nv);
uint32_t wgrt_oracle_xorshift(uint32_t s, int64_t gid, double *u);
void wgrt_oracle_inside_many(const double *pts, int64_t n, const double *xy, int64_t nv, int32_t *out);

#ifdef __cplusplus
}
#endif
#endif
