/*
 * wgrt.h -- C ABI of the MI355X waveguide ray-tracing engine (libwgrt.so).
 *
 * Drop-in boundary for the reference's hot path, the Numba kernel call
 *
 *   process_rays_kernel_pro_fullColor[blocks, threads](
 *       x_v, y_v, gap_x_v, gap_y_v, pol_v, azi_v, m_v, n_v, lmd_num, te_v, tm_v, delta_phase_v,
 *       rng_states, IC, FC, FC_offset, OC, OC_offset, n_g,
 *       eff_reg1, eff_reg2, eff_reg_FOV, eff_reg_FOV_range,
 *       lut_ic1, lut_ic2, lut_ic3, lut_fc1, lut_fc2, lut_oc1, lut_oc2, lut_TIR, lut_gap, matrix_EB)
 *
 * (reference GPU_ray_tracing_functions.py:833-841, launched at
 * gpu_ray_tracing_pro_fullColor.py:169-177).  The 33 arguments split into
 *   - the scene (geometry + LUTs, 19 arguments, constant across launches):
 *       wgrt_scene_create()  -- replaces the cuda.to_device uploads at MAIN:40-57
 *   - the per-launch ray batch, RNG state and eyebox grid (14 arguments):
 *       wgrt_trace_fullcolor() -- replaces one kernel launch (MAIN:170)
 *
 * Conventions (same as the reference's): the caller owns every buffer; the
 * trace call allocates nothing, accumulates into matrix_EB (never zeroes it),
 * mutates rng_states, leaves the ray arrays untouched, and is asynchronous on
 * the given HIP stream (the caller synchronises, MAIN:178).  Differences: every
 * entry point validates its arguments and returns a wgrt_status instead of
 * silently corrupting memory; out-of-range m / n / lmd_num rays are skipped
 * and counted (wgrt_trace_stats.bad_rays) rather than read out of bounds.
 *
 * All pointers passed to wgrt_trace_* are DEVICE pointers (hipMalloc'd or torch
 * ROCm tensors); all pointers in wgrt_scene_desc are HOST pointers.
 *
 * Devices: a scene lives on the HIP device it was created on.  Every entry point
 * that takes a scene allocates and launches on that device, and every entry point
 * leaves the calling thread's current device (hipGetDevice) as it found it, so one
 * host thread may drive scenes on several GPUs.  wgrt_rays_init and
 * wgrt_selftest_math launch on their stream's device (the current one for the null
 * stream).  A stream passed with a scene must belong to the scene's device.
 */
#ifndef WGRT_H
#define WGRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WGRT_ABI_VERSION 7

typedef enum {
    WGRT_OK = 0,
    WGRT_ERR_INVALID_ARGUMENT = 1,
    WGRT_ERR_HIP = 2,
    WGRT_ERR_OUT_OF_MEMORY = 3,
    WGRT_ERR_UNSUPPORTED = 4,
} wgrt_status;

/* Geometry + look-up tables, exactly the arrays couplers_coor_full_color() and the
 * seven lut_*_fullColor.npy files provide (reference couplers_coor.py:740-750,
 * gpu_ray_tracing_pro_fullColor.py:19-34).  Host pointers, C-contiguous. */
typedef struct {
    const double *IC;                 /* [n_ic, 2]                                   */
    int64_t n_ic;
    const double *FC;                 /* [FC_offset[n_fc_slices], 2]                  */
    const int64_t *FC_offset;         /* [n_fc_slices + 1]                            */
    int64_t n_fc_slices;
    const double *OC;                 /* [OC_offset[n_oc_slices], 2]                  */
    const int64_t *OC_offset;         /* [n_oc_slices + 1]                            */
    int64_t n_oc_slices;
    double n_g;                       /* substrate index                              */
    const double *eff_reg1;           /* [n_eff_reg1, 2] whole effective region       */
    int64_t n_eff_reg1;
    const double *eff_reg2;           /* [n_eff_reg2, 2] IC+FC effective region       */
    int64_t n_eff_reg2;
    const double *eff_reg_FOV;        /* [nx, ny, 4, 2] per-FoV eyebox rectangle      */
    const double *eff_reg_FOV_range;  /* [nx, ny, 4] = xmin, xmax, ymin, ymax         */
    /* complex128 tables, interleaved (re, im); channel counts ch5 (>= 41), ch3 (>= 20) */
    const double *lut_ic1, *lut_ic2, *lut_ic3;   /* [num_lmd, nx, ny, ch5]              */
    const double *lut_fc1, *lut_fc2;             /* [n_fc_slices, num_lmd, nx, ny, ch3] */
    const double *lut_oc1, *lut_oc2;             /* [n_oc_slices, num_lmd, nx, ny, ch5] */
    int32_t ch5, ch3;
    const double *lut_TIR;            /* [num_lmd, nx, ny, 4]                         */
    const double *lut_gap;            /* [num_lmd, nx, ny, 8]                         */
    int32_t num_lmd, nx, ny;
} wgrt_scene_desc;

typedef struct wgrt_scene wgrt_scene;   /* opaque, device-resident */

/* The twelve per-ray float32 columns of the reference (MAIN:65-76), device pointers.
 * Columns the kernel never reads (gap_x, gap_y, pol, azi: overwritten before use at
 * GRTF:872-894) may be NULL. */
typedef struct {
    const float *x, *y, *gap_x, *gap_y, *pol, *azi, *m, *n, *lmd_num, *te, *tm, *delta_phase;
} wgrt_rays;

/* The same twelve columns as outputs (wgrt_rays_init). */
typedef struct {
    float *x, *y, *gap_x, *gap_y, *pol, *azi, *m, *n, *lmd_num, *te, *tm, *delta_phase;
} wgrt_ray_columns;

typedef struct {
    uint64_t bounces;          /* ray-bounce events: 1 in-coupling + loop iterations, per ray      */
    uint64_t bad_rays;         /* rays skipped for out-of-range m / n / lmd_num                    */
    uint64_t eyebox_hits;      /* rays accumulated into matrix_EB                                  */
    uint64_t replayed;         /* Jones-vector variants: rays abandoned on an uncertain decision and
                                  re-traced with the reference arithmetic (included in the counts above) */
    uint64_t handoff_giveups;  /* fused launches (num_iter > 1): traces given up because the previous
                                  trace of their ray never handed over within the bound of
                                  wgrt_launch_opts.num_iter.  Never in a correct
                                  run: a nonzero count means the eyebox grid and the RNG states of
                                  this call are wrong, and the Python layer raises on it.           */
    uint64_t interactions;     /* ABI 5.  Monte-Carlo interactions of the bounce loop (the iterations of
                                  GRTF:905 that draw: coupler hits in R0..R5).  The other bounces are the
                                  in-coupling events (one per traced ray, GRTF:860-904) and the iterations
                                  without a draw: miss hops, R3 -> R4 switches, terminations.          */
    uint64_t libm_rays;        /* ABI 7.  Traces decided in the ener-underflow regime: a guard product
                                  ener * e_k (GRTF:1020, 1073, 1136, ...) of a nonzero efficiency fell below
                                  2^-1000, where whether it rounds to zero -- and so the ray's path --
                                  depends on the last bits of cos / sin / atan2 (glibc vs the device libm),
                                  not on the reference's formula alone.  Such traces are decided by the
                                  reference arithmetic (the Jones-vector lane abandons them to it), and
                                  are counted here; the Python layer warns (LUTPrecisionWarning) when the
                                  count is nonzero.  0 on every BASELINE configuration. */
} wgrt_trace_stats;

typedef struct {
    int64_t tile_bytes;        /* packed per-(lambda, FoV) LUT tile                   */
    int64_t tiles;             /* num_lmd * nx * ny                                   */
    int64_t grid_cells_x, grid_cells_y;
    double grid_cell_mm;
    int64_t grid_edge_cells;   /* cells whose class needs the exact polygon test      */
    int32_t n_polygons;
    int32_t device;
    int64_t jtile_bytes;       /* Jones-vector tile per (lambda, FoV) (variants 7 / 9)  */
    int64_t nonunitary_blocks; /* ABI 7.  Interaction blocks whose taken branches' Jones matrices are not
                                  scaled-unitary (kappa^2 > 1 + 1e-6): the Jones-vector variants then run
                                  their amplification-tracked certification             */
} wgrt_scene_info;

/* Build the device-resident scene (packs LUT tiles, builds the exact polygon
 * locator) on HIP device `device`.  Replaces MAIN:40-57. */
wgrt_status wgrt_scene_create(const wgrt_scene_desc *desc, int device, wgrt_scene **out);

/* Scene build options (wgrt_scene_create uses the defaults). */
typedef struct {
    double cell_mm;   /* locator grid cell (mm); 0 = default 1/128 mm (fastest on C3) */
    int host_build;   /* 1: build the cell words and tiles on the host (the reference the device build
                         is checked against; slow); 0: on the device                              */
    int lut_f32_angles;   /* ABI 4.  Bit k set: LUT k (lut_ic1, ic2, ic3, fc1, fc2, oc1, oc2) was a
                             complex64 table in the reference's run (MAIN:28-34 loads the .npy files as
                             stored).  Compiled numba takes math.cos of a complex64 table's float32 .real
                             in single precision (GRTF:866-869 and every cos ratio after it), so the
                             scene's cosines of that table's angles are cosf of the float32 angle,
                             widened.  The coefficients themselves enter E_field_cal widened exactly, as
                             numba promotes complex64 x complex128.  0: double-precision cos (complex128).
                             ABI 5: only 0 and 0x7f (all seven tables complex64) are accepted; a mixed set
                             is WGRT_ERR_UNSUPPORTED (numba would carry the ray's angle as complex128 while a
                             complex64 table's own cosine stays float32: see wgrt_scene_create_ex). */
} wgrt_scene_opts;
wgrt_status wgrt_scene_create_ex(const wgrt_scene_desc *desc, int device, const wgrt_scene_opts *opts,
                                 wgrt_scene **out);
wgrt_status wgrt_scene_destroy(wgrt_scene *scene);
wgrt_status wgrt_scene_get_info(const wgrt_scene *scene, wgrt_scene_info *info);

/* One launch of the full-colour bounce kernel over rays [0, n_rays) whose global
 * ray index is gid_offset + i (gid seeds the zero-state RNG fix-up, GRTF:28-29, and
 * keeps results independent of sharding).  rng_states[n_rays] is read and written;
 * matrix_EB [num_lmd, ny, nx, 80, 120] float32 is accumulated into.
 *   stats:          optional DEVICE pointer to a wgrt_trace_stats that is ADDED to
 *                   (zero it yourself);
 *   per_ray_bounces: optional DEVICE uint32[n_rays] of per-ray bounce counts;
 *   stream:         hipStream_t (NULL = default stream).
 * Replaces gpu_ray_tracing_pro_fullColor.py:170 (GRTF:833-1246). */
wgrt_status wgrt_trace_fullcolor(const wgrt_scene *scene, const wgrt_rays *rays, int64_t n_rays,
                                 int64_t gid_offset, uint32_t *rng_states, float *matrix_EB,
                                 wgrt_trace_stats *stats, uint32_t *per_ray_bounces, void *stream);

/* Same as wgrt_trace_fullcolor with launch tuning: kernel variant and workgroup
 * count for the persistent variants (0 = automatic).  variant:
 *   0 auto (7 when the scene has <= 16 polygons, else 9; 1 beyond 2^32 - 1 rays);
 *   1 one ray per lane over a ceil(N / 256) x 256 grid (the reference's launch shape) with the
 *     reference's arithmetic;
 *   7 the persistent wave loop over the Jones-vector state with certified decisions, 32-bit
 *     locator cell words (<= 16 polygons, else WGRT_ERR_UNSUPPORTED);
 *   9 the same with 64-bit cell words (<= 32 polygons).
 * Variants 7 / 9 re-trace the rays whose decision they cannot certify with the reference
 * arithmetic in a second kernel on the same stream (wgrt_trace_stats.replayed counts them); the
 * first such launch on a stream allocates per-stream scratch (see wgrt_scene_reserve).  Other
 * values (the retired variants 2-6 and 8 of ABI 1) are WGRT_ERR_INVALID_ARGUMENT.  All variants
 * produce identical results. */
wgrt_status wgrt_trace_fullcolor_ex(const wgrt_scene *scene, const wgrt_rays *rays, int64_t n_rays,
                                    int64_t gid_offset, uint32_t *rng_states, float *matrix_EB,
                                    wgrt_trace_stats *stats, uint32_t *per_ray_bounces, void *stream,
                                    int variant, int workgroups);

/* One launch of the single-wavelength bounce kernel process_rays_kernel_pro
 * (reference GPU_ray_tracing_functions.py:419-831): the 32-argument form without the
 * lmd_num column, LUTs [nx, ny, ch] / [n_slices, nx, ny, ch] (a wgrt_scene_desc with
 * num_lmd = 1 has exactly that memory layout), matrix_EB [ny, nx, 80, 120], and the
 * R2..R5 branch guard ener * efficiency > 1e-15 (GRTF:444) instead of > 0.
 * rays->lmd_num is ignored and may be NULL.  WGRT_ERR_INVALID_ARGUMENT if the scene has
 * num_lmd != 1.  Everything else as wgrt_trace_fullcolor / _ex. */
wgrt_status wgrt_trace_single(const wgrt_scene *scene, const wgrt_rays *rays, int64_t n_rays, int64_t gid_offset,
                              uint32_t *rng_states, float *matrix_EB, wgrt_trace_stats *stats,
                              uint32_t *per_ray_bounces, void *stream);
wgrt_status wgrt_trace_single_ex(const wgrt_scene *scene, const wgrt_rays *rays, int64_t n_rays,
                                 int64_t gid_offset, uint32_t *rng_states, float *matrix_EB,
                                 wgrt_trace_stats *stats, uint32_t *per_ray_bounces, void *stream, int variant,
                                 int workgroups);

/* Launch options for wgrt_trace_opts. */
typedef struct wgrt_debug_opts wgrt_debug_opts;   /* include/wgrt_debug.h (test / profiling hooks) */
typedef struct {
    int kernel;          /* 0 process_rays_kernel_pro_fullColor, 1 process_rays_kernel_pro (single lambda) */
    int variant;         /* as wgrt_trace_fullcolor_ex (0 auto)                                           */
    int workgroups;      /* persistent variants: resident workgroups (0 auto)                             */
    /* Persistent variants: order in which the 64-ray chunks [64 c, 64 c + 64) are handed to
     * the waves -- a DEVICE int32 permutation of 0 .. ceil(n_rays / 64) - 1, or NULL for
     * ascending order.  Results do not depend on it (rays are independent).  The permutation
     * is not validated on the device. */
    const int32_t *chunk_order;
    int64_t n_chunk_order;
    /* Chained traces per call (0 or 1: one).  num_iter = K gives exactly the results of K
     * successive launches over the same rays (the reference's num_iter loop, MAIN:169-177):
     * every ray is traced K times, each trace starting from the RNG state the previous one
     * left, all out-couplings binned into matrix_EB, rng_states left at the last trace's
     * states, stats summed over the K traces.  Variants 7-9 run the K traces in ONE
     * persistent launch (one iteration's straggler tail overlaps the next one's bulk);
     * the others issue K launches.  1 <= num_iter <= 255; num_iter > 1 needs
     * per_ray_bounces == NULL and chunk_order == NULL. */
    int num_iter;
    /* Global ray ids of a shard made of several FoV x wavelength block ranges (multi-GPU
     * interleaved sharding): when gid_blocks (DEVICE int64[ceil(n_rays / gid_block_rays)]) is
     * non-NULL, local ray i has global id gid_blocks[i / gid_block_rays] + i % gid_block_rays
     * and the call's gid_offset must be 0; NULL: global id gid_offset + i.  The global id seeds
     * the zero-state RNG fix-up (GRTF:28-29) and nothing else, so results equal a single trace
     * of the whole batch whatever the assignment. */
    const int64_t *gid_blocks;
    int64_t gid_block_rays;
    const wgrt_debug_opts *debug;   /* NULL in production (include/wgrt_debug.h) */
    /* ABI 5.  Single traces (num_iter <= 1) with workgroups == 0: the persistent grid is
     * ceil(grid_sqrt_k * sqrt(work items)) workgroups, at most the resident grid (a single trace
     * ends with the drain of its longest ray chains, which run faster on a less crowded chip;
     * DESIGN.md §5.4).  0 = the default 6.5; a negative value = the resident grid. */
    double grid_sqrt_k;
} wgrt_launch_opts;

/* One launch of either bounce kernel with launch options (everything else as
 * wgrt_trace_fullcolor / wgrt_trace_single). */
wgrt_status wgrt_trace_opts(const wgrt_scene *scene, const wgrt_rays *rays, int64_t n_rays, int64_t gid_offset,
                            uint32_t *rng_states, float *matrix_EB, wgrt_trace_stats *stats,
                            uint32_t *per_ray_bounces, void *stream, const wgrt_launch_opts *opts);

/* Pre-allocates the launch scratch the Jones-vector variants (7-9) use on `stream` for
 * launches of up to n_rays rays x num_iter chained traces (work-queue heads, replay list,
 * out-coupling queue, fused-launch hand-off words), so that no later launch within those
 * sizes allocates or synchronises.  Optional: a launch grows the scratch itself.  Not part
 * of the reference (its launches allocate nothing on the device). */
wgrt_status wgrt_scene_reserve(const wgrt_scene *scene, int64_t n_rays, int num_iter, void *stream);

/* Device-side ray setup (replaces the host loop MAIN:59-115 and the seeding at MAIN:158):
 * fills FoV x wavelength blocks [block_lo, block_hi) of the batch -- block b =
 * (ii * ny + jj) * n_lambdas + k, rays [b * R, (b + 1) * R) -- into DEVICE columns of
 * (block_hi - block_lo) * R floats, i.e. one rank's shard at local index 0:
 *   x, y = points[r] (first R/2 rays, TE: te 1, tm 0) / points[r - R/2] (TM: te 0, tm 1),
 *   m = ii, n = jj, lmd_num = lambdas[k] (HOST int32[n_lambdas], n_lambdas <= 8;
 *   MAIN uses 0..2), gap_x = gap_y = pol = azi = delta_phase = 0.
 * points: DEVICE float64 [R / 2, 2] (generate_points_in_polygon, GRTF:12-23), rounded to
 * float32 as numpy assignment does.  Odd R: the last ray of each block is all-zero, as in
 * MAIN.  rng_states (optional, DEVICE uint32) = 0x9E3779B9 * (gid + 1) with global gid =
 * block_lo * R + i.  Any column may be NULL (not written).  Asynchronous on stream. */
wgrt_status wgrt_rays_init(const double *points, int64_t rays_per_fov, int32_t nx, int32_t ny,
                           const int32_t *lambdas, int32_t n_lambdas, int64_t block_lo, int64_t block_hi,
                           const wgrt_ray_columns *out, uint32_t *rng_states, void *stream);

/* Multi-GPU eyebox collection (the strong-scaling gather of distributed.EyeboxGather; the reference
 * runs one GPU and accumulates matrix_EB in place, MAIN:167-178).  Each rank traces its own FoV x
 * wavelength blocks, so it owns whole (lambda, n, m) slabs of 80 x 120 floats of matrix_EB, plus -- by
 * the compiled-numba aliasing of an out-coupling exactly on the eyebox's top edge (GRTF:154-165) -- the
 * first WGRT_EB_SPILL floats of the slab after an owned one.  A rank's payload is one flat float
 * buffer of wgrt_eyebox_payload_floats(nb) floats: nb slab rows of WGRT_EB_SLAB floats, then nb spill
 * rows of WGRT_EB_SPILL floats (16-B aligned: the spill part is padded to 4 floats).
 *   pack:     row j (j < n) <- slab slabs[j]; spill row j <- the first WGRT_EB_SPILL floats of slab
 *             next[j], times spill_mask[j] (0 or 1); rows n .. nb-1 untouched.
 *   assemble: eb slab dst[r * nb + j] <- slab row j of rank r's payload (recv + r * payload floats),
 *             for every dst >= 0; then the spill rows with spill_dst[r * nb + j] >= 0 are ADDED to the
 *             first WGRT_EB_SPILL floats of that slab (after every copy).  Slabs no dst names are left
 *             as they are.
 * Every pointer is DEVICE memory (slabs / next / dst / spill_dst int64, spill_mask float); both
 * launch on `stream` (its device) and are asynchronous.  Not part of the reference. */
#define WGRT_EB_SLAB 9600
#define WGRT_EB_SPILL 121
int64_t wgrt_eyebox_payload_floats(int64_t nb);
wgrt_status wgrt_eyebox_pack(const float *eb, int64_t n_slabs, const int64_t *slabs, const int64_t *next,
                             const float *spill_mask, int64_t n, int64_t nb, float *payload, void *stream);
wgrt_status wgrt_eyebox_assemble(float *eb, int64_t n_slabs, const float *recv, int32_t world, int64_t nb,
                                 const int64_t *dst, const int64_t *spill_dst, void *stream);

/* Polygon membership of n points (DEVICE xy[n, 2]) through the scene's locator:
 * bit k of out_mask[i] = is_inside_or_on_edge(point i, polygon k) with polygon order
 * 0 eff_reg1, 1 eff_reg2, 2 IC, 3.. FC slices, then OC slices (GRTF:63-71).  Bit 63 is set
 * if the two exact fallbacks the kernels use (CSR row lists, 128-B band records) disagreed
 * for any polygon.  Test hook. */
wgrt_status wgrt_scene_classify(const wgrt_scene *scene, const double *xy, int64_t n,
                                uint64_t *out_mask, void *stream);

/* Host-only replica of the locator (no GPU needed; test hook): builds the scene's
 * locator with cell size cell_mm and classifies n HOST points exactly as the kernels do. */
wgrt_status wgrt_locator_classify_host(const wgrt_scene_desc *desc, double cell_mm, const double *xy, int64_t n,
                                       uint64_t *out_mask);

/* The test / profiling hooks (certification shadow, scene copies, wave timeline, launch
 * overrides) are declared in include/wgrt_debug.h. */

/* Device math self-test (test hook): for i < n, out[k * n + i] holds
 * k=0 sqrt(a), 1 a / b, 2 hypot_cr(a, b), 3 atan2(a, b), 4 sin(a), 5 cos(a), 6 wrap(a). */
wgrt_status wgrt_selftest_math(const double *a, const double *b, int64_t n, double *out, void *stream);

const char *wgrt_status_string(wgrt_status s);
const char *wgrt_last_error(void);   /* detail of the last failure on this thread */
int wgrt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* WGRT_H */
