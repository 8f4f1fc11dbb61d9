/*
 * wgrt_debug.h -- test and profiling hooks of libwgrt.so (not part of the drop-in boundary).
 *
 * Nothing here is process-wide state: every hook is either a separate entry point or a
 * per-call option block (wgrt_launch_opts.debug), so these hooks are as thread-safe as the
 * calls they ride on.  The production path passes debug = NULL and runs instantiations of the
 * kernels that contain none of this code (the wave timeline is a template parameter of the
 * persistent kernel, off in the product instantiation).
 */
#ifndef WGRT_DEBUG_H
#define WGRT_DEBUG_H

#include "wgrt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Per-call overrides of a Jones-vector launch (wgrt_launch_opts.debug). */
struct wgrt_debug_opts {
    /* Base of the double-precision certification bound (0: default 1e-10) and of the
     * single-precision estimate's (0: default 8e-6; the effective value is max(this, cert_tol)).
     * Larger values make more decisions uncertain (more double-precision re-evaluations, more
     * rays through the replay kernel); results unchanged. */
    double cert_tol;
    double cert_tol32;
    /* Rays per work-queue item (0: 64; at most 64: an item is staged one ray per lane).
     * Smaller items make a refill span several items; results unchanged. */
    int chunk_rays;
    /* Wave timeline: when non-NULL, the launch runs the instrumented instantiation and records,
     * per wave w < timeline_waves of its grid, 8 words at timeline[8 w ..]: start,
     * queue-exhausted and end times (s_memrealtime, 100 MHz), passes of the wave loop,
     * lane-passes with a ray in flight, XCD id, and the passes and lane-passes before the
     * queue ran dry (DEVICE buffer). */
    unsigned long long *timeline;
    int64_t timeline_waves;
    /* Fault injection: 1 makes the call return WGRT_ERR_HIP right after the trace kernel is
     * enqueued, before the epilogue kernel (the recovery path of a launch that fails half-way;
     * the next call on the stream must still be exact). */
    int fail_after_trace;
    /* Fused launches: hand-off wait bound in s_memrealtime ticks (100 MHz); 0 = the default
     * derived from num_iter.  A tiny bound makes waiting traces give up
     * (counted in wgrt_trace_stats.handoff_giveups).  Without it, a trace is given up only once the
     * default bound has passed AND the waiting wave has run 4096 passes since the wait began (a wave
     * that was descheduled does not give up a correct hand-off); a given-up ray is marked abandoned,
     * so its later traces in the call skip it instead of waiting again. */
    uint64_t handoff_wait_ticks;
};

/* Certification shadow of the Jones-vector variants (diagnostic; wgrt_shadow.hip).  Traces rays
 * [0, n_rays) with the reference's own arithmetic (unwrapped delta_phase, hypot / atan2 / wrap,
 * GRTF:132-152 and 905-1246) and, at every Monte-Carlo decision, evaluates the Jones-vector lane's
 * thresholds and certification bound tol (default bases) on the same state.  rng_states (DEVICE,
 * in/out) and the optional per_ray_bounces follow the reference's path, so they equal one launch
 * of the exact kernel; matrix_EB is not written.  stats: DEVICE pointer, ADDED to (zero it
 * yourself); max fields are max-combined.  single: the single-wavelength kernel (threshold 1e-15). */
typedef struct {
    uint64_t decisions;          /* Monte-Carlo decisions evaluated                                 */
    uint64_t uncertain;          /* decisions the Jones lane cannot certify (its rays are replayed)   */
    uint64_t silent_flips;       /* certified Jones decisions that differ from the reference's: 0    */
    uint64_t bounces;            /* ray-bounce events traced                                          */
    uint64_t fallbacks;          /* decisions the single-precision estimate leaves to the double one  */
    double max_ratio;            /* max over decisions / thresholds of |c_jones64 - c_ref| / tol64    */
    double max_ratio32;          /* the same for the single-precision estimate against tol32          */
    double max_ratio_by_depth[6];   /* max_ratio32 by bounce depth [1,10) [10,30) [30,100) [100,300)
                                       [300,1000) [1000,inf)                                          */
    uint64_t decisions_by_depth[6];
    uint64_t ratio_hist[20];     /* decisions by log10 of their ratio32: bucket b = [1e(b-18),
                                    1e(b-17)); bucket 0 also holds smaller ratios, 19 larger ones    */
    double max_ener_ratio;       /* single wavelength: max |ener_jones / ener_ref - 1| / tracked bound */
    double max_amp;              /* the largest amplification bound a Jones lane carried (JRay::amp; 1 on
                                    scaled-unitary LUTs) */
} wgrt_shadow_stats;

wgrt_status wgrt_debug_shadow(const wgrt_scene *scene, const wgrt_rays *rays, int64_t n_rays, int64_t gid_offset,
                              int single, uint32_t *rng_states, uint32_t *per_ray_bounces, wgrt_shadow_stats *stats,
                              void *stream);

/* Copies one of a scene's device structures to host memory dst (bytes must equal its size):
 * which = 0 the locator cell words (uint64, ncx * ncy), 1 the exact lane's tiles, 2 the
 * Jones-vector tiles (doubles, tiles * tile / jtile doubles; wgrt_scene_info). */
wgrt_status wgrt_debug_scene_copy(const wgrt_scene *scene, int which, void *dst, int64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* WGRT_DEBUG_H */
