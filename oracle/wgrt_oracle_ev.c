/* wgrt_oracle_ev.c -- TEST INFRASTRUCTURE ONLY: the CPU oracle (wgrt_oracle.c, the reference's FSM,
 * GPU_ray_tracing_functions.py:833-1246 / 419-831) compiled with an event hook that counts the
 * Monte-Carlo draws of the bounce loop: ORACLE_EV(0, region, ...) marks every draw, region 9 the
 * in-coupling event's (GRTF:860-869) -- so draws in regions 0..5 are the coupler interactions of the
 * loop iterations (GRTF:908-1246), the count the product kernels report as
 * wgrt_trace_stats.interactions.  Same arithmetic and outputs as libwgrt_oracle.so; a separate
 * library (oracle/build/libwgrt_oracle_ev.so) so the checker the parity tests use stays hook-free. */
#include <stdint.h>

static int64_t oracle_ev_draws;   /* OpenMP threads add with relaxed atomics */

#define ORACLE_EV(ev, region, x, y, gx, gy)                                        \
    do {                                                                           \
        if ((ev) == 0 && (region) != 9) __atomic_fetch_add(&oracle_ev_draws, 1, __ATOMIC_RELAXED); \
    } while (0)

#include "wgrt_oracle.c"

/* Interactions counted since the last reset (reset != 0: zero the count after reading it). */
int64_t wgrt_oracle_ev_interactions(int reset) {
    return reset ? __atomic_exchange_n(&oracle_ev_draws, 0, __ATOMIC_RELAXED)
                 : __atomic_load_n(&oracle_ev_draws, __ATOMIC_RELAXED);
}
