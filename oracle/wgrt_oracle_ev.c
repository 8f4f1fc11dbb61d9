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

/* ... and the rays whose trace enters the ener-underflow regime: a guard product ener * e below
 * 2^-1000, i.e. next to the subnormal range, where whether it rounds to zero (and fails the full-colour
 * guard ener * e > 0, GRTF:1020) hangs on the last bits of e -- of the libm's cos / sin / atan2.  Such a
 * ray's path is not determined by the reference's formula alone: a one-ulp change of atan2 or cos moves
 * it (tests/test_gpu_certification.py). */
static __thread int oracle_ev_underflow;
static uint8_t *oracle_ev_flags;

#define ORACLE_ENER(en)                                          \
    do {                                                         \
        if ((en) < 0x1p-1000) oracle_ev_underflow = 1;           \
    } while (0)
#define ORACLE_RAY_BEGIN(i) (oracle_ev_underflow = 0)
#define ORACLE_RAY_END(i)                                        \
    do {                                                         \
        if (oracle_ev_flags) oracle_ev_flags[i] = (uint8_t)oracle_ev_underflow; \
    } while (0)

#include "wgrt_oracle.c"

/* Per-ray underflow flags of the next traces go to flags[n_rays] (NULL: not recorded). */
void wgrt_oracle_ev_set_flags(uint8_t *flags) { oracle_ev_flags = flags; }

/* Interactions counted since the last reset (reset != 0: zero the count after reading it). */
int64_t wgrt_oracle_ev_interactions(int reset) {
    return reset ? __atomic_exchange_n(&oracle_ev_draws, 0, __ATOMIC_RELAXED)
                 : __atomic_load_n(&oracle_ev_draws, __ATOMIC_RELAXED);
}
