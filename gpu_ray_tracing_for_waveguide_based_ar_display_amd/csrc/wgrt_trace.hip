// wgrt_trace.hip -- CDNA4 (gfx950) kernels of the waveguide Monte-Carlo bounce loop
// and the C ABI declared in include/wgrt.h.
//
// Restates the reference's full-colour kernel process_rays_kernel_pro_fullColor
// (GPU_ray_tracing_functions.py = GRTF:833-1246, call at gpu_ray_tracing_pro_fullColor.py:170)
// and its single-wavelength twin process_rays_kernel_pro (GRTF:419-831).  One ray per lane
// (wave64); the ray record lives in VGPRs for its whole life; the only global writes are the
// final RNG state, optional per-ray bounce counts, one float atomic per eyebox hit (GRTF:164)
// and one set of 64-bit stats atomics per wave.
//
// Two lanes implement the reference's per-ray state machine (R0..R5):
//   * the exact lane (variant 1, the replay kernel, the diagnostic shadow): the reference's
//     float64 arithmetic in its expression order (E_field_cal with correctly rounded hypot,
//     GRTF:132-152), compiled with -ffp-contract=off;
//   * the Jones-vector lane (variants 7 / 9, the product path): the same decisions from the
//     field carried as a complex Jones vector, each certified against a bound on the
//     difference to the exact arithmetic; an uncertain decision abandons the ray, which the
//     replay kernel re-traces with the exact lane.
// Polygon membership goes through the exact grid locator (wgrt_scene_build.cpp).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <atomic>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wgrt.h"
#include "../../include/wgrt_debug.h"
#include "wgrt_common.h"
#include "wgrt_device.h"
#include "wgrt_scene.h"
#include "wgrt_scene_build.h"

using namespace wgrt;

namespace wgrt {
thread_local std::string g_last_error;
wgrt_status fail(wgrt_status s, const std::string &msg) {
    g_last_error = msg;
    return s;
}
}  // namespace wgrt

namespace {

// Cell size (mm) of the global-memory locator grid (wgrt_scene_opts.cell_mm = 0): 1/128 mm, a 71 MB
// grid at C3; fewer EDGE-cell exact tests than coarser grids (fastest on C3).
#ifndef WGRT_CELL_MM
#define WGRT_CELL_MM 0.0078125
#endif
constexpr double kDefaultCellMm = WGRT_CELL_MM;


#define DEVICE_SCOPE(name, dev)                                                                      \
    DeviceScope name(dev);                                                                          \
    if (name.error() != hipSuccess)                                                                 \
        return fail(WGRT_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(name.error()))

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(WGRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

// Variant 1: one ray per lane over a 1-D grid (the reference's launch shape, MAIN:167).
__global__ __launch_bounds__(256) void trace_grid_kernel(TraceArgs A) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t b = 0, h = 0, bad = 0, ni = 0, lm = 0;
    if (i < A.n_rays) trace_one(A, i, b, h, bad, nullptr, &ni, &lm);
    add_stats(A.stats, b, h, bad, ni, lm);
}

// Launch scratch counters of the Jones-vector variants: kHeads work-queue heads, then the replay
// count, the out-coupling queue and full-block counts, and a single launch's epilogue totals and done
// count, each on its own 128-B line.
constexpr int kHeadStride = 16;   // unsigned long longs between heads (128 B)
constexpr int kHeads = 8;
constexpr int kScratchCtr = (kHeads + 5) * kHeadStride;   // heads, replay / queue / full-block counts, epilogue totals / done

// Single launches do their epilogue in the trace kernel (fused launches keep epilogue_kernel, whose
// replays chain the traces after an abandoned one): every wave bins the out-coupling blocks it filled
// when it ends (a chain of block links, its own stores), every workgroup adds its counter totals with
// agent-scope atomics and counts itself done, and the workgroup that counts last adds the totals to
// *stats, zeroes the next launch's counter set and re-traces the abandoned rays (an inlined trace_one
// whose arguments are read from the kernarg segment there: replay_tail; none in practice).  A non-inlined
// trace_one call gave the wave loop 128 VGPRs and 536 B of scratch per lane and lost 14-27 %; the
// inlined one costs SGPR spills outside the loop only (round 6).  WGRT_INKERNEL_EPI=0 builds the
// epilogue-kernel design for single launches too.
//
// The hand-off to the last workgroup is MI355X_MICROARCH.md's measured form "one lane of each storing
// workgroup signals with an agent-scope atomic add after every storing wave's vmcnt(0) wait; the
// workgroup whose add came last loads with sc1 (agent-scope) loads": the totals are agent-scope atomics,
// the replay-list entries agent-scope stores each waited for by its lane, and the last workgroup reads
// both with agent-scope loads.  A release / acquire pair on the done count would add an L2 write-back
// and an L1 invalidate per workgroup (the guide prices them at ~1.7 us each), so the order rests on the
// explicit s_waitcnt vmcnt(0), which on gfx950 covers stores and no-return atomics (GFX9 has no
// separate store counter; this file targets gfx950 only).
#ifndef WGRT_INKERNEL_EPI
#define WGRT_INKERNEL_EPI 1
#endif
constexpr bool kInKernelEpilogue = WGRT_INKERNEL_EPI != 0;

// Runs right behind every fused Jones-vector launch on its stream (and every single launch built with
// WGRT_INKERNEL_EPI=0) -- the launch's only other kernel:
//  1. bins the out-coupling queue blocks the trace waves filled (a wave bins the block it holds
//     when it leaves; cells count hits, +1.0f, so the binning order does not matter);
//  2. re-traces the rays the launch abandoned (uncertain decisions; nothing of them was written)
//     from their launch-start state with the reference arithmetic (usually none);
//  3. adds the counters to *stats: workgroup 0 sums the trace kernel's per-workgroup partials,
//     any workgroup with replay or binning work adds its own (rare, so the atomics are not
//     contended);
//  4. zeroes the other counter set, which the next launch on the stream uses (this launch's set
//     is still being read by the other workgroups; the launch after next finds it zeroed).
constexpr int kEpilogueGroups = 256;
#ifndef WGRT_QBLOCK
#define WGRT_QBLOCK 32
#endif
constexpr int kQBlock = WGRT_QBLOCK;    // out-coupling queue slots a wave reserves at a time (a C3 wave
                               // out-couples ~10 rays per trace)
static_assert(kQBlock >= 1 && kQBlock <= 64, "a queue block is binned by one lane per entry");

__global__ __launch_bounds__(256) void epilogue_kernel(TraceArgs A) {
    __shared__ unsigned long long red[4][6];
    const unsigned long long nr = *A.replay_count, nf = *A.full_count;
    const unsigned long long tid = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long nth = (unsigned long long)gridDim.x * blockDim.x;
    uint64_t h = 0, b = 0, bad = 0, gu = 0, ni = 0, lm = 0;
    for (unsigned long long e = tid; e < nf * kQBlock; e += nth) {
        {
            const unsigned long long j = (unsigned long long)A.full_list[e / kQBlock] * kQBlock + e % kQBlock;
            const uint32_t g = A.q_i[j];   // tile index (lambda * nx + m) * ny + n
            const double2 p = A.q_xy[j];
            const int n = (int)(g % (uint32_t)A.ny), m = (int)(g / (uint32_t)A.ny % (uint32_t)A.nx);
            const int l = (int)(g / ((uint32_t)A.ny * (uint32_t)A.nx));
            h += eyebox_add(A, l, m, n, p.x, p.y);
        }
    }
    for (unsigned long long k = tid; k < nr; k += nth) {
        const int64_t i = (int64_t)A.replay_list[k];
        if (A.n_iter <= 1) {
            trace_one(A, i, b, h, bad, nullptr, &ni, &lm);
        } else {   // fused launch: the traces from the abandoned one to the last, chained
            const uint64_t w = A.rng64[i];
            uint32_t st = (uint32_t)(w >> 32);
            for (int it = (int)(w & 0xffu); it < A.n_iter; ++it) trace_one(A, i, b, h, bad, &st, &ni, &lm);
            A.rng[i] = st;
        }
    }
    if (blockIdx.x == 0) {
        for (int k = threadIdx.x; k < A.n_trace_waves; k += blockDim.x) {
            const unsigned long long *slot = A.part + kPartWords * (size_t)k;
            b += slot[0];
            bad += slot[1];
            h += slot[2];
            gu += slot[3];
            ni += slot[4];
        }
        if (threadIdx.x < kScratchCtr) A.other_ctr[threadIdx.x] = 0ull;
    }
    const int w = threadIdx.x >> 6;
    b = wave_sum(b);
    bad = wave_sum(bad);
    h = wave_sum(h);
    gu = wave_sum(gu);
    ni = wave_sum(ni);
    lm = wave_sum(lm);
    if ((threadIdx.x & 63) == 0) {
        red[w][0] = b;
        red[w][1] = bad;
        red[w][2] = h;
        red[w][3] = gu;
        red[w][4] = ni;
        red[w][5] = lm;
    }
    __syncthreads();
    if (threadIdx.x == 0 && A.stats) {
        wgrt_trace_stats *st = A.stats;
        const unsigned long long t0 = red[0][0] + red[1][0] + red[2][0] + red[3][0];
        const unsigned long long t1 = red[0][1] + red[1][1] + red[2][1] + red[3][1];
        const unsigned long long t2 = red[0][2] + red[1][2] + red[2][2] + red[3][2];
        const unsigned long long t3 = red[0][3] + red[1][3] + red[2][3] + red[3][3];
        const unsigned long long t4 = red[0][4] + red[1][4] + red[2][4] + red[3][4];
        const unsigned long long t5 = red[0][5] + red[1][5] + red[2][5] + red[3][5];
        if (t4) atomicAdd((unsigned long long *)&st->interactions, t4);
        if (t5) atomicAdd((unsigned long long *)&st->libm_rays, t5);
        if (t0) atomicAdd((unsigned long long *)&st->bounces, t0);
        if (t1) atomicAdd((unsigned long long *)&st->bad_rays, t1);
        if (t2) atomicAdd((unsigned long long *)&st->eyebox_hits, t2);
        if (t3) atomicAdd((unsigned long long *)&st->handoff_giveups, t3);
        if (blockIdx.x == 0 && nr) atomicAdd((unsigned long long *)&st->replayed, nr);
    }
}

// Work queue of the Jones-vector variants: one head per XCD (each on its own 128-B line), head
// x handing out the stripes s = x, x + 8, ... of kStripe consecutive chunks, in order, so a
// die's waves share its stripes' FoV x wavelength tiles in that XCD's L2 and the dequeue atomics
// spread over 8 addresses; a wave whose head runs dry moves on to the next head.  The XCD id
// steers placement only: any wave may take any chunk, so correctness never depends on it.
constexpr int kFusedRefill = 16;

#ifndef WGRT_STRIPE
#define WGRT_STRIPE 16
#endif
constexpr int64_t kStripe = WGRT_STRIPE;
// -DWGRT_SEG=2: wave-uniform segment marks at the top level of a pass (tools/segments.py)
#if defined(WGRT_SEG) && WGRT_SEG == 2
#define SEG_TMARK(sg, k, dep) SEG_MARK_DEP(sg, k, dep)
#else
#define SEG_TMARK(sg, k, dep) ((void)0)
#endif

// Compiler-visible waits (round 6).  A pass already waits for every load in flight before
// advance() reads the cell word; stating that wait with the builtin at the top of the pass (and the staging
// wait, and one at the exit of the rare EDGE test in advance(), wgrt_device.h WGRT_EDGE_WAIT) tells the
// compiler's wait insertion that nothing older is pending.  Without them it merged, over the rare paths,
// loads it could not prove landed, and so waited for everything in flight -- the pass's miss-hop gathers
// among them -- before the interaction could issue its line-0 loads: -0.3 to -2.6 % per single launch.
#ifndef WGRT_MAIN_TOPWAIT
#define WGRT_MAIN_TOPWAIT 1
#endif
#ifndef WGRT_TAIL_TOPWAIT
#define WGRT_TAIL_TOPWAIT 1
#endif
#ifndef WGRT_ONE_RETIRE
#define WGRT_ONE_RETIRE 1
#endif
constexpr bool kOneRetire = WGRT_ONE_RETIRE != 0;   // one retire site per pass (single launches)   // chunks per stripe of the work queue (1024 rays: one C3 tile)

// How long a fused-launch lane may wait for its ray's previous trace before it gives the trace
// up (wgrt_trace_stats.handoff_giveups; the Python layer raises on it).  A legitimate wait for
// trace k of ray i ends once trace k - 1 of ray i has ended.  Item (k - 1, c) was dequeued from the
// same head before (k, c) (heads hand out iteration-major), and the wave holding it starts the
// ray within the lifetime of the rays on its lanes, then traces it: each at most kMaxLoop + 1
// bounces = passes of that wave, and that wave's lanes may themselves wait on iteration k - 2.
// With a pass at most ~5 us (bulk C3 passes take 5.8 us / 64 lanes of 4 waves per SIMD, a
// lone wave's about 3 us) one trace or one start delay is under 0.5 s, so a correct wait
// is below k * 2 * 0.5 s: the bound is 1 s per chained trace plus 1 s.  It turns a hand-off bug
// (epoch / tag) into a visible count within seconds instead of a hung GPU; it cannot be ms
// without failing legitimate 1e5-bounce rays.
constexpr unsigned long long kHandoffTicksPerIter = 100000000ull;   // s_memrealtime: 100 MHz
// ... and the waiting lane's own wave must also have run this many passes since the wait began: the
// clock runs while a wave is preempted or time-sliced (another queue, CWSR, profiler replay), its
// passes do not, so a waiter that was merely descheduled does not give a correct hand-off up
constexpr uint32_t kHandoffMinPasses = 4096;

// A wave-uniform copy of v (lane 0's value, in SGPRs): the wave loop's queue state is uniform,
// and keeping it scalar lets its branches be scalar branches instead of exec-mask juggling.
__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ int xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 7u);
}

// Tag of a fused launch's per-ray RNG word: launch epoch, broken flag, traces completed.
__device__ __forceinline__ uint32_t iter_tag(uint32_t epoch, uint32_t k, bool broken) {
    return (epoch << 9) | (broken ? 0x100u : 0u) | k;
}

// Single launches re-trace their abandoned rays inside the trace kernel (the workgroup that counts
// itself done last: replay_tail), so no replay kernel follows the launch: -0.2 to -1.6 % per single
// launch.  WGRT_INKERNEL_REPLAY=0 builds the round-5 design (replay_kernel behind it).
#ifndef WGRT_INKERNEL_REPLAY
#define WGRT_INKERNEL_REPLAY 1
#endif

// An abandoned ray (kUncertain) onto the replay list.  With the in-kernel replay the entry is stored at
// agent scope and waited for here, so it is in memory before this lane's workgroup counts itself done
// (the last workgroup reads the list at agent scope); rare, so the wait costs nothing measurable.
__device__ __forceinline__ void record_abandoned(const KArgs &K, uint32_t i) {
    uint32_t *const slot = KA(replay_list) + atomicAdd(KA(replay_count), 1ull);
#if WGRT_INKERNEL_REPLAY
    __hip_atomic_store(slot, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
    *slot = i;
#endif
}

#if WGRT_INKERNEL_REPLAY
#ifdef WGRT_REPLAY_NOINLINE
#define WGRT_REPLAY_INL __attribute__((noinline))
#else
#define WGRT_REPLAY_INL __forceinline__
#endif
// The single launch's replay inside the trace kernel (the last workgroup; wgrt_trace.hip jones_body): the
// reference-arithmetic lane (trace_one) over the replay list, its TraceArgs read from the kernarg segment
// here, so nothing of it is live across the wave loop.
__device__ WGRT_REPLAY_INL void replay_tail(const KArgs &K, unsigned long long nr) {
    TraceArgs R{};
    R.x = KA(x); R.y = KA(y); R.m = KA(m); R.n = KA(n); R.l = KA(l);
    R.te = KA(te); R.tm = KA(tm); R.dph = KA(dph);
    R.rng = KA(rng); R.eb = KA(eb); R.stats = KA(stats); R.per_ray = KA(per_ray);
    R.n_rays = KA(n_rays); R.gid_offset = KA(gid_offset);
    R.gid_blocks = KA(gid_blocks); R.gid_block_rays = KA(gid_block_rays);
    R.tiles = KA(tiles); R.tile_d = KA(tile_d);
    R.nfc = KA(nfc); R.noc = KA(noc); R.nx = KA(nx); R.ny = KA(ny); R.nl = KA(nl);
    R.n_g = KA(n_g); R.inv_n_g = KA(inv_n_g); R.threshold = KA(threshold);
    R.loc.cells = KLOC(cells); R.loc.verts = KLOC(verts); R.loc.poly_off = KLOC(poly_off);
    R.loc.row_off = KLOC(row_off); R.loc.row_edges = KLOC(row_edges); R.loc.bands = KLOC(bands);
    R.loc.x0 = KLOC(x0); R.loc.y0 = KLOC(y0); R.loc.inv_h = KLOC(inv_h); R.loc.ncx = KLOC(ncx); R.loc.ncy = KLOC(ncy);
    const uint32_t *const list = KA(replay_list);
    uint64_t b = 0, h = 0, bad = 0, ni = 0, lm = 0;
    for (unsigned long long k = threadIdx.x; k < nr; k += blockDim.x)
        trace_one(R, (int64_t)__hip_atomic_load(list + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), b, h, bad,
                  nullptr, &ni, &lm);
    add_stats(R.stats, b, h, bad, ni, lm);
    if (threadIdx.x == 0 && R.stats) atomicAdd((unsigned long long *)&R.stats->replayed, nr);
}
#endif

// The persistent loop of the Jones-vector variants.  Work items are 64-ray chunks handed out
// by the per-XCD heads.  FUSED: a launch runs A.n_iter chained traces of every ray (the
// reference's num_iter loop of launches, MAIN:169-177, each starting from the RNG state the
// previous one left): head x hands out (iteration, chunk) items iteration-major, so one
// iteration's drain overlaps the next one's bulk.  A trace of iteration k >= 1 may start only
// once the ray's trace k - 1 has ended: its end writes the 8-byte granule {state, tag} with an
// agent-scope store, and a lane that takes the ray polls that granule with agent-scope loads
// (waiting in place, lane idle, until the tag says k) -- the granule hand-off of
// MI355X_MICROARCH.md's price list, valid whatever the XCD placement.  Results are identical
// to n_iter launches: each ray's traces run in order from the same states; eyebox adds commute.
// TL: the debug wave timeline (wgrt_debug_opts.timeline); the product instantiations have TL = false
// and contain none of its code.
template <bool FUSED, bool SINGLE, bool TL, bool AMP, class Loc>
__device__ __forceinline__ void jones_body(const TraceArgs &A, const KArgs &K, const Loc &loc, unsigned long long *heads,
                                          int chunk) {
    constexpr bool EPI = !FUSED && kInKernelEpilogue;
    // single launches retire a finished trace at one place per pass, right after advance(): the rays
    // that ended in the previous pass's interaction and those advance() ends (fused launches retire at
    // once: their hand-off would wait a pass)
    constexpr bool ONE = !FUSED && kOneRetire;
    bool fin = false;
    const int lane = threadIdx.x & 63;
    const int64_t n_chunks = (A.n_rays + chunk - 1) / chunk;
    const int64_t n_iter = FUSED ? A.n_iter : 1;
    int head = xcc_id();
    // rays of the current item still to hand out (wave-uniform; 32-bit: variants 7 / 9 index < 2^32 rays,
    // so the refill's compares stay scalar)
    uint32_t cur = 0, end = 0;
    // debug timeline (TL instantiations only): per wave, start / queue exhausted / end
    // (s_memrealtime, 100 MHz), passes, lane-passes with a ray in flight, XCD, and the passes /
    // lane-passes up to the queue running dry
    unsigned long long *const tl = TL ? KA(timeline) : nullptr;
#ifdef WGRT_SEG
    constexpr int kTlWords = 16;   // diagnostic segment build: 8 timeline words + 8 segment sums per wave
#else
    constexpr int kTlWords = 8;
#endif
    const int64_t tl_wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const bool tl_on = TL && tl != nullptr && tl_wave < KA(timeline_waves) * 8 / kTlWords;
    unsigned long long tl_passes = 0, tl_lanes = 0;
    if (tl_on && lane == 0) tl[kTlWords * tl_wave] = __builtin_amdgcn_s_memrealtime();
    uint32_t cur_k = 0;               // the item's iteration
    bool exhausted = false;
    bool active = false, waiting = false, taken = false;
    JLane L;
    int blk = 0, kind = 0;
    bool entry = false;
    // per-lane totals in 32 bits: a lane's bounce total is added to the stats directly before it
    // could overflow (2^31 bounces on one lane: never in practice)
    uint32_t tot_b = 0, tot_bad = 0, tot_giveup = 0, tot_int = 0;
    unsigned long long wait_t0 = 0;    // fused: when this lane started waiting for its ray (s_memrealtime)
    uint32_t wait_passes = 0;          // ... and the wave's passes since then
    unsigned long long qbase = 0;      // this wave's block of out-coupling slots ...
    int qfill = kQBlock;               // ... and how many of them are used (none reserved yet)
    bool qblk = false;                 // a block has been reserved

    // head x's items: stripes of kStripe consecutive chunks, stripe s on head s % 8, iteration-
    // major.  Every die gets a mix of all FoVs and wavelengths -- ray lifetimes differ by tile,
    // and with one contiguous eighth of the tiles per head the die holding the long-lived tiles
    // ended the launch 60 us after the first (striping: -6 % per single launch on C3) -- while
    // a stripe's rays still share their tiles in that die's L2.
    const int64_t ns = (n_chunks + kStripe - 1) / kStripe, last = n_chunks - (ns - 1) * kStripe;
    auto decode = [&](int x, int64_t q, int64_t &c, uint32_t &k) -> bool {
        if (x >= ns) return false;
        int64_t cx = ((ns - x + kHeads - 1) / kHeads) * kStripe;
        if ((ns - 1) % kHeads == x) cx -= kStripe - last;
        if (q >= cx * n_iter) return false;
        // the item's iteration: 0 for a single trace; else q / cx (< 256) from a double quotient,
        // corrected -- no 64-bit integer division on the dequeue path
        int64_t kk = 0;
        if (FUSED) {
            kk = (int64_t)((double)q / (double)cx);
            kk -= kk * cx > q;
            kk += (kk + 1) * cx <= q;
        }
        k = (uint32_t)kk;
        const int64_t r = q - kk * cx;
        c = ((r / kStripe) * kHeads + x) * kStripe + r % kStripe;
        return true;
    };
    // this wave's two LDS buffers of staged ray columns (wgrt_device.h stage_chunk): a refill takes
    // rays of at most two chunks, the one being used up and the next
    __shared__ uint32_t stage_buf[4][2][kStageCols * 64];
    LdsU32 *const sbufs = (LdsU32 *)&stage_buf[threadIdx.x >> 6][0][0];
    // wave-uniform: the buffer of the current item, its first ray and the previous item's first
    // ray (the other buffer).  A taken lane finds its slot from its ray index: items are disjoint
    // ranges of at most 64 rays.
    int sb = 0;
    uint32_t sbase = 0, sbase_prev = 0;
    // start the trace (L.i, L.k) on this lane: active, waiting (previous trace still running) or
    // skipped (bad ray / ray already handed to the replay)
    auto start = [&]() {
        uint64_t w = 0;
        const uint32_t oc = L.i - sbase;
        const bool in_cur = oc < 64u;
        const bool ok = lane_load_staged(sbufs + (in_cur ? sb : sb ^ 1) * (kStageCols * 64),
                                         (int)(in_cur ? oc : L.i - sbase_prev), L.i, L,
                                         (FUSED && L.k > 0) ? KA(rng64) + L.i : nullptr, &w);
        waiting = false;
        active = false;
        if (__builtin_expect(!ok, 0)) {
            ++tot_bad;
            return;
        }
        if (FUSED && L.k > 0) {
            const uint32_t tag = (uint32_t)w;
            if (tag == iter_tag(A.iter_epoch, L.k, false)) {
                L.r.s = (uint32_t)(w >> 32);
            } else if ((tag >> 8) == ((A.iter_epoch << 1) | 1u)) {
                return;   // abandoned in an earlier iteration: the replay kernel finishes it
            } else {
                waiting = true;
                wait_t0 = __builtin_amdgcn_s_memrealtime();
                wait_passes = 0;
                return;
            }
        }
        L.s0 = L.r.s;
        active = true;
        blk = 0;
        kind = 0;
        entry = true;
    };
    // a trace's counters are added when it ends: an abandoned trace (kUncertain) adds nothing, and its
    // replay (replay_kernel or, fused, epilogue_kernel: trace_one) counts the whole trace once
    auto retire = [&]() {
        tot_b += L.bounces;
        tot_int += L.inter;
        if (__builtin_expect(tot_b >= 0x80000000u, 0)) {
            wgrt_trace_stats *const st = KA(stats);
            if (st) atomicAdd((unsigned long long *)&st->bounces, (unsigned long long)tot_b);
            tot_b = 0;
        }
        if (FUSED && (int64_t)L.k + 1 < n_iter) {
            const uint64_t hand = ((uint64_t)L.r.s << 32) | iter_tag(A.iter_epoch, L.k + 1, false);
            if (L.k > 0) {
                // the granule still holds what this trace started from, unless the waiter for the next
                // trace has given up and marked the ray abandoned meanwhile: the mark then stays (a
                // compare-and-swap whose result is not used: no return, no wait), so the ray's later
                // traces skip it instead of each waiting out the bound again
                uint64_t was = ((uint64_t)L.s0 << 32) | iter_tag(A.iter_epoch, L.k, false);
                __hip_atomic_compare_exchange_strong(KA(rng64) + L.i, &was, hand, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                // trace 0 read no granule (its start state is rng_states): a give-up that raced this
                // store costs the ray's next waiter one more bound before it gives up too
                __hip_atomic_store(KA(rng64) + L.i, hand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            KA(rng)[L.i] = L.r.s;
            uint32_t *const pr = KA(per_ray);
            if (!FUSED && pr) pr[L.i] = L.bounces;
        }
        active = false;
    };

    // the second half of a pass: the interaction of the lanes at one, then this pass's
    // out-couplings into the wave's block of queue slots (a contended returning atomic per pass
    // would put its latency on every pass; a new block is needed about once per hundred passes)
    // this pass's out-couplings into the wave's block of queue slots (a contended returning atomic per
    // pass would put its latency on every pass; a new block is needed about once per hundred passes)
    auto queue_out = [&](bool out) {
        const uint64_t om = __ballot(out);
        if (om != 0ull) {
            const int nout = __popcll(om), rem = kQBlock - qfill;
            const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(om >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)om, 0));
            // the entries past the current block take ceil(extra / kQBlock) new consecutive blocks, all
            // but the last of them filled by this pass (a wave can out-couple more rays at once than a
            // block holds)
            const int extra = nout - rem;
            const int nblk = extra > 0 ? (extra + kQBlock - 1) / kQBlock : 0;
            unsigned long long nb = 0;
            if (nblk) {
                if (lane == 0) nb = atomicAdd(KA(q_count), (unsigned long long)nblk * kQBlock);
                nb = uni64(__shfl(nb, 0));
            }
            if (out) {   // entry: out-coupling position and the ray's (lambda, m, n) tile index
                const unsigned long long j = rank < rem ? qbase + qfill + rank : nb + (rank - rem);
                KA(q_xy)[j] = double2{L.r.x, L.r.y};
                KA(q_i)[j] = L.tix;
            }
            if (nblk) {
                const uint32_t b0 = (uint32_t)(nb / kQBlock), old = (uint32_t)(qbase / kQBlock);
                if (EPI) {
                    // new block k links to the block this wave filled before it (+1; 0: none): the wave
                    // walks the chain back when it ends and bins every block it filled
                    if (lane < nblk) KA(full_list)[b0 + lane] = lane > 0 ? b0 + lane : (qblk ? old + 1u : 0u);
                } else {
                    // the filled blocks -- the old one, and every new one but the last -- go to the epilogue
                    const int nfull = (qblk ? 1 : 0) + nblk - 1;
                    if (lane < nfull)
                        KA(full_list)[atomicAdd(KA(full_count), 1ull)] =
                            qblk ? (lane == 0 ? old : b0 + lane - 1) : b0 + lane;
                }
                qbase = nb + (unsigned long long)(nblk - 1) * kQBlock;
                qfill = extra - (nblk - 1) * kQBlock;
                qblk = true;
            } else {
                qfill += nout;
            }
        }
    };
    // the outcome of an interaction (next region, or kDie / kOut / kUncertain): retire bookkeeping
    auto outcome = [&](int next) {
        if (ONE) {
            // straight-line: a trace that ended (out-coupled or died) is retired at the next
            // pass's retire site; an abandoned one (rare) goes to the replay list
            fin = (next < 0) & (next != kUncertain);
            active = next >= 0;
            L.r.region = next >= 0 ? next : L.r.region;
            if (__builtin_expect(next == kUncertain, 0)) record_abandoned(K, L.i);
        } else {
            // one retire site for both ends of a trace (out-coupled, died)
            L.r.region = next >= 0 ? next : L.r.region;
            if (__builtin_expect(next == kUncertain, 0)) {
                // abandoned with no side effect; the replay re-traces it (fused: epilogue_kernel,
                // from this iteration on, so later iterations skip the ray)
                if (FUSED)
                    __hip_atomic_store(KA(rng64) + L.i,
                                       ((uint64_t)L.s0 << 32) | iter_tag(A.iter_epoch, L.k, true),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                record_abandoned(K, L.i);
                active = false;
            } else if (next < 0) {
                retire();
            }
        }
    };

    // the second half of a pass: the interaction of the lanes at one, and this pass's out-couplings
    auto interact_pass = [&](SegAcc *sg) {
        if (TL && tl_on) {
            ++tl_passes;
            tl_lanes += __popcll(__ballot(active));
        }
        bool out = false;
        if (active && blk >= 0) {
            L.inter += entry ? 0u : 1u;
            const int next = interact<SINGLE, AMP>(A, K, loc, L, blk, kind, entry, sg);
            out = next == kOut;
            outcome(next);
        }
        SEG_TMARK(sg, 5, L.r.er);
        queue_out(out);
        SEG_MARK(sg, 6);
    };

    for (;;) {
#if WGRT_MAIN_TOPWAIT
        __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
#endif
        if (active) {
            blk = advance(A, K, loc, L, kind);
            entry = false;
            if (ONE) fin |= blk == kDie;
            else if (blk == kDie) retire();
        }
        if (ONE && fin) {   // before the refill, which reuses the lane
            retire();
            fin = false;
        }
        if (FUSED && waiting) {
            // poll only the previous trace's granule: the ray's columns are still in L from the
            // start() that found it not ready
            const uint64_t w = __hip_atomic_load(KA(rng64) + L.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t tag = (uint32_t)w;
            if (tag == iter_tag(A.iter_epoch, L.k, false)) {
                L.r.s = (uint32_t)(w >> 32);
                L.s0 = L.r.s;
                waiting = false;
                active = true;
                blk = 0;
                kind = 0;
                entry = true;
            } else if ((tag >> 8) == ((A.iter_epoch << 1) | 1u)) {
                waiting = false;   // abandoned in an earlier iteration: the replay kernel finishes it
            } else if ((++wait_passes > A.handoff_min_passes) &
                       (__builtin_amdgcn_s_memrealtime() - wait_t0 > A.handoff_wait_ticks)) {
                // hand-off never arrived: give the trace up, visibly, and mark the ray abandoned from this
                // trace on, so that its later traces skip it instead of each waiting out the bound again (the
                // call's results are invalid; the Python layer raises).  Only if the granule still holds the
                // value just polled: a hand-off that arrived since is taken by the next pass's poll instead
                uint64_t seen = w;
                if (__hip_atomic_compare_exchange_strong(KA(rng64) + L.i, &seen,
                                                         (uint64_t)iter_tag(A.iter_epoch, L.k, true), __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    waiting = false;
                    ++tot_giveup;
                }
            }
        }
        uint64_t need = __ballot(!active && !waiting);
        // fused launches refill in batches of kFusedRefill free lanes (or when the wave is empty):
        // a refill's column loads are one round trip the whole wave waits for, and in a fused
        // launch idle lanes are cheap (the next trace's rays keep the chip full): -4 % per trace
        // on C3; single-trace launches gained nothing measurable from batching
        if (FUSED && __popcll(need) < kFusedRefill && __ballot(active || waiting) != 0ull) need = 0ull;
        int staged = 0;                // chunks staged by this refill (at most 1, see below)
        while (need != 0ull && !exhausted) {
            if (cur >= end) {
                // the lanes this refill fills read the current item's buffer and the new one's: a
                // second new item would overwrite rays not yet read
                if (staged == 1) break;
                // dequeue an item when it is needed.  Claiming the next item ahead (to hide the
                // atomic's latency) doubled the rays a wave holds when the queue runs dry, and the
                // launch's tail with them: single launches ran 3 % slower with it
                int64_t c = -1;
                uint32_t k = 0;
                bool got = false;
                for (int tries = 0; !got && tries < kHeads; ++tries) {
                    const int x = (head + tries) & (kHeads - 1);
                    unsigned long long q = 0;
                    if (lane == 0) q = atomicAdd(heads + kHeadStride * x, 1ull);
                    q = uni64(__shfl(q, 0));
                    if (decode(x, (int64_t)q, c, k)) {
                        head = x;
                        got = true;
                    }
                }
                if (!got) {
                    exhausted = true;
                    if (TL && tl_on && lane == 0) {
                        tl[kTlWords * tl_wave + 1] = __builtin_amdgcn_s_memrealtime();
                        tl[kTlWords * tl_wave + 6] = tl_passes;
                        tl[kTlWords * tl_wave + 7] = tl_lanes;
                    }
                    break;
                }
                const int32_t *const ord = KA(order);
                const int64_t cc = (!FUSED && ord) ? (int64_t)ord[c] : c;
                cur = (uint32_t)(cc * chunk);
                const int64_t nr = KA(n_rays);
                end = (uint32_t)((int64_t)cur + chunk < nr ? (int64_t)cur + chunk : nr);
                cur_k = k;
                sb ^= 1;
                sbase_prev = sbase;
                sbase = cur;
                ++staged;
                if (lane < (int)(end - cur)) stage_chunk(K, sbufs + sb * (kStageCols * 64), (int64_t)cur + lane);
            }
            const int want = __popcll(need);
            const uint32_t avail = end - cur;
            const int take = (uint32_t)want < avail ? want : (int)avail;
            if ((need >> lane) & 1ull) {
                const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0));
                if (rank < take) {
                    L.i = cur + (uint32_t)rank;
                    L.k = cur_k;
                    taken = true;
                }
            }
            cur += (uint32_t)take;
            need = __ballot(!active && !waiting && !taken);
        }
        // the rays taken from every item of this refill start together: one round trip for
        // their columns however many items they came from
        if (staged) {
#if WGRT_MAIN_TOPWAIT
            __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);   // the staging loads have landed (the builtin, so
            asm volatile("" ::: "memory");        // the compiler's wait insertion knows nothing is in flight)
#else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the staging loads have landed
#endif
            // lane j prepares slot j of the new chunk; the LDS stores precede the refilled lanes'
            // reads of other lanes' slots in the wave's (in-order) LDS queue
            if (lane < (int)(end - sbase)) prep_staged(A, K, sbufs + sb * (kStageCols * 64), lane);
            asm volatile("" ::: "memory");
        }
        if (taken) {
            start();
            taken = false;
        }
        if (__ballot(active || waiting) == 0ull) break;   // queue exhausted, nothing in flight
        // single-trace launches: once the queue has run dry, the wave's remaining rays finish in
        // the tail loop below
        if (!FUSED && exhausted) break;
        interact_pass(nullptr);
    }
    if (!FUSED && __ballot(active) != 0ull) {
        // the launch tail: the same passes without the refill.  A loop of its own, so the rays in
        // flight when the queue ran dry finish without the refill's code and ballots on every pass
        // (-1.6 % per single launch on C3).  Issuing both branches' matrices or both candidate
        // cell words before the decision here (one or two round trips less per interaction) lost
        // 1.5 % and 6 %: the chip is still full of rays when the queue runs dry.
        // Prefetching the next interaction's line 0 into LDS at each move, its block predicted from
        // the new position (round 6, commit 6b094d1), lost 18-48 %.
        // The first pass continues the one the main loop broke off (advance and refill done).
#ifdef WGRT_SEG
        __shared__ uint32_t seg_lds[4][16];
        SegAcc seg{(uint32_t __attribute__((address_space(3))) *)&seg_lds[threadIdx.x >> 6][0]};
        if (lane < 9) seg.p[lane] = 0u;
        SegAcc *const sg = TL ? &seg : nullptr;   // compile-time: the stamps are straight-line code
#else
        SegAcc *const sg = nullptr;
#endif
        for (bool first = true;; first = false) {
#if WGRT_TAIL_TOPWAIT
            __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
#endif
#ifdef WGRT_SEG
            if (sg) {
                const uint32_t t0 = seg_stamp();
                if (seg_first_lane()) seg.p[8] = t0;
            }
#endif
            if (!first && active) {
                blk = advance(A, K, loc, L, kind);
                entry = false;
                if (ONE) fin |= blk == kDie;
                else if (blk == kDie) retire();
            }
            SEG_MARK_DEP(sg, 0, (double)blk + L.r.x);
            if (ONE && fin) {
                retire();
                fin = false;
            }
            if (__ballot(active) == 0ull) break;
            SEG_MARK(sg, 1);
#ifdef WGRT_SEG
            if (seg_first_lane()) seg.p[7] += 1u;
#endif
            interact_pass(sg);
        }
#ifdef WGRT_SEG
        // segment sums: words 8..15 of a 16-word wave record (tools/segments.py)
        if (TL && tl_on && lane == 0)
            for (int k = 0; k < 8; ++k) tl[kTlWords * tl_wave + 8 + k] = seg.p[k];
#endif
    }
    // the block this wave holds is binned by the wave itself (GRTF:1162-1171, 1231-1240): one
    // lane per entry, its own stores read back (agent-scope loads, past the L1)
    uint32_t tot_h = 0;
    auto bin = [&](unsigned long long j) {
        const uint32_t g = __hip_atomic_load(KA(q_i) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double *pq = (const double *)(KA(q_xy) + j);
        const double px = __hip_atomic_load(pq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double py = __hip_atomic_load(pq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int ny = KA(ny), nx = KA(nx);
        const int en = (int)(g % (uint32_t)ny), em = (int)(g / (uint32_t)ny % (uint32_t)nx);
        const int el = (int)(g / ((uint32_t)ny * (uint32_t)nx));
        tot_h += eyebox_add(A, el, em, en, px, py) ? 1u : 0u;
    };
    if (qblk) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane < qfill) bin(qbase + lane);
        if (EPI) {   // ... and, with the in-kernel epilogue, every block it filled before, along the links
            uint32_t prev = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(KA(full_list) + qbase / kQBlock, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            while (prev != 0u) {
                const uint32_t b = prev - 1u;
                if (lane < kQBlock) bin((unsigned long long)b * kQBlock + lane);
                prev = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(KA(full_list) + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            }
        }
    }
    if (TL && tl_on && lane == 0) {
        tl[kTlWords * tl_wave + 2] = __builtin_amdgcn_s_memrealtime();
        tl[kTlWords * tl_wave + 3] = tl_passes;
        tl[kTlWords * tl_wave + 4] = tl_lanes;
        tl[kTlWords * tl_wave + 5] = (unsigned long long)xcc_id();
    }
    // the workgroup's counters: a fused launch's go to its partial slot (summed by epilogue_kernel), a
    // single launch's to the epilogue totals below (one atomic each per workgroup: not contended)
    __shared__ unsigned long long red[4][5];
    const uint64_t sum_b = wave_sum((uint64_t)tot_b);
    const uint64_t sum_bad = wave_sum((uint64_t)tot_bad);
    const uint64_t sum_h = wave_sum((uint64_t)tot_h);
    const uint64_t sum_g = FUSED ? wave_sum((uint64_t)tot_giveup) : 0ull;
    const uint64_t sum_i = wave_sum((uint64_t)tot_int);
    if (lane == 0) {
        red[threadIdx.x >> 6][0] = sum_b;
        red[threadIdx.x >> 6][1] = sum_bad;
        red[threadIdx.x >> 6][2] = sum_h;
        red[threadIdx.x >> 6][3] = sum_g;
        red[threadIdx.x >> 6][4] = sum_i;
    }
    if (!EPI) {
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long *slot = KA(part) + kPartWords * (size_t)blockIdx.x;
            slot[0] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
            slot[1] = red[0][1] + red[1][1] + red[2][1] + red[3][1];
            slot[2] = red[0][2] + red[1][2] + red[2][2] + red[3][2];
            slot[3] = red[0][3] + red[1][3] + red[2][3] + red[3][3];
            slot[4] = red[0][4] + red[1][4] + red[2][4] + red[3][4];
        }
        return;
    }
    // In-kernel epilogue: one lane adds the workgroup's totals with agent-scope atomics, waits for
    // them, and counts the workgroup done; the workgroup that counts last reads the totals at agent
    // scope, adds them to *stats and zeroes the next launch's counter set (every other workgroup has
    // left this one's)
    __shared__ int last_wg;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long *const acc = KA(epi_acc);
        const unsigned long long t_b = red[0][0] + red[1][0] + red[2][0] + red[3][0];
        const unsigned long long t_bad = red[0][1] + red[1][1] + red[2][1] + red[3][1];
        const unsigned long long t_h = red[0][2] + red[1][2] + red[2][2] + red[3][2];
        const unsigned long long t_i = red[0][4] + red[1][4] + red[2][4] + red[3][4];
        if (t_b) atomicAdd(acc + 0, t_b);
        if (t_bad) atomicAdd(acc + 1, t_bad);
        if (t_h) atomicAdd(acc + 2, t_h);
        if (t_i) atomicAdd(acc + 3, t_i);
        // gfx9: vmcnt counts the no-return atomics too, so they have been performed at the device-coherent
        // level before the done count below; an acq_rel increment instead would write back this XCD's
        // whole L2 (buffer_wbl2) per workgroup for values that never sit in it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last_wg = atomicAdd(KA(epi_done), 1ull) == (unsigned long long)gridDim.x - 1ull;
    }
    __syncthreads();
    if (!last_wg) return;
    unsigned long long *const oc = KA(other_ctr);
    for (int k = threadIdx.x; k < kScratchCtr; k += blockDim.x) oc[k] = 0ull;
    wgrt_trace_stats *const st = KA(stats);
    if (threadIdx.x == 0 && st) {
        unsigned long long *const acc = KA(epi_acc);
        unsigned long long t[4];
        for (int k = 0; k < 4; ++k) t[k] = __hip_atomic_load(acc + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t[3]) atomicAdd((unsigned long long *)&st->interactions, t[3]);
        if (t[0]) atomicAdd((unsigned long long *)&st->bounces, t[0]);
        if (t[1]) atomicAdd((unsigned long long *)&st->bad_rays, t[1]);
        if (t[2]) atomicAdd((unsigned long long *)&st->eyebox_hits, t[2]);
    }
#if WGRT_INKERNEL_REPLAY
    // the abandoned rays (none in practice): re-traced here, by the workgroup that counted last, with
    // the reference arithmetic -- no replay kernel behind the launch.  Every list entry was stored at
    // agent scope and waited for by its lane before that lane's workgroup counted itself done.
    const unsigned long long nr = __hip_atomic_load(KA(replay_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_expect(nr != 0ull, 0)) replay_tail(K, nr);
#endif
}

// The replay kernel behind a single launch with the in-kernel epilogue: re-traces the launch's
// abandoned rays from their launch-start state with the reference arithmetic, one per thread (usually
// there are none: every workgroup reads one count and leaves).
constexpr int kReplayGroups = 64;
__global__ __launch_bounds__(256) void replay_kernel(TraceArgs A) {
    const unsigned long long nr = *A.replay_count;
    if (nr == 0ull) return;
    uint64_t b = 0, h = 0, bad = 0, ni = 0, lm = 0;
    for (unsigned long long k = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; k < nr;
         k += (unsigned long long)gridDim.x * blockDim.x)
        trace_one(A, (int64_t)A.replay_list[k], b, h, bad, nullptr, &ni, &lm);
    add_stats(A.stats, b, h, bad, ni, lm);
    if (blockIdx.x == 0 && threadIdx.x == 0 && A.stats) atomicAdd((unsigned long long *)&A.stats->replayed, nr);
}

// Variants 7 / 9: the persistent loop over the Jones-vector path (32-bit cell words; 64-bit
// cell words for scenes of more than 16 polygons).  Waves per SIMD: 4 (<= 128 VGPRs, no spills).
// At 96 VGPRs (5 waves) the full-colour single-trace kernel spills 88 B per lane and runs 36 %
// slower than at 4; WGRT_JONES_WAVES=5 builds it so.
#ifndef WGRT_JONES_WAVES
#define WGRT_JONES_WAVES 4
#endif
template <class CellT, bool FUSED, bool SINGLE>
constexpr int jones_waves() {
    return (sizeof(CellT) == 4 && !FUSED && !SINGLE) ? WGRT_JONES_WAVES : 4;
}
// AMP: with the amplification step of the certification bound (wgrt_device.h; scenes with a block whose
// branch matrices are not scaled-unitary)
template <class CellT, bool FUSED, bool SINGLE, bool AMP>
__global__ __launch_bounds__(256, (jones_waves<CellT, FUSED, SINGLE>())) void trace_jones_kernel(TraceArgs A, LocatorT<CellT> loc,
                                                             unsigned long long *counter, int chunk) {
    jones_body<FUSED, SINGLE, false, AMP>(
        A, kernel_kargs<decltype(trace_jones_kernel<CellT, FUSED, SINGLE, AMP>)>(), loc, counter, chunk);
}

// The same loop with the debug wave timeline (wgrt_debug_opts.timeline; tools/timeline.py): a
// separate instantiation, so the product kernels carry none of its code.
template <class CellT, bool FUSED, bool SINGLE>
__global__ __launch_bounds__(256, (jones_waves<CellT, FUSED, SINGLE>())) void trace_jones_tl_kernel(
    TraceArgs A, LocatorT<CellT> loc, unsigned long long *counter, int chunk) {
    jones_body<FUSED, SINGLE, true, false>(A, kernel_kargs<decltype(trace_jones_tl_kernel<CellT, FUSED, SINGLE>)>(),
                                           loc, counter, chunk);
}

__global__ __launch_bounds__(256) void classify_kernel(Locator L, int npoly, const double *xy, int64_t n,
                                                       uint64_t *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = xy[2 * i], y = xy[2 * i + 1];
    const Cell w = locate(L, x, y);
    const uint64_t ww = locate_w(L, x, y);
    uint64_t mask = 0, mism = 0;
    for (int k = 0; k < npoly; ++k) {
        const bool a = in_poly(L, w, k, x, y);      // CSR row lists (exact lane)
        const bool b = in_poly_w(L, ww, k, x, y);   // 128-B band records (Jones-vector lane)
        if (a) mask |= 1ull << k;
        if (a != b) mism = 1ull << 63;
    }
    out[i] = mask | mism;
}

// Ray setup of FoV x wavelength blocks [blk_lo, blk_lo + n / R) (reference MAIN:65-115, 158):
// ray i of block b = (ii * ny + jj) * nl + k takes origin point r = i % R (TE half) or
// r - R/2 (TM half); m = ii, n = jj, lmd_num = lambdas[k]; gap / angles / phase 0.  With an
// odd R the reference leaves the last ray of every block all-zero (its two halves cover
// 2 * floor(R / 2) rays), and so does this.
struct RayInitArgs {
    const double *points;   // [R / 2, 2]
    float *col[12];         // wgrt_ray_columns order, NULL = not written
    uint32_t *rng;
    int64_t n, R, blk_lo, gid_offset;
    int ny, nl;
    float lambdas[8];
};

__global__ __launch_bounds__(256) void rays_init_kernel(RayInitArgs A) {
    const int64_t half = A.R / 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t blk = A.blk_lo + i / A.R, r = i % A.R;
        const int k = (int)(blk % A.nl);
        const int64_t fov = blk / A.nl;
        const int jj = (int)(fov % A.ny), ii = (int)(fov / A.ny);
        float v[12] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (r < 2 * half) {
            const int64_t p = r < half ? r : r - half;
            v[0] = (float)A.points[2 * p];       // x    (float64 -> float32, round to nearest)
            v[1] = (float)A.points[2 * p + 1];   // y
            v[6] = (float)ii;                    // m
            v[7] = (float)jj;                    // n
            v[8] = A.lambdas[k];                 // lmd_num
            v[9] = r < half ? 1.f : 0.f;         // te
            v[10] = r < half ? 0.f : 1.f;        // tm
        }
#pragma unroll
        for (int c = 0; c < 12; ++c)
            if (A.col[c]) A.col[c][i] = v[c];
        if (A.rng) A.rng[i] = 0x9E3779B9u * (uint32_t)(A.gid_offset + i + 1);   // MAIN:158, mod 2^32
    }
}

// Eyebox collection of the strong-scaling gather (include/wgrt.h wgrt_eyebox_*): row copies of whole
// 80 x 120 slabs as 16-B loads / stores, one workgroup per (row, 1/kEbSlabParts of the slab).  The
// spill rows (121 floats) move as dwords.
constexpr int kEbSlabF4 = WGRT_EB_SLAB / 4;   // 2400 float4 per slab
constexpr int kEbSlabParts = 3;               // 800 float4 per workgroup: 256 threads x 3-4

__host__ __device__ inline int64_t eb_spill_floats(int64_t nb) { return (nb * WGRT_EB_SPILL + 3) / 4 * 4; }

__global__ __launch_bounds__(256) void eyebox_pack_kernel(const float *eb, int64_t n_slabs, const int64_t *slabs,
                                                          const int64_t *next, const float *mask, int64_t n, int64_t nb,
                                                          float *payload) {
    const int64_t j = blockIdx.y;
    if (j >= n) return;
    const int64_t s = slabs[j];
    if (s < 0 || s >= n_slabs) return;
    const float4 *src = (const float4 *)(eb + s * WGRT_EB_SLAB);
    float4 *out = (float4 *)(payload + j * WGRT_EB_SLAB);
    const int lo = (int)blockIdx.x * (kEbSlabF4 / kEbSlabParts), hi = lo + kEbSlabF4 / kEbSlabParts;
    for (int c = lo + threadIdx.x; c < hi; c += blockDim.x) out[c] = src[c];
    if (blockIdx.x == 0 && threadIdx.x < WGRT_EB_SPILL) {
        const int64_t t = next[j];
        const float v = (t >= 0 && t < n_slabs) ? eb[t * WGRT_EB_SLAB + threadIdx.x] * mask[j] : 0.0f;
        payload[nb * WGRT_EB_SLAB + j * WGRT_EB_SPILL + threadIdx.x] = v;
    }
}

__global__ __launch_bounds__(256) void eyebox_copy_kernel(float *eb, int64_t n_slabs, const float *recv, int64_t nb,
                                                          int64_t plen, const int64_t *dst) {
    const int64_t row = blockIdx.y;   // r * nb + j
    const int64_t s = dst[row];
    if (s < 0 || s >= n_slabs) return;
    const int64_t r = row / nb, j = row % nb;
    const float4 *src = (const float4 *)(recv + r * plen + j * WGRT_EB_SLAB);
    float4 *out = (float4 *)(eb + s * WGRT_EB_SLAB);
    const int lo = (int)blockIdx.x * (kEbSlabF4 / kEbSlabParts), hi = lo + kEbSlabF4 / kEbSlabParts;
    for (int c = lo + threadIdx.x; c < hi; c += blockDim.x) out[c] = src[c];
}

__global__ __launch_bounds__(128) void eyebox_spill_kernel(float *eb, int64_t n_slabs, const float *recv, int64_t nb,
                                                           int64_t plen, const int64_t *spill_dst) {
    const int64_t row = blockIdx.x;
    const int64_t s = spill_dst[row];
    if (s < 0 || s >= n_slabs || threadIdx.x >= WGRT_EB_SPILL) return;
    const int64_t r = row / nb, j = row % nb;
    // one spill row per target slab (slab s's spill comes only from slab s - 1): no atomics needed
    eb[s * WGRT_EB_SLAB + threadIdx.x] += recv[r * plen + nb * WGRT_EB_SLAB + j * WGRT_EB_SPILL + threadIdx.x];
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

// ---------------------------------------------------------------------------------------------
// Scene build on the device (wgrt_scene_create): the locator's cell words and the LUT tiles.
// ---------------------------------------------------------------------------------------------
// EDGE marks: one thread per (polygon edge, grid row); the row's cells the edge reaches get the
// polygon's bit (wgrt_pack.h edge_row_span, the host build's rule).
__global__ __launch_bounds__(256) void edge_mark_kernel(const double *verts, const int32_t *poly_off, int npoly,
                                                        double x0, double y0, double h, int ncx, int ncy,
                                                        uint32_t *mask) {
    const int e = blockIdx.y;   // global edge index: polygon k's edge (i - 1 -> i), i = e - poly_off[k]
    int k = 0;
    while (k + 1 < npoly && poly_off[k + 1] <= e) ++k;
    const int a = poly_off[k], nv = poly_off[k + 1] - a, i = e - a;
    if (nv <= 0 || i < 0 || i >= nv) return;
    const int j = i == 0 ? nv - 1 : i - 1;
    const double ax = verts[2 * (a + j)], ay = verts[2 * (a + j) + 1];
    const double bx = verts[2 * (a + i)], by = verts[2 * (a + i) + 1];
    int cy0, cy1;
    edge_rows(ay, by, y0, h, ncy, cy0, cy1);
    const int cy = cy0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (cy > cy1) return;
    int cx0, cx1;
    if (!edge_row_span(ax, ay, bx, by, cy, x0, y0, h, ncx, cx0, cx1)) return;
    for (int cx = cx0; cx <= cx1; ++cx) atomicOr(mask + (size_t)cy * ncx + cx, 1u << k);
}

// Cell words: EDGE where marked, else the reference predicate's crossing parity at the cell
// centre over the row's edges (every edge crossing the row's centre line is in its band list).
__global__ __launch_bounds__(256) void classify_cells_kernel(const double *verts, const int32_t *poly_off, int npoly,
                                                             const int32_t *row_off, const int32_t *row_edges,
                                                             double x0, double y0, double h, int ncx, int ncy,
                                                             const uint32_t *mask, uint64_t *cells, uint32_t *cells32,
                                                             unsigned long long *edge_cells) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t edges = 0;
    if (c < (int64_t)ncx * ncy) {
        const int cy = (int)(c / ncx), cx = (int)(c % ncx);
        const double px = x0 + (cx + 0.5) * h, py = y0 + (cy + 0.5) * h;
        const uint32_t mk = mask[c];
        uint64_t w = 0;
        for (int k = 0; k < npoly; ++k) {
            uint64_t cls;
            if ((mk >> k) & 1u) {
                cls = 2;
                ++edges;
            } else {
                const int a = poly_off[k], nv = poly_off[k + 1] - a;
                const int r = k * ncy + cy;
                unsigned cnt = 0;
                for (int e = row_off[r]; e < row_off[r + 1]; ++e) {
                    const int i = row_edges[e], j = i == 0 ? nv - 1 : i - 1;
                    const double xi = verts[2 * (a + i)], yi = verts[2 * (a + i) + 1];
                    const double xj = verts[2 * (a + j)], yj = verts[2 * (a + j) + 1];
                    if ((yi > py) != (yj > py)) cnt += px < (xj - xi) * (py - yi) / (yj - yi + 1e-20) + xi;
                }
                cls = cnt & 1u;
            }
            w |= cls << (2 * k);
        }
        cells[c] = w;
        if (cells32) cells32[c] = (uint32_t)w;
    }
    edges = wave_sum(edges);
    if ((threadIdx.x & 63) == 0 && edges) atomicAdd(edge_cells, (unsigned long long)edges);
}

// One thread per (lambda, m, n) tile: the exact lane's tile and its Jones-vector tile
// (wgrt_pack.h pack_tile, the host build's code); flags any non-finite value.
// Blocks of the Jones tiles flagged non-scaled-unitary (the sign bit of their float Wsum, wgrt_pack.h):
// counted once per scene, to pick the trace kernel instantiation (AMP) for its launches.
__global__ __launch_bounds__(256) void nonunitary_kernel(const double *jtiles, int64_t ntiles, int jd, int nblk,
                                                         unsigned long long *count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntiles * nblk) return;
    const int64_t g = i / nblk, b = i % nblk;
    const float w = *(const float *)(jtiles + g * jd + kJHeader + kJBlock * b + kJBlockF32);
    if (__float_as_uint(w) >> 31) atomicAdd(count, 1ull);
}

__global__ __launch_bounds__(64) void pack_tiles_kernel(PackView v, int64_t ntiles, double *tiles, double *jtiles,
                                                        int td, int jd, int *nonfinite) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ntiles) return;
    double *T = tiles + g * td;
    pack_tile(v, g, T, jtiles + g * jd);
    bool bad = false;
    for (int k = 0; k < td; ++k) bad |= !isfinite(T[k]);
    if (bad) atomicOr(nonfinite, 1);
}

}  // namespace

namespace {

// hipMalloc + copy of n elements (n may be 0)
template <class T>
wgrt_status upload_n(const T *src, size_t n, T **dst) {
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    hipError_t e = hipMalloc((void **)dst, bytes);
    if (e == hipErrorOutOfMemory) return fail(WGRT_ERR_OUT_OF_MEMORY, "hipMalloc: out of memory");
    if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    if (n) HIP_TRY(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return WGRT_OK;
}

template <class T>
wgrt_status alloc_n(size_t n, T **dst) {
    hipError_t e = hipMalloc((void **)dst, std::max<size_t>(n, 1) * sizeof(T));
    if (e == hipErrorOutOfMemory) return fail(WGRT_ERR_OUT_OF_MEMORY, "hipMalloc: out of memory");
    if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    return WGRT_OK;
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
    return wgrt_scene_create_ex(desc, device, nullptr, out);
}

wgrt_status wgrt_scene_create_ex(const wgrt_scene_desc *desc, int device, const wgrt_scene_opts *opts,
                                 wgrt_scene **out) {
    if (!desc || !out) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL desc / out");
    *out = nullptr;
    const wgrt_scene_desc &d = *desc;
    const double cell_mm = (opts && opts->cell_mm > 0.0) ? opts->cell_mm : kDefaultCellMm;
    if (opts && !(opts->cell_mm >= 0.0)) return fail(WGRT_ERR_INVALID_ARGUMENT, "cell_mm must be >= 0");
    const bool host_build = opts && opts->host_build != 0;
    const int f32_angles = opts ? opts->lut_f32_angles : 0;
    if (f32_angles & ~0x7f) return fail(WGRT_ERR_INVALID_ARGUMENT, "lut_f32_angles has bits beyond the 7 LUTs");
    // A mixed set: compiled numba unifies the ray's theta (assigned from every table, GRTF:850, 872, 1021,
    // ...) to complex128 as soon as one table is complex128, so the carried cos(theta.real) would be a
    // double cosine of a single-precision table's angle while that table's numerator stays cosf --
    // two cosines per branch the scene does not hold.  Only uniform sets are supported.
    if (f32_angles != 0 && f32_angles != 0x7f)
        return fail(WGRT_ERR_UNSUPPORTED, "lut_f32_angles must be 0 (complex128 LUTs) or 0x7f (all seven complex64): "
                                          "a mixed-precision LUT set is not supported");
    // host: validation, the locator's geometry (extent, vertices, row bands) and the trig table
    // (every cos / sin on the host libm); the cell words and the tiles are built on the device
    // (host_build: both on the host, the reference build the device one is checked against)
    SceneHost host;
    try {
        build_scene_host(d, cell_mm, host, host_build, host_build, f32_angles);
    } catch (const std::exception &e) {
        return fail(WGRT_ERR_INVALID_ARGUMENT, e.what());
    }
    DEVICE_SCOPE(dev_scope, device);   // the caller's current device is restored on return
    auto *s = new wgrt_scene();
    s->device = device;
    s->nx = d.nx;
    s->ny = d.ny;
    s->nl = d.num_lmd;
    s->nfc = (int)d.n_fc_slices;
    s->noc = (int)d.n_oc_slices;
    s->tile_d = host.tile_doubles;
    s->jtile_d = host.jtile_doubles;
    s->npoly = 3 + s->nfc + s->noc;
    s->n_g = d.n_g;
    s->tiles = (int64_t)s->nl * s->nx * s->ny;
    wgrt_status st;
    auto bail = [&](wgrt_status e) {
        wgrt_scene_destroy(s);
        return e;
    };
    if ((st = upload(host.loc.verts, &s->d_verts)) != WGRT_OK ||
        (st = upload(host.loc.poly_off, &s->d_poly_off)) != WGRT_OK ||
        (st = upload(host.loc.row_off, &s->d_row_off)) != WGRT_OK ||
        (st = upload(host.loc.row_edges, &s->d_row_edges)) != WGRT_OK ||
        (st = upload(host.loc.bands, &s->d_bands)) != WGRT_OK)
        return bail(st);
    const size_t ncells = (size_t)host.loc.ncx * host.loc.ncy;
    if (host_build) {
        if ((st = upload(host.tiles, &s->d_tiles)) != WGRT_OK || (st = upload(host.jtiles, &s->d_jtiles)) != WGRT_OK ||
            (st = upload(host.loc.cells, &s->d_cells)) != WGRT_OK)
            return bail(st);
        if (s->npoly <= 16) {
            const std::vector<uint32_t> c32(host.loc.cells.begin(), host.loc.cells.end());
            if ((st = upload(c32, &s->d_cells32)) != WGRT_OK) return bail(st);
        }
        s->edge_cells = host.loc.edge_cells;
    } else {
        // the raw arrays the tiles are packed from, on the device for the packing only
        const int64_t g = (int64_t)d.num_lmd * d.nx * d.ny, nfc = d.n_fc_slices, noc = d.n_oc_slices;
        const size_t n5 = (size_t)g * d.ch5 * 2, n3 = (size_t)g * d.ch3 * 2;
        double *raw[12] = {};
        auto free_raw = [&]() {
            for (double *p : raw) (void)hipFree(p);
        };
        const double *src[12] = {d.lut_ic1, d.lut_ic2, d.lut_ic3, d.lut_fc1, d.lut_fc2, d.lut_oc1, d.lut_oc2,
                                 d.lut_TIR, d.lut_gap, d.eff_reg_FOV, d.eff_reg_FOV_range, host.trig.data()};
        const size_t cnt[12] = {n5, n5, n5, nfc * n3, nfc * n3, noc * n5, noc * n5, (size_t)g * 4, (size_t)g * 8,
                                (size_t)d.nx * d.ny * 8, (size_t)d.nx * d.ny * 4, host.trig.size()};
        for (int k = 0; k < 12; ++k)
            if ((st = upload_n(cnt[k] ? src[k] : nullptr, cnt[k], &raw[k])) != WGRT_OK) {
                free_raw();
                return bail(st);
            }
        PackView v = pack_view(d, raw[11]);
        v.ic1 = raw[0], v.ic2 = raw[1], v.ic3 = raw[2], v.fc1 = raw[3], v.fc2 = raw[4], v.oc1 = raw[5], v.oc2 = raw[6];
        v.tir = raw[7], v.gap = raw[8], v.fov = raw[9], v.fovr = raw[10];
        int *flag = nullptr;
        unsigned long long *ecount = nullptr;
        uint32_t *mask = nullptr;
        auto free_tmp = [&]() {
            free_raw();
            (void)hipFree(flag);
            (void)hipFree(ecount);
            (void)hipFree(mask);
        };
        if ((st = alloc_n((size_t)g * s->tile_d, &s->d_tiles)) != WGRT_OK ||
            (st = alloc_n((size_t)g * s->jtile_d, &s->d_jtiles)) != WGRT_OK || (st = alloc_n(1, &flag)) != WGRT_OK ||
            (st = alloc_n(1, &ecount)) != WGRT_OK || (st = alloc_n(ncells, &mask)) != WGRT_OK ||
            (st = alloc_n(ncells, &s->d_cells)) != WGRT_OK ||
            (s->npoly <= 16 && (st = alloc_n(ncells, &s->d_cells32)) != WGRT_OK)) {
            free_tmp();
            return bail(st);
        }
        HIP_TRY(hipMemset(s->d_tiles, 0, (size_t)g * s->tile_d * sizeof(double)));
        HIP_TRY(hipMemset(s->d_jtiles, 0, (size_t)g * s->jtile_d * sizeof(double)));
        HIP_TRY(hipMemset(flag, 0, sizeof(int)));
        HIP_TRY(hipMemset(ecount, 0, sizeof(unsigned long long)));
        HIP_TRY(hipMemset(mask, 0, ncells * sizeof(uint32_t)));
        hipLaunchKernelGGL(pack_tiles_kernel, dim3((unsigned)((g + 63) / 64)), dim3(64), 0, 0, v, g, s->d_tiles,
                           s->d_jtiles, s->tile_d, s->jtile_d, flag);
        HIP_TRY(hipGetLastError());
        const LocatorHost &L = host.loc;
        const int npoly = (int)L.poly_off.size() - 1, n_edges = L.poly_off.back();
        if (n_edges > 0) {
            hipLaunchKernelGGL(edge_mark_kernel, dim3((unsigned)((L.ncy + 255) / 256), (unsigned)n_edges), dim3(256),
                               0, 0, s->d_verts, s->d_poly_off, npoly, L.x0, L.y0, L.h, L.ncx, L.ncy, mask);
            HIP_TRY(hipGetLastError());
        }
        hipLaunchKernelGGL(classify_cells_kernel, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, 0, s->d_verts,
                           s->d_poly_off, npoly, s->d_row_off, s->d_row_edges, L.x0, L.y0, L.h, L.ncx, L.ncy, mask,
                           s->d_cells, s->d_cells32, ecount);
        HIP_TRY(hipGetLastError());
        int bad = 0;
        unsigned long long ec = 0;
        HIP_TRY(hipMemcpy(&bad, flag, sizeof(int), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(&ec, ecount, sizeof(ec), hipMemcpyDeviceToHost));
        free_tmp();
        if (bad) {
            // The kernels' cheap branch estimates assume finite tables (an inf / NaN coefficient
            // would make the reference's efficiencies NaN); such LUTs are rejected instead.
            return bail(fail(WGRT_ERR_INVALID_ARGUMENT,
                             "non-finite value in the LUTs / lut_TIR / lut_gap / eyebox tables"));
        }
        s->edge_cells = (int64_t)ec;
    }
    {   // the scene's non-scaled-unitary blocks (the trace kernel instantiation its launches run)
        const int nblk = 3 + 2 * s->nfc + 2 * s->noc;
        const int64_t nt = (int64_t)s->nl * s->nx * s->ny;
        unsigned long long *cnt = nullptr;
        HIP_TRY(hipMalloc((void **)&cnt, sizeof(unsigned long long)));
        hipError_t e = hipMemset(cnt, 0, sizeof(unsigned long long));
        if (e == hipSuccess && nt * nblk > 0) {
            hipLaunchKernelGGL(nonunitary_kernel, dim3((unsigned)((nt * nblk + 255) / 256)), dim3(256), 0, 0, s->d_jtiles,
                               nt, s->jtile_d, nblk, cnt);
            e = hipGetLastError();
        }
        unsigned long long nu = 0;
        if (e == hipSuccess) e = hipMemcpy(&nu, cnt, sizeof(nu), hipMemcpyDeviceToHost);
        (void)hipFree(cnt);
        if (e != hipSuccess) return bail(fail(WGRT_ERR_HIP, std::string("nonunitary_kernel: ") + hipGetErrorString(e)));
        s->nonunitary_blocks = (int64_t)nu;
    }
    {
        int cus = 0, per_cu = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        // resident workgroups of each instantiation (cell width x fused x single wavelength)
        auto grid_of = [&](const void *k, int &out) -> hipError_t {
            const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0);
            out = std::max(1, cus * std::max(1, per_cu));
            return e;
        };
#define WGRT_GRID(CELL, C, F, S)                                                                              \
        HIP_TRY(grid_of((const void *)trace_jones_kernel<CELL, F, S, false>, s->jones_grid[C][F][S]));        \
        {   /* the AMP instantiation: the smaller of the two grids */                                        \
            int g2 = 0;                                                                                       \
            HIP_TRY(grid_of((const void *)trace_jones_kernel<CELL, F, S, true>, g2));                        \
            s->jones_grid[C][F][S] = std::min(s->jones_grid[C][F][S], g2);                                   \
        }
        WGRT_GRID(uint32_t, 0, false, false);
        WGRT_GRID(uint32_t, 0, false, true);
        WGRT_GRID(uint32_t, 0, true, false);
        WGRT_GRID(uint32_t, 0, true, true);
        WGRT_GRID(uint64_t, 1, false, false);
        WGRT_GRID(uint64_t, 1, false, true);
        WGRT_GRID(uint64_t, 1, true, false);
        WGRT_GRID(uint64_t, 1, true, true);
#undef WGRT_GRID
        // the debug timeline instantiations (32-bit cells, full colour, single / fused)
        HIP_TRY(grid_of((const void *)trace_jones_tl_kernel<uint32_t, false, false>, s->jones_tl_grid[0]));
        HIP_TRY(grid_of((const void *)trace_jones_tl_kernel<uint32_t, true, false>, s->jones_tl_grid[1]));
    }
    s->loc_host = host.loc;
    s->loc_host.cells.clear();
    s->loc_host.cells.shrink_to_fit();
    s->loc_host.row_edges.clear();
    s->loc_host.row_edges.shrink_to_fit();
    s->loc_host.bands.clear();
    s->loc_host.bands.shrink_to_fit();
    *out = s;
    return WGRT_OK;
}

wgrt_status wgrt_scene_destroy(wgrt_scene *s) {
    if (!s) return WGRT_OK;
    DeviceScope dev_scope(s->device);
    (void)hipFree(s->d_tiles);
    (void)hipFree(s->d_jtiles);
    (void)hipFree(s->d_cells);
    (void)hipFree(s->d_cells32);
    (void)hipFree(s->d_verts);
    (void)hipFree(s->d_poly_off);
    (void)hipFree(s->d_row_off);
    (void)hipFree(s->d_row_edges);
    (void)hipFree(s->d_bands);
    for (auto &kv : s->scratch) {
        (void)hipFree(kv.second.ctr);
        (void)hipFree(kv.second.list);
        (void)hipFree(kv.second.q_xy);
        (void)hipFree(kv.second.q_i);
        (void)hipFree(kv.second.full);
        (void)hipFree(kv.second.rng64);
        (void)hipFree(kv.second.part);
    }
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
    info->grid_edge_cells = s->edge_cells;
    info->n_polygons = s->npoly;
    info->device = s->device;
    info->jtile_bytes = (int64_t)s->jtile_d * 8;
    info->nonunitary_blocks = s->nonunitary_blocks;
    return WGRT_OK;
}

}  // extern "C"

namespace {

// The Jones-vector variants' per-stream launch scratch (work-queue heads, replay list,
// out-coupling queue, fused-launch granules), grown to n_rays x num_iter traces on `grid`
// workgroups.  Growing synchronises the stream (the old buffers may be in use).  For a launch
// (parity != NULL) the counter set it uses is returned and the next launch is given the other
// one -- only once every allocation has succeeded, so a failed growth leaves the sets as they
// were; a launch that fails after this point marks the scratch dirty (mark_dirty), and the next
// call zeroes both sets before it uses either.  For a fused launch (epoch != NULL) the launch
// epoch of the granule tags is advanced here, under the same lock, and returned.
wgrt_status ensure_scratch(wgrt_scene *ms, void *stream, int64_t n_rays, int num_iter, int64_t grid,
                           wgrt_scene::Scratch **out, uint32_t *epoch = nullptr, uint32_t *parity = nullptr) {
    hipStream_t st = (hipStream_t)stream;
    std::lock_guard<std::mutex> lk(ms->scratch_mu);
    wgrt_scene::Scratch *sc = &ms->scratch[stream];
    *out = sc;
    if (!sc->ctr) {
        // both counter sets zeroed once here; afterwards every launch's epilogue zeroes the set
        // the next launch uses
        hipError_t e = hipMalloc((void **)&sc->ctr, 2 * kScratchCtr * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMemset(sc->ctr, 0, 2 * kScratchCtr * sizeof(unsigned long long));
        if (e != hipSuccess) {
            (void)hipFree(sc->ctr);
            sc->ctr = nullptr;
            return fail(WGRT_ERR_HIP, std::string("hipMalloc(scratch): ") + hipGetErrorString(e));
        }
        sc->parity = 0;
        sc->dirty = false;
    }
    if (sc->dirty) {
        // an earlier launch failed half-way (its epilogue may not have zeroed the next set)
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemset(sc->ctr, 0, 2 * kScratchCtr * sizeof(unsigned long long)));
        sc->parity = 0;
        sc->dirty = false;
    }
    // counter partials: one slot per trace-kernel workgroup
    const int64_t slots = grid;
    if (sc->part_slots < slots) {
        HIP_TRY(hipStreamSynchronize(st));
        (void)hipFree(sc->part);
        sc->part = nullptr;
        sc->part_slots = 0;
        hipError_t e = hipMalloc((void **)&sc->part, (size_t)slots * kPartWords * sizeof(unsigned long long));
        if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("hipMalloc(launch scratch): ") + hipGetErrorString(e));
        sc->part_slots = slots;
    }
    if (sc->cap < n_rays) {
        // the old lists may still be in use by this stream's previous launch
        HIP_TRY(hipStreamSynchronize(st));
        (void)hipFree(sc->list);
        sc->list = nullptr;
        sc->cap = 0;
        hipError_t e = hipMalloc((void **)&sc->list, (size_t)n_rays * sizeof(uint32_t));
        if (e == hipErrorOutOfMemory) return fail(WGRT_ERR_OUT_OF_MEMORY, "hipMalloc(launch scratch): out of memory");
        if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("hipMalloc(launch scratch): ") + hipGetErrorString(e));
        sc->cap = n_rays;
    }
    // a trace out-couples at most once; each wave leaves at most one block partly unused
    const int64_t qn = n_rays * num_iter + grid * 4 * kQBlock;
    if (sc->qcap < qn) {
        HIP_TRY(hipStreamSynchronize(st));
        (void)hipFree(sc->q_xy);
        (void)hipFree(sc->q_i);
        (void)hipFree(sc->full);
        sc->q_xy = nullptr;
        sc->q_i = nullptr;
        sc->full = nullptr;
        sc->qcap = 0;
        hipError_t e = hipMalloc((void **)&sc->q_xy, (size_t)qn * sizeof(double2));
        if (e == hipSuccess) e = hipMalloc((void **)&sc->q_i, (size_t)qn * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc((void **)&sc->full, (size_t)(qn / kQBlock + 1) * sizeof(uint32_t));
        if (e == hipErrorOutOfMemory) return fail(WGRT_ERR_OUT_OF_MEMORY, "hipMalloc(launch scratch): out of memory");
        if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("hipMalloc(launch scratch): ") + hipGetErrorString(e));
        sc->qcap = qn;
    }
    if (num_iter > 1 && sc->cap64 < n_rays) {
        HIP_TRY(hipStreamSynchronize(st));
        (void)hipFree(sc->rng64);
        sc->rng64 = nullptr;
        sc->cap64 = 0;
        sc->iter_epoch = 0;
        hipError_t e = hipMalloc((void **)&sc->rng64, (size_t)n_rays * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMemset(sc->rng64, 0, (size_t)n_rays * sizeof(uint64_t));
        if (e == hipErrorOutOfMemory) return fail(WGRT_ERR_OUT_OF_MEMORY, "hipMalloc(launch scratch): out of memory");
        if (e != hipSuccess) return fail(WGRT_ERR_HIP, std::string("hipMalloc(launch scratch): ") + hipGetErrorString(e));
        sc->cap64 = n_rays;
    }
    if (epoch) {
        if (++sc->iter_epoch >= (1u << 23)) {   // granule tags wrapped: clear them
            HIP_TRY(hipMemsetAsync(sc->rng64, 0, (size_t)sc->cap64 * sizeof(uint64_t), st));
            sc->iter_epoch = 1;
        }
        *epoch = sc->iter_epoch;
    }
    if (parity) {   // a launch: its counter set; the next launch takes the other one
        *parity = sc->parity;
        sc->parity ^= 1u;
    }
    return WGRT_OK;
}

// A launch failed after ensure_scratch handed it a counter set: neither set can be trusted to be
// zero any more (see ensure_scratch).
void mark_dirty(wgrt_scene *ms, wgrt_scene::Scratch *sc) {
    std::lock_guard<std::mutex> lk(ms->scratch_mu);
    sc->dirty = true;
}

struct LaunchCfg {
    int variant = 0, workgroups = 0, num_iter = 1;
    bool single = false;
    const int32_t *chunk_order = nullptr;
    int64_t n_chunk_order = 0;
    const int64_t *gid_blocks = nullptr;
    int64_t gid_block_rays = 0;
    const wgrt_debug_opts *dbg = nullptr;
    double grid_k = 0.0;   // wgrt_launch_opts.grid_sqrt_k (0: kGridSqrtK; < 0: the resident grid)
};

// Single traces: ceil(kGridSqrtK * sqrt(work items)) workgroups (wgrt_launch_opts.grid_sqrt_k).
constexpr double kGridSqrtK = 6.5;

// One launch of the bounce kernel.  single: the single-wavelength kernel
// process_rays_kernel_pro (GRTF:419-831) -- no lmd_num column, wavelength 0 of a
// one-wavelength scene, threshold 1e-15; otherwise process_rays_kernel_pro_fullColor
// (GRTF:833-1246), threshold 0.  The two kernels differ in nothing else.
wgrt_status trace_launch(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays, int64_t gid_offset,
                         uint32_t *rng_states, float *matrix_EB, wgrt_trace_stats *stats, uint32_t *per_ray_bounces,
                         void *stream, LaunchCfg c) {
    if (!s || !rays) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL scene / rays");
    if (n_rays < 0 || gid_offset < 0) return fail(WGRT_ERR_INVALID_ARGUMENT, "negative n_rays / gid_offset");
    // launch scratch is allocated and the kernels launched on the scene's device
    DEVICE_SCOPE(dev_scope, s->device);
    const bool single = c.single;
    int variant = c.variant;
    int num_iter = c.num_iter;
    const wgrt_debug_opts *dbg = c.dbg;
    if (single && s->nl != 1)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "single-wavelength trace needs a scene built with num_lmd == 1");
    if (variant != 0 && variant != 1 && variant != 7 && variant != 9)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "kernel variant must be 0 (auto), 1, 7 or 9");
    if (num_iter < 1) num_iter = 1;
    if (num_iter > 255) return fail(WGRT_ERR_INVALID_ARGUMENT, "num_iter must be <= 255");
    if (num_iter > 1 && (per_ray_bounces || c.chunk_order))
        return fail(WGRT_ERR_INVALID_ARGUMENT, "num_iter > 1 takes no per_ray_bounces / chunk_order");
    if (c.chunk_order && variant == 1) return fail(WGRT_ERR_INVALID_ARGUMENT, "chunk_order needs variant 0, 7 or 9");
    if (c.gid_blocks && (c.gid_block_rays < 1 || gid_offset != 0))
        return fail(WGRT_ERR_INVALID_ARGUMENT, "gid_blocks needs gid_block_rays >= 1 and gid_offset == 0");
    if (dbg && (dbg->cert_tol < 0.0 || dbg->cert_tol32 < 0.0 || dbg->chunk_rays < 0 ||
                (dbg->timeline && dbg->timeline_waves < 0)))
        return fail(WGRT_ERR_INVALID_ARGUMENT, "bad wgrt_debug_opts");
    if (n_rays == 0) return WGRT_OK;
    if (!rays->x || !rays->y || !rays->m || !rays->n || (!single && !rays->lmd_num) || !rays->te || !rays->tm ||
        !rays->delta_phase || !rng_states || !matrix_EB)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL ray column / rng_states / matrix_EB");
    if (variant == 7 && !s->d_cells32) return fail(WGRT_ERR_UNSUPPORTED, "variant 7 needs <= 16 polygons");
    if (variant >= 7 && n_rays > 0xffffffffll)
        return fail(WGRT_ERR_UNSUPPORTED, "variants 7 / 9 index at most 2^32 - 1 rays per launch");
    if (variant == 0) variant = n_rays > 0xffffffffll ? 1 : (s->d_cells32 ? 7 : 9);   // auto
    const bool timeline = dbg && dbg->timeline && dbg->timeline_waves > 0;
    if (timeline && (variant != 7 || single))
        return fail(WGRT_ERR_UNSUPPORTED, "the wave timeline is built for the full-colour 32-bit-cell kernel only");
    if (timeline && kAmplify && s->nonunitary_blocks)
        return fail(WGRT_ERR_UNSUPPORTED, "the wave timeline is built without the amplification step: scaled-unitary "
                                          "LUTs only");
    if (num_iter > 1 && variant == 1) {   // chained launches, as the reference issues them
        LaunchCfg one = c;
        one.variant = variant;
        one.num_iter = 1;
        for (int it = 0; it < num_iter; ++it) {
            const wgrt_status e = trace_launch(s, rays, n_rays, gid_offset, rng_states, matrix_EB, stats, nullptr,
                                               stream, one);
            if (e != WGRT_OK) return e;
        }
        return WGRT_OK;
    }
    if (c.chunk_order && c.n_chunk_order != (n_rays + kChunk - 1) / kChunk)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "chunk_order must list ceil(n_rays / 64) chunks");
    TraceArgs A{};
    A.x = rays->x;
    A.y = rays->y;
    A.m = rays->m;
    A.n = rays->n;
    A.l = single ? nullptr : rays->lmd_num;
    A.threshold = single ? 1e-15 : 0.0;
    A.order = c.chunk_order;   // a permutation of the 64-ray chunks (trusted device data)
    A.te = rays->te;
    A.tm = rays->tm;
    A.dph = rays->delta_phase;
    A.rng = rng_states;
    A.eb = matrix_EB;
    A.stats = stats;
    A.per_ray = per_ray_bounces;
    A.n_rays = n_rays;
    A.gid_offset = gid_offset;
    A.gid_blocks = c.gid_blocks;
    A.gid_block_rays = c.gid_blocks ? c.gid_block_rays : 1;
    A.tiles = s->d_tiles;
    A.loc = make_locator(s);
    A.tile_d = s->tile_d;
    A.nfc = s->nfc;
    A.noc = s->noc;
    A.nx = s->nx;
    A.ny = s->ny;
    A.nl = s->nl;
    A.n_g = s->n_g;
    A.inv_n_g = 1.0 / s->n_g;
    A.cert_tol = (dbg && dbg->cert_tol > 0.0) ? dbg->cert_tol : kCertTol;
    // raising the double bound raises this one too
    A.cert_tol32 = std::max((dbg && dbg->cert_tol32 > 0.0) ? dbg->cert_tol32 : kCertTol32, A.cert_tol);
    A.timeline = timeline ? dbg->timeline : nullptr;
    A.timeline_waves = timeline ? dbg->timeline_waves : 0;
    A.jtiles = s->d_jtiles;
    A.jtile_d = s->jtile_d;
    A.n_iter = 1;
    hipStream_t st = (hipStream_t)stream;
    if (variant == 1) {
        const int64_t blocks = (n_rays + 255) / 256;
        if (blocks > 0x7fffffff) return fail(WGRT_ERR_INVALID_ARGUMENT, "too many rays for one launch");
        hipLaunchKernelGGL(trace_grid_kernel, dim3((unsigned)blocks), dim3(256), 0, st, A);
        HIP_TRY(hipGetLastError());
        return WGRT_OK;
    }
    int64_t grid = c.workgroups > 0 ? c.workgroups
                   : timeline     ? s->jones_tl_grid[num_iter > 1]
                                  : s->jones_grid[variant == 9][num_iter > 1][single];
    // a workgroup's 4 waves need 4 work items to all have work (debug chunk_rays: smaller items)
    const int64_t item = (dbg && dbg->chunk_rays > 0) ? std::min(dbg->chunk_rays, 64) : kChunk;
    const int64_t useful = (n_rays + 4 * item - 1) / (4 * item);
    if (c.workgroups <= 0 && num_iter <= 1 && c.grid_k >= 0.0) {
        // a single trace ends with the drain of its longest ray chains, and chains run faster
        // on a less crowded chip, while the bulk before it wants every resident wave: the grid
        // that balances bulk throughput (work / W) against drain crowding (~ W) grows as
        // sqrt(work items).  K = 6.5 workgroups per sqrt(item), measured: C2
        // (1,936 items, 287 workgroups) -11 %, half and quarter C3 shards -8 / -12 %; C3 (946)
        // unchanged; C4 and larger keep the resident grid
        const double K = c.grid_k > 0.0 ? c.grid_k : kGridSqrtK;
        const int64_t items = (n_rays + item - 1) / item;
        const int64_t want = std::max<int64_t>(1, (int64_t)std::ceil(K * std::sqrt((double)items)));
        if (grid > want) grid = want;
    }
    if (grid > useful) grid = useful;
    wgrt_scene *ms = const_cast<wgrt_scene *>(s);
    wgrt_scene::Scratch *sc = nullptr;
    uint32_t epoch = 0, parity = 0;
    {
        const wgrt_status e =
            ensure_scratch(ms, stream, n_rays, num_iter, grid, &sc, num_iter > 1 ? &epoch : nullptr, &parity);
        if (e != WGRT_OK) return e;
    }
    unsigned long long *const ctr = sc->ctr + (size_t)parity * kScratchCtr;
    if (num_iter > 1) {
        A.n_iter = num_iter;
        A.rng64 = sc->rng64;
        A.iter_epoch = epoch;
        A.handoff_wait_ticks = (dbg && dbg->handoff_wait_ticks) ? dbg->handoff_wait_ticks
                                                                : kHandoffTicksPerIter * (unsigned long long)(num_iter + 1);
        // a debug bound (fault-injection tests) gives up on the clock alone
        A.handoff_min_passes = (dbg && dbg->handoff_wait_ticks) ? 0u : kHandoffMinPasses;
    }
    A.replay_count = ctr + kHeads * kHeadStride;
    A.replay_list = sc->list;
    A.q_xy = sc->q_xy;
    A.q_i = sc->q_i;
    A.q_count = ctr + (kHeads + 1) * kHeadStride;
    A.full_count = ctr + (kHeads + 2) * kHeadStride;
    A.full_list = sc->full;
    A.epi_acc = ctr + (kHeads + 3) * kHeadStride;
    A.epi_done = ctr + (kHeads + 4) * kHeadStride;
    A.heads0 = ctr;
    A.other_ctr = sc->ctr + (size_t)(parity ^ 1u) * kScratchCtr;
    A.part = sc->part;
    A.n_trace_waves = (int)grid;   // one partial slot per trace workgroup
    // chunk_order is given in 64-ray chunks; a staged chunk is one ray per lane
    const int jchunk = A.order ? kChunk : ((dbg && dbg->chunk_rays > 0) ? std::min(dbg->chunk_rays, 64) : kChunk);
    const dim3 g3((unsigned)grid), b3(256);
    // instantiations: cell word width x fused chain x single-wavelength guard
#define WGRT_LAUNCH_JONES_A(CELL, LOCV, AMPV)                                                                      \
    do {                                                                                                           \
        if (num_iter > 1 && single)                                                                                \
            hipLaunchKernelGGL((trace_jones_kernel<CELL, true, true, AMPV>), g3, b3, 0, st, A, LOCV, ctr, jchunk);  \
        else if (num_iter > 1)                                                                                     \
            hipLaunchKernelGGL((trace_jones_kernel<CELL, true, false, AMPV>), g3, b3, 0, st, A, LOCV, ctr, jchunk); \
        else if (single)                                                                                           \
            hipLaunchKernelGGL((trace_jones_kernel<CELL, false, true, AMPV>), g3, b3, 0, st, A, LOCV, ctr, jchunk); \
        else                                                                                                       \
            hipLaunchKernelGGL((trace_jones_kernel<CELL, false, false, AMPV>), g3, b3, 0, st, A, LOCV, ctr, jchunk);\
    } while (0)
    // the amplification step only for scenes that need it (wgrt_device.h kAmplify)
#define WGRT_LAUNCH_JONES(CELL, LOCV)                                  \
    do {                                                               \
        if (kAmplify && s->nonunitary_blocks) WGRT_LAUNCH_JONES_A(CELL, LOCV, true);  \
        else WGRT_LAUNCH_JONES_A(CELL, LOCV, false);                   \
    } while (0)
    if (timeline) {
        const LocatorT<uint32_t> l32 = make_locator32(s);
        if (num_iter > 1)
            hipLaunchKernelGGL((trace_jones_tl_kernel<uint32_t, true, false>), g3, b3, 0, st, A, l32, ctr, jchunk);
        else
            hipLaunchKernelGGL((trace_jones_tl_kernel<uint32_t, false, false>), g3, b3, 0, st, A, l32, ctr, jchunk);
    } else if (variant == 9) {
        WGRT_LAUNCH_JONES(uint64_t, A.loc);
    } else {
        const LocatorT<uint32_t> l32 = make_locator32(s);
        WGRT_LAUNCH_JONES(uint32_t, l32);
    }
#undef WGRT_LAUNCH_JONES
#undef WGRT_LAUNCH_JONES_A
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && dbg && dbg->fail_after_trace) {
        mark_dirty(ms, sc);
        return fail(WGRT_ERR_HIP, "fault injection: failed after the trace kernel (wgrt_debug_opts.fail_after_trace)");
    }
    if (e == hipSuccess) {
        // fused launches keep the epilogue kernel (their replays chain the traces after the abandoned one)
        if (num_iter > 1 || !kInKernelEpilogue)
            hipLaunchKernelGGL(epilogue_kernel, dim3(kEpilogueGroups), dim3(256), 0, st, A);
        else if (!WGRT_INKERNEL_REPLAY)   // else the last trace workgroup replays (jones_body)
            hipLaunchKernelGGL(replay_kernel, dim3(kReplayGroups), dim3(256), 0, st, A);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        mark_dirty(ms, sc);
        return fail(WGRT_ERR_HIP, std::string("trace launch: ") + hipGetErrorString(e));
    }
    return WGRT_OK;
}

LaunchCfg cfg_of(int variant, int workgroups, bool single) {
    LaunchCfg c;
    c.variant = variant;
    c.workgroups = workgroups;
    c.single = single;
    return c;
}

}  // namespace

extern "C" {

wgrt_status wgrt_scene_reserve(const wgrt_scene *s, int64_t n_rays, int num_iter, void *stream) {
    if (!s) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL scene");
    if (n_rays < 0 || num_iter < 0 || num_iter > 255) return fail(WGRT_ERR_INVALID_ARGUMENT, "bad n_rays / num_iter");
    if (n_rays == 0) return WGRT_OK;
    DEVICE_SCOPE(dev_scope, s->device);
    int64_t grid = 0;
    for (int c = 0; c < 2; ++c)
        for (int f = 0; f < 2; ++f)
            for (int g = 0; g < 2; ++g) grid = std::max<int64_t>(grid, s->jones_grid[c][f][g]);
    wgrt_scene::Scratch *sc = nullptr;
    return ensure_scratch(const_cast<wgrt_scene *>(s), stream, n_rays, std::max(num_iter, 1),
                          std::min<int64_t>(grid, (n_rays + 255) / 256), &sc);
}

wgrt_status wgrt_trace_fullcolor_ex(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays,
                                    int64_t gid_offset, uint32_t *rng_states, float *matrix_EB,
                                    wgrt_trace_stats *stats, uint32_t *per_ray_bounces, void *stream,
                                    int variant, int workgroups) {
    return trace_launch(s, rays, n_rays, gid_offset, rng_states, matrix_EB, stats, per_ray_bounces, stream,
                        cfg_of(variant, workgroups, false));
}

wgrt_status wgrt_trace_fullcolor(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays,
                                 int64_t gid_offset, uint32_t *rng_states, float *matrix_EB,
                                 wgrt_trace_stats *stats, uint32_t *per_ray_bounces, void *stream) {
    return trace_launch(s, rays, n_rays, gid_offset, rng_states, matrix_EB, stats, per_ray_bounces, stream,
                        cfg_of(0, 0, false));
}

wgrt_status wgrt_trace_opts(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays, int64_t gid_offset,
                            uint32_t *rng_states, float *matrix_EB, wgrt_trace_stats *stats,
                            uint32_t *per_ray_bounces, void *stream, const wgrt_launch_opts *opts) {
    if (!opts) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL opts");
    if (opts->kernel != 0 && opts->kernel != 1) return fail(WGRT_ERR_INVALID_ARGUMENT, "kernel must be 0 or 1");
    LaunchCfg c = cfg_of(opts->variant, opts->workgroups, opts->kernel == 1);
    c.chunk_order = opts->chunk_order;
    c.n_chunk_order = opts->n_chunk_order;
    c.num_iter = opts->num_iter;
    c.gid_blocks = opts->gid_blocks;
    c.gid_block_rays = opts->gid_block_rays;
    c.dbg = opts->debug;
    c.grid_k = opts->grid_sqrt_k;
    if (!(c.grid_k == c.grid_k)) return fail(WGRT_ERR_INVALID_ARGUMENT, "grid_sqrt_k is NaN");
    return trace_launch(s, rays, n_rays, gid_offset, rng_states, matrix_EB, stats, per_ray_bounces, stream, c);
}

wgrt_status wgrt_trace_single_ex(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays, int64_t gid_offset,
                                 uint32_t *rng_states, float *matrix_EB, wgrt_trace_stats *stats,
                                 uint32_t *per_ray_bounces, void *stream, int variant, int workgroups) {
    return trace_launch(s, rays, n_rays, gid_offset, rng_states, matrix_EB, stats, per_ray_bounces, stream,
                        cfg_of(variant, workgroups, true));
}

wgrt_status wgrt_trace_single(const wgrt_scene *s, const wgrt_rays *rays, int64_t n_rays, int64_t gid_offset,
                              uint32_t *rng_states, float *matrix_EB, wgrt_trace_stats *stats,
                              uint32_t *per_ray_bounces, void *stream) {
    return trace_launch(s, rays, n_rays, gid_offset, rng_states, matrix_EB, stats, per_ray_bounces, stream,
                        cfg_of(0, 0, true));
}

wgrt_status wgrt_scene_classify(const wgrt_scene *s, const double *xy, int64_t n, uint64_t *out_mask,
                                void *stream) {
    if (!s || (n > 0 && (!xy || !out_mask))) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n <= 0) return WGRT_OK;
    DEVICE_SCOPE(dev_scope, s->device);
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(classify_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       make_locator(s), s->npoly, xy, n, out_mask);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

wgrt_status wgrt_rays_init(const double *points, int64_t rays_per_fov, int32_t nx, int32_t ny,
                           const int32_t *lambdas, int32_t n_lambdas, int64_t block_lo, int64_t block_hi,
                           const wgrt_ray_columns *out, uint32_t *rng_states, void *stream) {
    if (!out || !lambdas) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL columns / lambdas");
    if (rays_per_fov < 1 || nx < 1 || ny < 1) return fail(WGRT_ERR_INVALID_ARGUMENT, "sizes must be positive");
    if (n_lambdas < 1 || n_lambdas > 8) return fail(WGRT_ERR_INVALID_ARGUMENT, "1..8 wavelengths");
    const int64_t nblk = (int64_t)nx * ny * n_lambdas;
    if (block_lo < 0 || block_lo > block_hi || block_hi > nblk)
        return fail(WGRT_ERR_INVALID_ARGUMENT, "block range outside [0, nx * ny * n_lambdas]");
    if (rays_per_fov >= 2 && !points) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL points");
    RayInitArgs A{};
    A.points = points;
    float *const cols[12] = {out->x, out->y, out->gap_x, out->gap_y, out->pol, out->azi, out->m, out->n,
                             out->lmd_num, out->te, out->tm, out->delta_phase};
    for (int c = 0; c < 12; ++c) A.col[c] = cols[c];
    A.rng = rng_states;
    A.n = (block_hi - block_lo) * rays_per_fov;
    A.R = rays_per_fov;
    A.blk_lo = block_lo;
    A.gid_offset = block_lo * rays_per_fov;
    A.ny = ny;
    A.nl = n_lambdas;
    for (int k = 0; k < n_lambdas; ++k) A.lambdas[k] = (float)lambdas[k];
    if (A.n == 0) return WGRT_OK;
    // no scene: the kernel runs on the stream's device
    int sdev = 0;
    HIP_TRY(stream_device(stream, &sdev));
    DEVICE_SCOPE(dev_scope, sdev);
    const int64_t blocks = std::min<int64_t>((A.n + 255) / 256, 65536);
    hipLaunchKernelGGL(rays_init_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, A);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

int64_t wgrt_eyebox_payload_floats(int64_t nb) { return nb < 0 ? -1 : nb * WGRT_EB_SLAB + eb_spill_floats(nb); }

wgrt_status wgrt_eyebox_pack(const float *eb, int64_t n_slabs, const int64_t *slabs, const int64_t *next,
                             const float *spill_mask, int64_t n, int64_t nb, float *payload, void *stream) {
    if (n < 0 || nb < n || n_slabs < 0) return fail(WGRT_ERR_INVALID_ARGUMENT, "need 0 <= n <= nb and n_slabs >= 0");
    if (n == 0) return WGRT_OK;
    if (!eb || !slabs || !next || !spill_mask || !payload) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (((uintptr_t)eb | (uintptr_t)payload) & 15) return fail(WGRT_ERR_INVALID_ARGUMENT, "eb / payload must be 16-B aligned");
    if (n > 65535) return fail(WGRT_ERR_INVALID_ARGUMENT, "at most 65535 slabs per rank");
    int sdev = 0;
    HIP_TRY(stream_device(stream, &sdev));
    DEVICE_SCOPE(dev_scope, sdev);
    hipLaunchKernelGGL(eyebox_pack_kernel, dim3(kEbSlabParts, (unsigned)n), dim3(256), 0, (hipStream_t)stream, eb,
                       n_slabs, slabs, next, spill_mask, n, nb, payload);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

wgrt_status wgrt_eyebox_assemble(float *eb, int64_t n_slabs, const float *recv, int32_t world, int64_t nb,
                                 const int64_t *dst, const int64_t *spill_dst, void *stream) {
    if (world < 0 || nb < 0 || n_slabs < 0) return fail(WGRT_ERR_INVALID_ARGUMENT, "negative world / nb / n_slabs");
    const int64_t rows = (int64_t)world * nb;
    if (rows == 0) return WGRT_OK;
    if (!eb || !recv || !dst || !spill_dst) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (((uintptr_t)eb | (uintptr_t)recv) & 15) return fail(WGRT_ERR_INVALID_ARGUMENT, "eb / recv must be 16-B aligned");
    if (rows > 65535) return fail(WGRT_ERR_INVALID_ARGUMENT, "at most 65535 payload rows");
    int sdev = 0;
    HIP_TRY(stream_device(stream, &sdev));
    DEVICE_SCOPE(dev_scope, sdev);
    const int64_t plen = wgrt_eyebox_payload_floats(nb);
    hipLaunchKernelGGL(eyebox_copy_kernel, dim3(kEbSlabParts, (unsigned)rows), dim3(256), 0, (hipStream_t)stream, eb,
                       n_slabs, recv, nb, plen, dst);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(eyebox_spill_kernel, dim3((unsigned)rows), dim3(128), 0, (hipStream_t)stream, eb, n_slabs, recv,
                       nb, plen, spill_dst);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

wgrt_status wgrt_selftest_math(const double *a, const double *b, int64_t n, double *out, void *stream) {
    if (n > 0 && (!a || !b || !out)) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n <= 0) return WGRT_OK;
    int sdev = 0;
    HIP_TRY(stream_device(stream, &sdev));
    DEVICE_SCOPE(dev_scope, sdev);
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(selftest_math_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, b,
                       n, out);
    HIP_TRY(hipGetLastError());
    return WGRT_OK;
}

wgrt_status wgrt_locator_classify_host(const wgrt_scene_desc *desc, double cell_mm, const double *xy, int64_t n,
                                       uint64_t *out_mask) {
    if (!desc || (n > 0 && (!xy || !out_mask))) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (!(cell_mm > 0.0)) return fail(WGRT_ERR_INVALID_ARGUMENT, "cell_mm must be > 0");
    SceneHost host;
    try {
        build_scene_host(*desc, cell_mm, host);
    } catch (const std::exception &e) {
        return fail(WGRT_ERR_INVALID_ARGUMENT, e.what());
    }
    const int npoly = (int)host.loc.poly_off.size() - 1;
    // host replica of the device locator (same arithmetic as locate / in_poly)
    LocatorT<uint64_t> g{};
    g.cells = host.loc.cells.data();
    g.verts = host.loc.verts.data();
    g.poly_off = host.loc.poly_off.data();
    g.row_off = host.loc.row_off.data();
    g.row_edges = host.loc.row_edges.data();
    g.x0 = host.loc.x0, g.y0 = host.loc.y0, g.inv_h = host.loc.inv_h, g.ncx = host.loc.ncx, g.ncy = host.loc.ncy;
    for (int64_t i = 0; i < n; ++i) {
        const double x = xy[2 * i], y = xy[2 * i + 1];
        const double fx = std::floor((x - g.x0) * g.inv_h), fy = std::floor((y - g.y0) * g.inv_h);
        uint64_t w = 0;
        int cy = 0;
        if (fx >= 0.0 && fy >= 0.0 && fx < (double)g.ncx && fy < (double)g.ncy) {
            cy = (int)fy;
            w = g.cells[(size_t)cy * g.ncx + (int)fx];
        }
        uint64_t mask = 0;
        for (int k = 0; k < npoly; ++k) {
            const unsigned cls = (unsigned)(w >> (2 * k)) & 3u;
            bool in = cls == 1u;
            if (cls == 2u) {
                const int a = g.poly_off[k], nv = g.poly_off[k + 1] - a;
                const int r = k * g.ncy + cy;
                in = inside_or_on_edge_subset(x, y, g.verts + 2 * a, nv, g.row_edges + g.row_off[r],
                                              g.row_off[r + 1] - g.row_off[r]);
            }
            if (in) mask |= 1ull << k;
        }
        out_mask[i] = mask;
    }
    return WGRT_OK;
}

wgrt_status wgrt_debug_scene_copy(const wgrt_scene *s, int which, void *dst, int64_t bytes) {
    if (!s || !dst) return fail(WGRT_ERR_INVALID_ARGUMENT, "NULL scene / dst");
    const size_t ncells = (size_t)s->loc_host.ncx * s->loc_host.ncy;
    const void *src = nullptr;
    size_t n = 0;
    switch (which) {
        case 0: src = s->d_cells, n = ncells * sizeof(uint64_t); break;
        case 1: src = s->d_tiles, n = (size_t)s->tiles * s->tile_d * sizeof(double); break;
        case 2: src = s->d_jtiles, n = (size_t)s->tiles * s->jtile_d * sizeof(double); break;
        default: return fail(WGRT_ERR_INVALID_ARGUMENT, "which: 0 cells, 1 tiles, 2 jtiles");
    }
    if (bytes != (int64_t)n) return fail(WGRT_ERR_INVALID_ARGUMENT, "bytes must be " + std::to_string(n));
    DEVICE_SCOPE(dev_scope, s->device);
    HIP_TRY(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
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
