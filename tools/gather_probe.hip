// gather_probe.hip -- cost model of per-lane vector-memory gathers on gfx950 (what the bounce
// kernel's passes are made of).  Every CU runs `waves` resident waves; each wave issues `iters`
// rounds of 8 independent 16-B-per-lane loads (dwordx4), the next round's addresses depending
// on the previous round's data (a dependent chain, like a ray's bounces).  Knobs per run:
//   lanes  -- active lanes per load instruction (the others masked off)
//   lines  -- distinct 128-B lines one instruction touches (lane l reads line l % lines)
//   span   -- bytes of the table the lines are drawn from (L1-hot: 16 KB; L2: 2 MB; beyond: 64 MB+)
// Prints one JSON line per configuration: ns per round and CU cycles per load wave-instruction.
// Build: hipcc -O3 --offload-arch=gfx950 -o gather_probe tools/gather_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__global__ __launch_bounds__(256) void probe(const uint4 *tab, uint64_t span_lines, int lanes, int lines, int iters,
                                             unsigned *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    unsigned h = (unsigned)(wave * 2654435761u);
    unsigned acc = 0;
    if (lane < lanes) {
        for (int it = 0; it < iters; ++it) {
            uint4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                // one base line per (wave, round, k); lanes spread over `lines` lines near it
                const unsigned hk = (h + (unsigned)k * 0x9E3779B9u) * 0x85EBCA6Bu;
                const uint64_t line = ((uint64_t)hk + (uint64_t)(lane % lines) * 7919u) % span_lines;
                v[k] = tab[line * 8 + (lane & 7)];
            }
            unsigned s = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) s += v[k].x ^ v[k].w;
            acc += s;
            h = h * 1664525u + 1013904223u + (s == 0x5a5a5a5au);   // the next round depends on this one's data
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv) {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    int clk_khz = 0;
    CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    const size_t tab_bytes = (size_t)256 << 20;
    uint4 *tab = nullptr;
    unsigned *out = nullptr;
    CHECK(hipMalloc(&tab, tab_bytes));
    CHECK(hipMemset(tab, 1, tab_bytes));
    CHECK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int iters = 200;
    const int waves_opts[] = {20, 8};
    const int lanes_opts[] = {64, 32, 16, 4};
    const int lines_opts[] = {1, 4, 16, 64};
    const size_t span_opts[] = {(size_t)16 << 10, (size_t)2 << 20, (size_t)64 << 20};
    for (int waves : waves_opts)
        for (size_t span : span_opts)
            for (int lanes : lanes_opts)
                for (int lines : lines_opts) {
                    if (lines > lanes) continue;
                    const int wg = cus * waves / 4;
                    const uint64_t span_lines = span / 128;
                    hipLaunchKernelGGL(probe, dim3(wg), dim3(256), 0, 0, tab, span_lines, lanes, lines, 4, out);
                    CHECK(hipEventRecord(e0));
                    hipLaunchKernelGGL(probe, dim3(wg), dim3(256), 0, 0, tab, span_lines, lanes, lines, iters, out);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float ms = 0;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    const double ns_round = ms * 1e6 / iters;
                    // load wave-instructions per CU per round = waves * 8
                    const double cyc_per_inst = ns_round * 1e-9 * clk_khz * 1e3 / (waves * 8.0);
                    printf("{\"waves_per_cu\": %d, \"span\": %zu, \"lanes\": %d, \"lines\": %d, \"ns_per_round\": %.1f, "
                           "\"cu_cycles_per_load_inst\": %.2f}\n",
                           waves, span, lanes, lines, ns_round, cyc_per_inst);
                    fflush(stdout);
                }
    return 0;
}
