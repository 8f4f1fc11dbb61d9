// chase_probe.hip -- dependent-load latency on gfx950 for the bounce kernel's cell-word gathers:
// every lane follows its own pointer chain (4-B words, a random cyclic permutation over `span`
// bytes), so each load waits for the previous one.  Runs `waves` waves per CU; prints one JSON
// line per (span, waves, lanes): ns and shader cycles per dependent load.
// Build: hipcc -O3 --offload-arch=gfx950 -o chase_probe tools/chase_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__global__ __launch_bounds__(256) void chase(const uint32_t *next, uint32_t n, int lanes, int hops, uint32_t *out) {
    const int lane = threadIdx.x & 63;
    if (lane >= lanes) return;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t p = (uint32_t)((g * 2654435761ull) % n);
    for (int h = 0; h < hops; ++h) p = next[p];
    if (p == 0xffffffffu) out[0] = p;
}

int main() {
    int cus = 0, clk_khz = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    uint32_t *out = nullptr;
    CHECK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const size_t spans[] = {(size_t)1 << 20, (size_t)2 << 20, (size_t)4 << 20, (size_t)8 << 20, (size_t)72 << 20};
    std::mt19937_64 rng(1);
    for (size_t span : spans) {
        const uint32_t n = (uint32_t)(span / 4);
        // a random cyclic permutation (Sattolo), chains stride across the whole span
        std::vector<uint32_t> perm(n);
        std::iota(perm.begin(), perm.end(), 0u);
        for (uint32_t i = n - 1; i > 0; --i) std::swap(perm[i], perm[rng() % i]);
        uint32_t *d = nullptr;
        CHECK(hipMalloc(&d, span));
        CHECK(hipMemcpy(d, perm.data(), span, hipMemcpyHostToDevice));
        const int cfg[][2] = {{1, 1}, {1, 64}, {4, 20}, {16, 20}, {16, 64}};   // {waves per CU, lanes}
        for (auto &c : cfg) {
            const int waves = c[0], lanes = c[1];
            const int wg = std::max(1, cus * waves / 4);
            const int hops = 2000;
            hipLaunchKernelGGL(chase, dim3(wg), dim3(waves == 1 ? 64 : 256), 0, 0, d, n, lanes, 50, out);
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(chase, dim3(waves == 1 ? cus : wg), dim3(waves == 1 ? 64 : 256), 0, 0, d, n, lanes,
                               hops, out);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double ns = ms * 1e6 / hops;
            printf("{\"span_mb\": %zu, \"waves_per_cu\": %d, \"lanes\": %d, \"ns_per_load\": %.1f, \"cycles_per_load\": %.0f}\n",
                   span >> 20, waves, lanes, ns, ns * clk_khz * 1e-6);
            fflush(stdout);
        }
        CHECK(hipFree(d));
    }
    return 0;
}
