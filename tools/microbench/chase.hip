// Dependent-load latency on the GPU: one lane pointer-chases a random cyclic permutation
// of uint32 indices spread over a buffer of S bytes (one index per 64-B line), and reports
// shader-clock cycles per load.  Tells what one locator-cell / tile fetch costs at idle.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ void chase(const uint32_t *next, int steps, uint32_t start, unsigned long long *out) {
    uint32_t p = start;
    // warm the TLB / caches along the path once
    for (int k = 0; k < steps; ++k) p = next[p];
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int k = 0; k < steps; ++k) p = next[p];
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[0] = t1 - t0;
    out[1] = p;
}

int main() {
    const size_t sizes_mb[] = {1, 4, 16, 36, 128, 512, 2048};
    for (size_t mb : sizes_mb) {
        const size_t bytes = mb << 20;
        const size_t lines = bytes / 64;
        std::vector<uint32_t> perm(lines);
        for (size_t i = 0; i < lines; ++i) perm[i] = (uint32_t)i;
        std::mt19937_64 g(42);
        std::shuffle(perm.begin(), perm.end(), g);
        std::vector<uint32_t> host(bytes / 4, 0);
        for (size_t i = 0; i < lines; ++i) host[(size_t)perm[i] * 16] = perm[(i + 1) % lines] * 16;
        uint32_t *d = nullptr;
        unsigned long long *o = nullptr;
        if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 16) != hipSuccess) return 1;
        if (hipMemcpy(d, host.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return 1;
        const int steps = 4096;
        hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, d, steps, perm[0] * 16, o);
        unsigned long long r[2];
        if (hipMemcpy(r, o, 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("{\"buffer_mb\": %zu, \"cycles_per_load\": %.1f}\n", mb, (double)r[0] / steps);
        fflush(stdout);
        (void)hipFree(d);
        (void)hipFree(o);
    }
    return 0;
}
