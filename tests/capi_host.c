/*
 * capi_host.c -- a plain C99 host of libwgrt.so: the drop-in boundary used without Python.
 *
 * It does what the reference driver does around its kernel (gpu_ray_tracing_pro_fullColor.py:
 * 40-57 upload the scene, :158-177 seed and launch num_iter times, :178-179 copy back), through
 * include/wgrt.h and the HIP runtime only:
 *
 *   capi_host IN OUT
 *
 * IN (written by tests/test_capi_host.py): a sequence of records, each an int64 element count
 * followed by the elements, in the order read below (geometry, LUTs as interleaved complex128,
 * the scalar block, the eight float32 ray columns the kernel reads, the uint32 RNG states).
 * OUT: rng_states after the launches (uint32[n]), matrix_EB (float32), wgrt_trace_stats (7 x u64, ABI 7).
 * Exit status 0 on success; a failing call prints wgrt_last_error() and exits 2.
 * Built by __graft_entry__.build() (gcc, tests/_capi.py) into tests/bin/; no torch, no Python.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "wgrt.h"

#define HIP_CHECK(e)                                                                        \
    do {                                                                                    \
        hipError_t err_ = (e);                                                              \
        if (err_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #e, hipGetErrorString(err_)); \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

#define WGRT_CHECK(e)                                                                           \
    do {                                                                                        \
        wgrt_status st_ = (e);                                                                  \
        if (st_ != WGRT_OK) {                                                                   \
            fprintf(stderr, "%s: %s (%s)\n", #e, wgrt_status_string(st_), wgrt_last_error());   \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

static FILE *in_file;

/* One record of elem-byte elements; *count receives the element count. */
static void *read_record(size_t elem, int64_t *count) {
    int64_t n = 0;
    if (fread(&n, sizeof n, 1, in_file) != 1 || n < 0) {
        fprintf(stderr, "truncated input\n");
        exit(2);
    }
    void *p = malloc(n > 0 ? (size_t)n * elem : 1);
    if (!p || (n > 0 && fread(p, elem, (size_t)n, in_file) != (size_t)n)) {
        fprintf(stderr, "truncated input\n");
        exit(2);
    }
    if (count) *count = n;
    return p;
}

/* A host array copied to a new device buffer. */
static void *to_device(const void *h, size_t bytes) {
    void *d = NULL;
    HIP_CHECK(hipMalloc(&d, bytes > 0 ? bytes : 1));
    if (bytes) HIP_CHECK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s IN OUT\n", argv[0]);
        return 1;
    }
    if (wgrt_abi_version() != WGRT_ABI_VERSION) {
        fprintf(stderr, "libwgrt ABI %d, header %d\n", wgrt_abi_version(), WGRT_ABI_VERSION);
        return 2;
    }
    in_file = fopen(argv[1], "rb");
    if (!in_file) {
        perror(argv[1]);
        return 2;
    }
    int64_t n_ic, n_fc, n_fco, n_oc, n_oco, n_e1, n_e2, n_sc;
    wgrt_scene_desc d;
    memset(&d, 0, sizeof d);
    d.IC = read_record(sizeof(double), &n_ic);
    d.FC = read_record(sizeof(double), &n_fc);
    d.FC_offset = read_record(sizeof(int64_t), &n_fco);
    d.OC = read_record(sizeof(double), &n_oc);
    d.OC_offset = read_record(sizeof(int64_t), &n_oco);
    d.eff_reg1 = read_record(sizeof(double), &n_e1);
    d.eff_reg2 = read_record(sizeof(double), &n_e2);
    d.eff_reg_FOV = read_record(sizeof(double), NULL);
    d.eff_reg_FOV_range = read_record(sizeof(double), NULL);
    d.lut_ic1 = read_record(sizeof(double), NULL);
    d.lut_ic2 = read_record(sizeof(double), NULL);
    d.lut_ic3 = read_record(sizeof(double), NULL);
    d.lut_fc1 = read_record(sizeof(double), NULL);
    d.lut_fc2 = read_record(sizeof(double), NULL);
    d.lut_oc1 = read_record(sizeof(double), NULL);
    d.lut_oc2 = read_record(sizeof(double), NULL);
    d.lut_TIR = read_record(sizeof(double), NULL);
    d.lut_gap = read_record(sizeof(double), NULL);
    /* scalars: n_g as a double record, then int64 {ch5, ch3, num_lmd, nx, ny, num_iter} */
    const double *ng = read_record(sizeof(double), NULL);
    const int64_t *sc = read_record(sizeof(int64_t), &n_sc);
    if (n_sc != 6) {
        fprintf(stderr, "bad scalar record\n");
        return 2;
    }
    d.n_ic = n_ic / 2;
    d.n_fc_slices = n_fco - 1;
    d.n_oc_slices = n_oco - 1;
    d.n_eff_reg1 = n_e1 / 2;
    d.n_eff_reg2 = n_e2 / 2;
    d.n_g = ng[0];
    d.ch5 = (int32_t)sc[0];
    d.ch3 = (int32_t)sc[1];
    d.num_lmd = (int32_t)sc[2];
    d.nx = (int32_t)sc[3];
    d.ny = (int32_t)sc[4];
    const int num_iter = (int)sc[5];

    /* the eight columns the kernel reads (MAIN:65-76 order without gap_x, gap_y, pol, azi) */
    int64_t n = 0;
    float *cols[8];
    for (int k = 0; k < 8; ++k) {
        int64_t nk = 0;
        cols[k] = read_record(sizeof(float), &nk);
        if (k == 0) n = nk;
        if (nk != n) {
            fprintf(stderr, "ragged ray columns\n");
            return 2;
        }
    }
    int64_t n_rng = 0;
    uint32_t *rng = read_record(sizeof(uint32_t), &n_rng);
    fclose(in_file);
    if (n_rng != n) {
        fprintf(stderr, "rng_states length %lld != %lld rays\n", (long long)n_rng, (long long)n);
        return 2;
    }

    HIP_CHECK(hipSetDevice(0));
    wgrt_scene *scene = NULL;
    WGRT_CHECK(wgrt_scene_create(&d, 0, &scene));   /* MAIN:40-57 */

    const size_t fb = (size_t)n * sizeof(float);
    wgrt_rays rays;
    memset(&rays, 0, sizeof rays);   /* gap_x, gap_y, pol, azi: never read (GRTF:872-894) */
    rays.x = to_device(cols[0], fb);
    rays.y = to_device(cols[1], fb);
    rays.m = to_device(cols[2], fb);
    rays.n = to_device(cols[3], fb);
    rays.lmd_num = to_device(cols[4], fb);
    rays.te = to_device(cols[5], fb);
    rays.tm = to_device(cols[6], fb);
    rays.delta_phase = to_device(cols[7], fb);
    uint32_t *d_rng = to_device(rng, (size_t)n * sizeof(uint32_t));
    const size_t eb_n = (size_t)d.num_lmd * d.ny * d.nx * 80 * 120;   /* MAIN:37 */
    float *d_eb = NULL;
    HIP_CHECK(hipMalloc((void **)&d_eb, eb_n * sizeof(float)));
    HIP_CHECK(hipMemset(d_eb, 0, eb_n * sizeof(float)));
    wgrt_trace_stats *d_stats = NULL;
    HIP_CHECK(hipMalloc((void **)&d_stats, sizeof(wgrt_trace_stats)));
    HIP_CHECK(hipMemset(d_stats, 0, sizeof(wgrt_trace_stats)));
    hipStream_t stream;
    HIP_CHECK(hipStreamCreate(&stream));

    /* the reference's launch loop, MAIN:169-177: num_iter launches, one call each */
    for (int it = 0; it < num_iter; ++it)
        WGRT_CHECK(wgrt_trace_fullcolor(scene, &rays, n, 0, d_rng, d_eb, d_stats, NULL, stream));
    HIP_CHECK(hipStreamSynchronize(stream));   /* MAIN:178 */

    float *eb = malloc(eb_n * sizeof(float));
    wgrt_trace_stats stats;
    if (!eb) return 2;
    HIP_CHECK(hipMemcpy(rng, d_rng, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(eb, d_eb, eb_n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(&stats, d_stats, sizeof stats, hipMemcpyDeviceToHost));
    FILE *out = fopen(argv[2], "wb");
    if (!out) {
        perror(argv[2]);
        return 2;
    }
    fwrite(rng, sizeof(uint32_t), (size_t)n, out);
    fwrite(eb, sizeof(float), eb_n, out);
    fwrite(&stats, sizeof stats, 1, out);
    fclose(out);

    HIP_CHECK(hipStreamDestroy(stream));
    WGRT_CHECK(wgrt_scene_destroy(scene));
    printf("capi_host: %lld rays x %d launches, %llu bounces, %llu eyebox hits\n", (long long)n, num_iter,
           (unsigned long long)stats.bounces, (unsigned long long)stats.eyebox_hits);
    return 0;
}
