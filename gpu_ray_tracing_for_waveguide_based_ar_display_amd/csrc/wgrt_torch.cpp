// wgrt_torch.cpp -- the bounce kernel as a PyTorch-ROCm operator: torch.ops.wgrt.trace.
//
// The launch path the Python layer takes for torch tensors (engine.trace_fullcolor / trace_single):
// one call of process_rays_kernel_pro_fullColor[blocks, tpb](...) or process_rays_kernel_pro[...]
// (GRTF:833-1246 / 419-831, launched at MAIN:167-177) on device tensors, forwarded to the C ABI's
// wgrt_trace_opts (include/wgrt.h) on the caller's stream.  The operator holds no state and does
// no arithmetic: it checks every tensor against the scene (device, dtype, layout, length), builds
// the wgrt_rays / wgrt_launch_opts records and returns the library's status; the Python layer
// raises on a nonzero status with wgrt_last_error()'s detail.  Tensor misuse raises here
// (c10::Error) even for callers that skip the Python checks.
//
// libwgrt.so is not a link dependency: its symbols resolve against the global scope, where the
// Python layer loaded it (RTLD_GLOBAL, _lib.load) -- the in-tree build or the one WGRT_LIB names,
// so the operator and the ctypes entry points always share one library and one set of scenes.  The
// extension is linked with -z now, so loading it without libwgrt fails at load time, not mid-call.
#include <torch/library.h>

#include <ATen/core/Tensor.h>
#include <c10/core/DeviceGuard.h>

#include <cstdint>
#include <optional>

#include "wgrt.h"

namespace {

using at::Tensor;

struct Ctx {
    c10::Device dev;
    int64_t rays;   // length of every ray column (the batch)
};

void on_device(const Tensor &t, const char *name, const Ctx &c) {
    TORCH_CHECK(t.device() == c.dev, "wgrt.trace: ", name, " must be on ", c.dev, ", got ", t.device());
    TORCH_CHECK(t.is_contiguous(), "wgrt.trace: ", name, " must be contiguous");
}

const float *column(const Tensor &t, const char *name, const Ctx &c) {
    on_device(t, name, c);
    TORCH_CHECK(t.scalar_type() == at::kFloat, "wgrt.trace: ray column ", name, " must be float32");
    TORCH_CHECK(t.numel() == c.rays, "wgrt.trace: ray column ", name, " has ", t.numel(), " rays, x has ", c.rays);
    return static_cast<const float *>(t.const_data_ptr());
}

// uint32 buffers arrive as uint32 tensors or as int32 views of them
void *u32(const Tensor &t, const char *name, const Ctx &c, int64_t need) {
    on_device(t, name, c);
    TORCH_CHECK(t.scalar_type() == at::kInt || t.scalar_type() == at::kUInt32, "wgrt.trace: ", name,
                " must be uint32 (or an int32 view)");
    TORCH_CHECK(t.numel() >= need, "wgrt.trace: ", name, " holds ", t.numel(), " entries, needs ", need);
    return t.data_ptr();
}

int64_t trace(int64_t scene, const Tensor &x, const Tensor &y, const Tensor &m, const Tensor &n,
              const std::optional<Tensor> &lmd_num, const Tensor &te, const Tensor &tm, const Tensor &delta_phase,
              Tensor rng_states, Tensor matrix_EB, std::optional<Tensor> stats, std::optional<Tensor> per_ray_bounces,
              int64_t n_rays, int64_t gid_offset, int64_t stream, int64_t kernel, int64_t variant, int64_t workgroups,
              const std::optional<Tensor> &chunk_order, int64_t num_iter, const std::optional<Tensor> &gid_blocks,
              int64_t gid_block_rays, int64_t debug, double grid_sqrt_k) {
    const wgrt_scene *s = reinterpret_cast<const wgrt_scene *>(static_cast<uintptr_t>(scene));
    TORCH_CHECK(s != nullptr, "wgrt.trace: NULL scene");
    wgrt_scene_info info{};
    const wgrt_status st = wgrt_scene_get_info(s, &info);
    if (st != WGRT_OK) return st;
    const Ctx c{c10::Device(c10::DeviceType::CUDA, static_cast<c10::DeviceIndex>(info.device)), x.numel()};
    // the scene's device is current for the call (the library selects it too, include/wgrt.h) and the
    // caller's comes back on return
    const c10::DeviceGuard guard(c.dev);
    TORCH_CHECK(n_rays >= 0 && n_rays <= c.rays, "wgrt.trace: n_rays=", n_rays, " out of range for ", c.rays, " rays");
    TORCH_CHECK(kernel == 0 || kernel == 1, "wgrt.trace: kernel must be 0 (full colour) or 1 (single wavelength)");

    wgrt_rays r{};
    r.x = column(x, "x", c);
    r.y = column(y, "y", c);
    r.m = column(m, "m", c);
    r.n = column(n, "n", c);
    if (kernel == 0) {
        TORCH_CHECK(lmd_num.has_value(), "wgrt.trace: the full-colour kernel needs lmd_num");
        r.lmd_num = column(*lmd_num, "lmd_num", c);
    }
    r.te = column(te, "te", c);
    r.tm = column(tm, "tm", c);
    r.delta_phase = column(delta_phase, "delta_phase", c);

    uint32_t *rng = static_cast<uint32_t *>(u32(rng_states, "rng_states", c, c.rays));
    on_device(matrix_EB, "matrix_EB", c);
    TORCH_CHECK(matrix_EB.scalar_type() == at::kFloat, "wgrt.trace: matrix_EB must be float32");
    const int64_t eb_want = (int64_t)info.tiles * 80 * 120;   // [L,] NY, NX, 80, 120
    TORCH_CHECK(matrix_EB.numel() == eb_want, "wgrt.trace: matrix_EB holds ", matrix_EB.numel(),
                " floats, the scene's grid has ", eb_want);
    wgrt_trace_stats *stp = nullptr;
    if (stats) {
        on_device(*stats, "stats", c);
        TORCH_CHECK(stats->scalar_type() == at::kLong && stats->numel() * 8 == (int64_t)sizeof(wgrt_trace_stats),
                    "wgrt.trace: stats must be int64[", sizeof(wgrt_trace_stats) / 8, "]");
        stp = static_cast<wgrt_trace_stats *>(stats->data_ptr());
    }
    uint32_t *per = per_ray_bounces ? static_cast<uint32_t *>(u32(*per_ray_bounces, "per_ray_bounces", c, c.rays))
                                    : nullptr;

    wgrt_launch_opts o{};
    o.kernel = (int)kernel;
    o.variant = (int)variant;
    o.workgroups = (int)workgroups;
    if (chunk_order) {
        on_device(*chunk_order, "chunk_order", c);
        const int64_t chunks = (n_rays + 63) / 64;
        TORCH_CHECK(chunk_order->scalar_type() == at::kInt && chunk_order->numel() == chunks,
                    "wgrt.trace: chunk_order must be int32[", chunks, "]");
        o.chunk_order = static_cast<const int32_t *>(chunk_order->const_data_ptr());
        o.n_chunk_order = chunks;
    }
    o.num_iter = (int)num_iter;
    if (gid_blocks) {
        on_device(*gid_blocks, "gid_blocks", c);
        TORCH_CHECK(gid_block_rays >= 1, "wgrt.trace: gid_blocks needs gid_block_rays >= 1");
        const int64_t blocks = (n_rays + gid_block_rays - 1) / gid_block_rays;
        TORCH_CHECK(gid_blocks->scalar_type() == at::kLong && gid_blocks->numel() >= blocks,
                    "wgrt.trace: gid_blocks must be int64 with >= ", blocks, " entries");
        o.gid_blocks = static_cast<const int64_t *>(gid_blocks->const_data_ptr());
        o.gid_block_rays = gid_block_rays;
    }
    // test / profiling hooks: the address of a wgrt_debug_opts record the caller keeps alive (0: none)
    o.debug = reinterpret_cast<const wgrt_debug_opts *>(static_cast<uintptr_t>(debug));
    o.grid_sqrt_k = grid_sqrt_k;
    return wgrt_trace_opts(s, &r, n_rays, gid_offset, rng, matrix_EB.data_ptr<float>(), stp, per,
                           reinterpret_cast<void *>(static_cast<uintptr_t>(stream)), &o);
}

}  // namespace

TORCH_LIBRARY(wgrt, m) {
    m.def("trace(int scene, Tensor x, Tensor y, Tensor m, Tensor n, Tensor? lmd_num, Tensor te, Tensor tm, "
          "Tensor delta_phase, Tensor(a!) rng_states, Tensor(b!) matrix_EB, Tensor(c!)? stats, "
          "Tensor(d!)? per_ray_bounces, int n_rays, int gid_offset, int stream, int kernel, int variant, "
          "int workgroups, Tensor? chunk_order, int num_iter, Tensor? gid_blocks, int gid_block_rays, int debug, "
          "float grid_sqrt_k) -> int",
          &trace);
}
