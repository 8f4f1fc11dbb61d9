// wgrt_scene.h -- the device-resident scene behind the opaque wgrt_scene handle (include/wgrt.h),
// shared by the C-ABI translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>

#include "wgrt_device.h"

struct wgrt_scene {
    int device = 0;
    int nx = 0, ny = 0, nl = 0, nfc = 0, noc = 0, tile_d = 0, npoly = 0;
    double n_g = 0;
    double *d_tiles = nullptr;
    double *d_jtiles = nullptr;
    int jtile_d = 0;
    uint64_t *d_cells = nullptr;
    uint32_t *d_cells32 = nullptr;   // 32-bit copy of the cell words (npoly <= 16), else NULL
    double *d_verts = nullptr;
    int32_t *d_poly_off = nullptr;
    int32_t *d_row_off = nullptr;
    int32_t *d_row_edges = nullptr;
    double *d_bands = nullptr;
    wgrt::LocatorHost loc_host;  // grid parameters (cells / verts vectors released after upload)
    int64_t tiles = 0;
    int64_t edge_cells = 0;        // locator cells with an EDGE class
    int jones_grid[2][2][2] = {};   // resident 256-thread workgroups: [64-bit cells][fused][single wavelength]
    int jones_tl_grid[2] = {};      // ... of the debug timeline instantiations (32-bit cells): [fused]
    int64_t nonunitary_blocks = 0;  // Jones blocks whose branch matrices are not scaled-unitary (their launches
                                    // run the AMP instantiations: wgrt_device.h, the amplification step)
    // Jones-vector launches: per-stream launch scratch (launches on one stream are ordered, so
    // they may share it; launches on different streams never do)
    struct Scratch {
        // two counter sets (kHeads chunk heads kHeadStride apart, replay count, queue count,
        // full-block count), used by alternate launches: a launch's epilogue zeroes the other one
        unsigned long long *ctr = nullptr;
        uint32_t parity = 0;                 // the set the next launch uses
        bool dirty = false;                  // a launch failed half-way: both sets need zeroing
        uint32_t *full = nullptr;            // full-block list (qcap / kQBlock entries)
        uint32_t *list = nullptr;            // replay list
        int64_t cap = 0;                     // replay list entries
        double2 *q_xy = nullptr;             // out-coupling queue: position, ray index
        uint32_t *q_i = nullptr;
        int64_t qcap = 0;
        unsigned long long *part = nullptr;  // per-wave counter partials (kPartWords words per slot)
        int64_t part_slots = 0;
        uint64_t *rng64 = nullptr;           // fused launches: per-ray {state, tag} granules
        uint32_t iter_epoch = 0;             // < 2^23 (iter_tag)
        int64_t cap64 = 0;
    };
    std::mutex scratch_mu;
    std::map<void *, Scratch> scratch;
};

namespace wgrt {

// Record the detail of a failing entry point for wgrt_last_error() and return its status.
wgrt_status fail(wgrt_status s, const std::string &msg);

// The C ABI's device discipline: an entry point that works on a scene (or allocates, or launches on
// a stream) makes the scene's device current for its own scope and gives the caller's current
// device back when it returns, so a host that drives several GPUs from one thread keeps whatever
// device it had selected.  hipSetDevice only when the device differs (a thread-local switch).
class DeviceScope {
    int prev_ = -1;
    hipError_t err_ = hipSuccess;

public:
    explicit DeviceScope(int device) {
        err_ = hipGetDevice(&prev_);
        if (err_ != hipSuccess) prev_ = -1;
        else if (prev_ != device) err_ = hipSetDevice(device);
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev_ >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev_) (void)hipSetDevice(prev_);
    }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
    hipError_t error() const { return err_; }
};

// The device a stream belongs to (the current device for the null stream).
inline hipError_t stream_device(void *stream, int *device) {
    if (!stream) return hipGetDevice(device);
    return hipStreamGetDevice((hipStream_t)stream, device);
}

inline Locator make_locator(const wgrt_scene *s) {
    Locator L;
    L.cells = s->d_cells;
    L.verts = s->d_verts;
    L.poly_off = s->d_poly_off;
    L.row_off = s->d_row_off;
    L.row_edges = s->d_row_edges;
    L.bands = s->d_bands;
    L.x0 = s->loc_host.x0;
    L.y0 = s->loc_host.y0;
    L.inv_h = s->loc_host.inv_h;
    L.ncx = s->loc_host.ncx;
    L.ncy = s->loc_host.ncy;
    return L;
}

inline LocatorT<uint32_t> make_locator32(const wgrt_scene *s) {
    const Locator g = make_locator(s);
    LocatorT<uint32_t> L;
    L.cells = s->d_cells32;
    L.verts = g.verts;
    L.poly_off = g.poly_off;
    L.row_off = g.row_off;
    L.row_edges = g.row_edges;
    L.bands = g.bands;
    L.x0 = g.x0, L.y0 = g.y0, L.inv_h = g.inv_h, L.ncx = g.ncx, L.ncy = g.ncy;
    return L;
}

}  // namespace wgrt
