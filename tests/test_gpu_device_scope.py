"""The C ABI's device discipline (include/wgrt.h, "Devices"): every entry point that takes a scene
runs on the scene's device and leaves the calling thread's current HIP device as it found it, so a
host driving scenes on several GPUs from one thread keeps its own selection.

The calls here are the ones that select a device (wgrt_scene_create_ex, the trace launch with its
scratch allocation, wgrt_scene_reserve, wgrt_rays_init, wgrt_scene_destroy); the current device is
read with hipGetDevice from the HIP runtime itself (not torch's cached view) before and after each.
One device suffices for what this checks: nothing leaves a different device current behind.  With
a second device the scene is also created on it while device 0 stays current.

Tolerance: exact (device ordinals; the trace's results are compared with the golden fixture)."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()
    # the HIP runtime this process already runs (torch's copy, which libwgrt.so binds too): loading
    # another libamdhip64 next to it would not see this process's device selection
    with open("/proc/self/maps") as f:
        paths = sorted({ln.split()[-1] for ln in f if "libamdhip64.so" in ln})
    assert paths, "no HIP runtime mapped"
    L = ctypes.CDLL(paths[0])
    L.hipGetDevice.argtypes = [ctypes.POINTER(ctypes.c_int)]
    L.hipSetDevice.argtypes = [ctypes.c_int]

    def current():
        d = ctypes.c_int(-1)
        assert L.hipGetDevice(ctypes.byref(d)) == 0
        return d.value

    def select(d):
        assert L.hipSetDevice(int(d)) == 0
    return current, select


def _trace_golden(scene_dev, hip):
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import (Scene, new_stats, rays_to_device, reserve,
                                                                           trace_fullcolor)
    from tests._fixtures import GoldenCase
    current, select = hip
    case = GoldenCase("c1_rgb")
    dev = torch.device("cuda", scene_dev)
    rays = rays_to_device(case.rays, dev)
    rng = torch.from_numpy(case.fresh_rng().view(np.int32)).to(dev)
    eb = torch.zeros(case.eb_shape(), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    select(0)
    scene = Scene.from_geometry(case.geom, case.luts, device=scene_dev)
    assert current() == 0, "wgrt_scene_create_ex left another device current"
    reserve(scene, case.N, 2)
    assert current() == 0, "wgrt_scene_reserve left another device current"
    st = new_stats(dev)
    with torch.cuda.device(scene_dev):
        stream = torch.cuda.current_stream(dev)
    select(0)
    trace_fullcolor(scene, rays, rng, eb, stats=st, stream=stream)
    assert current() == 0, "the trace launch left another device current"
    torch.cuda.synchronize(dev)
    select(0)
    scene.close()
    assert current() == 0, "wgrt_scene_destroy left another device current"
    return case, rng, eb


def test_entry_points_keep_the_current_device(hip):
    case, rng, eb = _trace_golden(0, hip)
    np.testing.assert_array_equal(rng.cpu().numpy().view(np.uint32), case.f["rng_after1"])
    np.testing.assert_array_equal(eb.cpu().numpy(), case.eb_expected(1))


def test_scene_on_second_device(hip):
    if torch.cuda.device_count() < 2:
        pytest.skip("one HIP device: the single-device test covers the restore")
    case, rng, eb = _trace_golden(1, hip)
    np.testing.assert_array_equal(rng.cpu().numpy().view(np.uint32), case.f["rng_after1"])
    np.testing.assert_array_equal(eb.cpu().numpy(), case.eb_expected(1))


def test_rays_init_keeps_the_current_device(hip):
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import init_rays
    current, select = hip
    dev = torch.device("cuda", 0)
    pts = torch.zeros((8, 2), dtype=torch.float64, device=dev)
    select(0)
    init_rays(pts, 2, 2, [0, 1, 2], 16, device=dev)
    assert current() == 0
    torch.cuda.synchronize()
