"""Drop-in for the reference module ``GPU_ray_tracing_functions.py`` (hot-path subset).

Keeps the call shape the reference's driver uses
(``gpu_ray_tracing_pro_fullColor.py:170-177``)::

    process_rays_kernel_pro_fullColor[blocks_per_grid, threads_per_block](
        x_v, y_v, gap_x_v, gap_y_v, pol_v, azi_v, m_v, n_v, lmd_num, te_v, tm_v, delta_phase_v,
        rng_states, IC, FC, FC_offset, OC, OC_offset, n_g,
        eff_reg1, eff_reg2, eff_reg_FOV, eff_reg_FOV_range,
        lut_ic1, lut_ic2, lut_ic3, lut_fc1, lut_fc2, lut_oc1, lut_oc2, lut_TIR, lut_gap, matrix_EB)

its single-wavelength sibling (GRTF:419-831, no ``lmd_num``, 32 arguments, LUTs without
the wavelength axis, matrix_EB [NY, NX, 80, 120])::

    process_rays_kernel_pro[blocks_per_grid, threads_per_block](
        x_v, y_v, gap_x_v, gap_y_v, pol_v, azi_v, m_v, n_v, te_v, tm_v, delta_phase_v,
        rng_states, IC, ..., lut_TIR, lut_gap, matrix_EB)

and the host sampler ``generate_points_in_polygon`` (GRTF:12-23).  The launch runs
the HIP kernel of ``libwgrt.so``; there is no CPU path.

Argument handling mirrors a numba kernel call: torch ROCm tensors are used in place
(the launch is asynchronous on torch's current stream), numpy arrays are copied to
the device and the two arrays the kernel writes (``rng_states``, ``matrix_EB``) are
copied back into them after the launch.  The 19 scene arguments are packed once into
a device-resident ``Scene`` and cached by the identity of the argument objects (call
``clear_scene_cache()`` after mutating a LUT in place).  As in the reference, only the
first ``blocks * threads`` rays are traced when the grid is smaller than the batch.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import RAY_COLUMNS, Scene, trace_fullcolor, trace_single
from .rays import generate_points_in_polygon  # noqa: F401  (GRTF:12-23)

_SCENE_CACHE: dict = {}
_SCENE_CACHE_MAX = 4


def clear_scene_cache():
    for entry in _SCENE_CACHE.values():
        entry[1].close()
    _SCENE_CACHE.clear()


def _host(a):
    if isinstance(a, torch.Tensor):
        return a.detach().cpu().numpy()
    return np.asarray(a)


def _scene_for(args, device_index: int) -> Scene:
    key = (device_index,) + tuple(id(a) for a in args)
    hit = _SCENE_CACHE.get(key)
    if hit is not None:
        return hit[1]
    (IC, FC, FC_offset, OC, OC_offset, n_g, eff_reg1, eff_reg2, eff_reg_FOV, eff_reg_FOV_range,
     lut_ic1, lut_ic2, lut_ic3, lut_fc1, lut_fc2, lut_oc1, lut_oc2, lut_TIR, lut_gap) = args
    scene = Scene(*(_host(a) for a in (IC, FC, FC_offset, OC, OC_offset)), float(n_g),
                  *(_host(a) for a in (eff_reg1, eff_reg2, eff_reg_FOV, eff_reg_FOV_range, lut_ic1, lut_ic2,
                                       lut_ic3, lut_fc1, lut_fc2, lut_oc1, lut_oc2, lut_TIR, lut_gap)),
                  device=device_index)
    if len(_SCENE_CACHE) >= _SCENE_CACHE_MAX:
        old = next(iter(_SCENE_CACHE))
        _SCENE_CACHE.pop(old)[1].close()
    _SCENE_CACHE[key] = (args, scene)   # holding args keeps their ids valid
    return scene


class _Kernel:
    """A bounce kernel with numba launch syntax: ``process_rays_kernel_pro_fullColor``
    (GRTF:833-1246, 33 arguments) or ``process_rays_kernel_pro`` (GRTF:419-831, 32)."""

    def __init__(self, single: bool):
        self.single = single
        self.name = "process_rays_kernel_pro" if single else "process_rays_kernel_pro_fullColor"
        self.columns = tuple(c for c in RAY_COLUMNS if not (single and c == "lmd_num"))
        self.nargs = len(self.columns) + 21

    def __getitem__(self, cfg):
        if not (isinstance(cfg, tuple) and len(cfg) == 2):
            raise TypeError("launch configuration must be [blocks_per_grid, threads_per_block]")
        blocks, tpb = int(cfg[0]), int(cfg[1])
        if blocks < 0 or tpb <= 0:
            raise ValueError("blocks_per_grid must be >= 0 and threads_per_block > 0")
        return lambda *args: self._launch(blocks * tpb, *args)

    def _launch(self, n_threads, *args):
        if len(args) != self.nargs:
            raise TypeError(f"{self.name} takes {self.nargs} arguments, got {len(args)}")
        nc = len(self.columns)
        ray_args, rng_states, scene_args, matrix_EB = args[:nc], args[nc], args[nc + 1:nc + 20], args[nc + 20]
        if (np.ndim(scene_args[17]) == 3) != self.single:   # lut_TIR: [NX, NY, 4] single / [L, NX, NY, 4]
            raise ValueError(f"{self.name}: LUT shapes are for the "
                             f"{'full-colour' if self.single else 'single-wavelength'} kernel")
        dev = torch.device("cuda", torch.cuda.current_device())
        scene = _scene_for(scene_args, dev.index)

        def to_dev(a, dtype, name):
            if isinstance(a, torch.Tensor):
                return a
            arr = np.ascontiguousarray(np.asarray(a), dtype=dtype)
            return torch.from_numpy(arr).to(dev)

        rays = {k: to_dev(a, np.float32, k) for k, a in zip(self.columns, ray_args)}
        host_rng = None if isinstance(rng_states, torch.Tensor) else rng_states
        host_eb = None if isinstance(matrix_EB, torch.Tensor) else matrix_EB
        if host_rng is not None:
            if np.asarray(host_rng).dtype != np.uint32:
                raise TypeError("rng_states must be uint32")
            rng_t = torch.from_numpy(np.ascontiguousarray(host_rng).view(np.int32)).to(dev)
        else:
            rng_t = rng_states
        if host_eb is not None:
            if np.asarray(host_eb).dtype != np.float32:
                raise TypeError("matrix_EB must be float32")
            eb_t = torch.from_numpy(np.ascontiguousarray(host_eb)).to(dev)
        else:
            eb_t = matrix_EB
        n = min(rays["x"].numel(), n_threads)
        (trace_single if self.single else trace_fullcolor)(scene, rays, rng_t, eb_t, gid_offset=0, n_rays=n)
        if host_rng is not None:
            host_rng[...] = rng_t.cpu().numpy().view(np.uint32).reshape(np.shape(host_rng))
        if host_eb is not None:
            host_eb[...] = eb_t.cpu().numpy().reshape(np.shape(host_eb))


process_rays_kernel_pro_fullColor = _Kernel(single=False)
process_rays_kernel_pro = _Kernel(single=True)

__all__ = ["process_rays_kernel_pro_fullColor", "process_rays_kernel_pro", "generate_points_in_polygon",
           "clear_scene_cache"]
