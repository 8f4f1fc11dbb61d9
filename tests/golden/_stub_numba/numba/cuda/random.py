"""Placeholder: the traced kernel never calls numba's xoroshiro generator."""


def xoroshiro128p_uniform_float32(states, index):
    raise NotImplementedError("not used by process_rays_kernel_pro_fullColor")
