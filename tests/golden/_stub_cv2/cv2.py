"""Throwaway stand-in for OpenCV (absent here), used ONLY by tests/golden/gen_golden.py to run the
reference's AR_system_evaluation_functions unmodified: cvtColor (float RGB <-> HSV), split and
merge, routed to the package's restatement of OpenCV's float HSV conversion."""
import numpy as np

from gpu_ray_tracing_for_waveguide_based_ar_display_amd.AR_system_evaluation_functions import (hsv_to_rgb_f32,
                                                                                               rgb_to_hsv_f32)

COLOR_RGB2HSV = 67
COLOR_HSV2RGB = 71


def cvtColor(img, code):
    assert img.dtype == np.float32 and img.ndim == 3 and img.shape[-1] == 3
    if code == COLOR_RGB2HSV:
        return rgb_to_hsv_f32(img)
    if code == COLOR_HSV2RGB:
        return hsv_to_rgb_f32(img)
    raise ValueError(code)


def split(img):
    return tuple(np.ascontiguousarray(img[..., k]) for k in range(img.shape[-1]))


def merge(channels):
    return np.stack(list(channels), axis=-1)
