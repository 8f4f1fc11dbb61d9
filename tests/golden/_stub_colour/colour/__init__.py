"""Throwaway stand-in for colour-science (absent here), used ONLY by tests/golden/gen_golden.py to
run the reference's AR_system_evaluation_functions.evaluation unmodified.  Each entry point routes
to the package's restatement of the same third-party function, so the fixtures pin the reference's
own glue code (EVAL:45-163); the colour-science internals themselves stay unpinned."""
import numpy as np

from gpu_ray_tracing_for_waveguide_based_ar_display_amd.AR_system_evaluation_functions import (XYZ_D65_ASTM,
                                                                                               delta_e_ciede2000,
                                                                                               xyz_to_lab)

SDS_ILLUMINANTS = {"D65": "D65 spectral distribution (stand-in)"}


def sd_to_XYZ(sd):
    assert sd == SDS_ILLUMINANTS["D65"]
    return XYZ_D65_ASTM.copy()


def XYZ_to_Lab(XYZ):
    return xyz_to_lab(np.asarray(XYZ, dtype=np.float64))


def delta_E(a, b, method="CIE 2000"):
    assert method == "CIE 2000"
    return delta_e_ciede2000(a, b)
