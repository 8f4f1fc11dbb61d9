"""Test-only stand-in for ``numba`` used by ``tests/golden/gen_golden.py``.

It lets the reference's kernel module be imported *unmodified* on a machine
without numba and executes ``@cuda.jit`` kernels sequentially, one global
thread index at a time -- the semantics of numba's CUDA simulator.  The only
shared writes in the traced kernel are commutative ``+= 1.0`` atomics and
per-ray RNG slots, so sequential execution equals the parallel kernel.
Never imported by the product package.
"""
import numpy as _np

from . import cuda  # noqa: F401

int32 = _np.int32
uint32 = _np.uint32
float32 = _np.float32
float64 = _np.float64
