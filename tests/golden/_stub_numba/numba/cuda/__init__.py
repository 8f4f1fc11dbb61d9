"""Sequential CUDA-simulator semantics for the golden-vector harness (test-only)."""
import numpy as _np


class _State:
    gid = 0
    hook = None          # optional callable(gid) run before every thread


_state = _State()


def grid(ndim):
    return _state.gid


class _Kernel:
    def __init__(self, fn):
        self.fn = fn

    def __getitem__(self, cfg):
        blocks, tpb = cfg

        def launch(*args):
            for gid in range(int(blocks) * int(tpb)):
                _state.gid = gid
                if _state.hook is not None:
                    _state.hook(gid)
                self.fn(*args)
        return launch


def jit(fn=None, device=False, **kwargs):
    if fn is None:
        return (lambda f: f) if device else _Kernel
    return fn if device else _Kernel(fn)


class atomic:
    @staticmethod
    def add(arr, idx, value):
        """Compiled-numba addressing: negative indices wrap once, then the flat
        C-order offset is taken WITHOUT per-axis bounds checks (an index equal to
        an axis length aliases into the next row), guarded to the base buffer."""
        base = arr
        while base.base is not None and isinstance(base.base, _np.ndarray):
            base = base.base
        item = arr.itemsize
        start = (arr.__array_interface__["data"][0] - base.__array_interface__["data"][0]) // item
        off = start
        for k, (i, dim, st) in enumerate(zip(idx, arr.shape, arr.strides)):
            i = int(i)
            if i < 0:
                i += dim
            off += i * (st // item)
        if 0 <= off < base.size:
            base.reshape(-1)[off] += value
        return 0


def to_device(a, *args, **kwargs):
    return a


def synchronize():
    return None
