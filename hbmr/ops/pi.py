"""PiEstimator map on the GPU (native/kernels/pi.hip) and its CPU twin."""
from __future__ import annotations

import numpy as np

from . import _lib


def count_inside_gpu(offset: int, n: int, out=None, stream=None):
    """Launch the Halton count on the current (or given) stream; returns a device
    int64 tensor of shape [1] (accumulated into ``out`` when given)."""
    import torch
    lib = _lib.load()
    if out is None:
        out = torch.zeros(1, dtype=torch.int64, device="cuda")
    if n < 0 or offset < 0 or offset + n >= 1 << 62:
        raise ValueError("bad Halton range")
    _lib.check(lib.hbmr_pi_halton(offset, n, out.data_ptr(), _lib.stream_handle(stream)),
               "hbmr_pi_halton")
    return out


def count_inside_cpu(offset: int, n: int, chunk: int = 1 << 20) -> int:
    from ..examples.pi import halton
    inside = 0
    for a in range(0, n, chunk):
        idx = np.arange(offset + a, offset + min(n, a + chunk), dtype=np.int64)
        x = halton(idx, 2) - 0.5
        y = halton(idx, 3) - 0.5
        inside += int(np.count_nonzero(x * x + y * y <= 0.25))
    return inside
