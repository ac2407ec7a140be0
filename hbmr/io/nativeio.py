"""Native SequenceFile I/O for dense float vectors (native/io/seqpoints.cc in
``hbmr/lib/libhbmr_cpu.so``): write K-Means inputs, count and decode a
FileSplit's points straight into a (pinned) host buffer — the file→HBM path
(SURVEY.md §2.6 NativeIO row) without per-record Python.

Reference: SequenceFile.Reader / Writer (hadoop-1.0.3/src/core/org/apache/
hadoop/io/SequenceFile.java:828, 1411) for the format; NativeIO.c for the
"native I/O next to the Java code" idea.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                     "libhbmr_cpu.so")
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_PATH):
            raise RuntimeError(f"{_PATH} missing: run native/build.py")
        L = ctypes.CDLL(_PATH)
        P, L64, I = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
        L.hbmr_seq_write_points.argtypes = [ctypes.c_char_p, P, L64, I, L64]
        L.hbmr_seq_write_points.restype = I
        L.hbmr_seq_count_points.argtypes = [ctypes.c_char_p, L64, L64]
        L.hbmr_seq_count_points.restype = L64
        L.hbmr_seq_read_points.argtypes = [ctypes.c_char_p, L64, L64, I, P, L64]
        L.hbmr_seq_read_points.restype = L64
        L.hbmr_seq_last_error.restype = ctypes.c_char_p
        _LIB = L
    return _LIB


def _err():
    return lib().hbmr_seq_last_error().decode(errors="replace")


def write_points(path, points: np.ndarray, first_id: int = 0):
    x = np.ascontiguousarray(points, dtype=np.float32)
    n, d = x.shape
    if lib().hbmr_seq_write_points(str(path).encode(), x.ctypes.data, n, d, first_id):
        raise IOError(f"writing {path}: {_err()}")


def count_points(path, start, length) -> int:
    n = lib().hbmr_seq_count_points(str(path).encode(), start, length)
    if n < 0:
        raise IOError(f"reading {path}: {_err()}")
    return int(n)


def read_points_into(path, start, length, out: np.ndarray | int, d: int, cap: int) -> int:
    """Decode the split's points into ``out`` ([cap, d] fp32 array, or a raw
    address of such a buffer); returns the number read."""
    addr = out if isinstance(out, int) else out.ctypes.data
    n = lib().hbmr_seq_read_points(str(path).encode(), start, length, d, addr, cap)
    if n < 0:
        raise IOError(f"reading {path}: {_err()}")
    return int(n)


def read_points(path, start, length, d) -> np.ndarray:
    n = count_points(path, start, length)
    out = np.empty((n, d), dtype=np.float32)
    got = read_points_into(path, start, length, out, d, n)
    return out[:got]
