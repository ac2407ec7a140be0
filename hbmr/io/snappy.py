"""Snappy through native/io/snappy.cc (libhbmr_cpu.so): raw Snappy blocks and
Hadoop's BlockCompressorStream framing of them (SnappyCodec.java:95-110,
BlockCompressorStream.java:76-153, BlockDecompressorStream.java:55-110).

``compress``/``decompress`` are the raw format; ``hadoop_compress`` /
``hadoop_decompress`` the framed bytes a Hadoop SnappyCodec stream holds
(what SequenceFile RECORD/BLOCK values and ``.snappy`` files carry)."""
from __future__ import annotations

import ctypes

from .nativeio import _PATH

BUFFER_SIZE_KEY = "io.compression.codec.snappy.buffersize"
BUFFER_SIZE_DEFAULT = 256 * 1024

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        L = ctypes.CDLL(_PATH)
        P, L64, I = ctypes.c_char_p, ctypes.c_long, ctypes.c_int
        for name, args in (("hbmr_snappy_max_compressed_length", [L64]),
                           ("hbmr_snappy_compress", [P, L64, ctypes.c_void_p, L64]),
                           ("hbmr_snappy_uncompressed_length", [P, L64]),
                           ("hbmr_snappy_decompress", [P, L64, ctypes.c_void_p, L64]),
                           ("hbmr_snappy_hadoop_max_length", [L64, I]),
                           ("hbmr_snappy_hadoop_compress", [P, L64, I, ctypes.c_void_p, L64]),
                           ("hbmr_snappy_hadoop_uncompressed_length", [P, L64]),
                           ("hbmr_snappy_hadoop_decompress", [P, L64, ctypes.c_void_p, L64])):
            f = getattr(L, name)
            f.argtypes, f.restype = args, L64
        _LIB = L
    return _LIB


def _run(fn, data, cap, *extra):
    data = bytes(data)
    out = ctypes.create_string_buffer(max(cap, 1))
    n = fn(data, len(data), *extra, out, cap)
    if n < 0:
        raise IOError("snappy: malformed or oversized input")
    return out.raw[:n]


def compress(data) -> bytes:
    L = _lib()
    data = bytes(data)
    return _run(L.hbmr_snappy_compress, data, L.hbmr_snappy_max_compressed_length(len(data)))


def decompress(data) -> bytes:
    L = _lib()
    data = bytes(data)
    n = L.hbmr_snappy_uncompressed_length(data, len(data))
    if n < 0:
        raise IOError("snappy: bad length preamble")
    return _run(L.hbmr_snappy_decompress, data, n)


def hadoop_compress(data, buffer_size: int = BUFFER_SIZE_DEFAULT) -> bytes:
    L = _lib()
    data = bytes(data)
    cap = L.hbmr_snappy_hadoop_max_length(len(data), buffer_size)
    if cap < 0:
        raise ValueError(f"snappy buffer size {buffer_size} too small")
    out = ctypes.create_string_buffer(cap)
    n = L.hbmr_snappy_hadoop_compress(data, len(data), buffer_size, out, cap)
    if n < 0:
        raise IOError("snappy: compress failed")
    return out.raw[:n]


def hadoop_decompress(data) -> bytes:
    L = _lib()
    data = bytes(data)
    n = L.hbmr_snappy_hadoop_uncompressed_length(data, len(data))
    if n < 0:
        raise IOError("snappy: truncated or malformed block stream")
    return _run(L.hbmr_snappy_hadoop_decompress, data, n)
