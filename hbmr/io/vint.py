"""Hadoop variable-length integer codec (WritableUtils.writeVLong / readVLong).

Bit-compatible with hadoop-1.0.3/src/core/org/apache/hadoop/io/WritableUtils.java
(writeVLong/readVLong/decodeVIntSize) and the C++ SerialUtils
(src/c++/utils/impl/SerialUtils.cc:178-231): values in [-112, 127] are one
byte; otherwise a length/sign marker byte followed by the big-endian magnitude
(one's complement for negatives).
"""
from __future__ import annotations

import struct


def encode_vlong(i: int) -> bytes:
    if -112 <= i <= 127:
        return struct.pack(">b", i)
    length = -112
    if i < 0:
        i = ~i
        length = -120
    tmp = i
    while tmp != 0:
        tmp >>= 8
        length -= 1
    out = bytearray(struct.pack(">b", length))
    n = -(length + 120) if length < -120 else -(length + 112)
    for idx in range(n, 0, -1):
        shift = (idx - 1) * 8
        out.append((i >> shift) & 0xFF)
    return bytes(out)


encode_vint = encode_vlong


def decode_vint_size(first: int) -> int:
    """Total encoded size (including the first byte) given the signed first byte."""
    if first >= -112:
        return 1
    if first < -120:
        return -119 - first
    return -111 - first


def is_negative_vint(first: int) -> bool:
    return first < -120 or (-112 <= first < 0)


def decode_vlong(buf, pos: int = 0):
    """Decode a VLong from ``buf`` at ``pos``; returns (value, new_pos)."""
    first = buf[pos]
    if first > 127:
        first -= 256
    size = decode_vint_size(first)
    if size == 1:
        return first, pos + 1
    i = 0
    for b in buf[pos + 1:pos + size]:
        i = (i << 8) | b
    if is_negative_vint(first):
        i = ~i
    return i, pos + size


decode_vint = decode_vlong


def read_vlong(stream) -> int:
    b = stream.read(1)
    if not b:
        raise EOFError("EOF reading VLong")
    first = b[0] - 256 if b[0] > 127 else b[0]
    size = decode_vint_size(first)
    if size == 1:
        return first
    rest = stream.read(size - 1)
    if len(rest) != size - 1:
        raise EOFError("EOF reading VLong body")
    i = 0
    for x in rest:
        i = (i << 8) | x
    return ~i if is_negative_vint(first) else i


read_vint = read_vlong


def vint_size(i: int) -> int:
    return len(encode_vlong(i))
