"""IFile: the intermediate (map output / spill) record format and SpillRecord index.

Format (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/IFile.java:51, 119-128,
162-188; IFileOutputStream.java; SpillRecord.java:106):

    repeat: VInt keyLen, VInt valueLen, key bytes, value bytes
    EOF   : VInt -1, VInt -1
    then a 4-byte CRC32 of everything before it (IFileOutputStream checksum)

A map output file holds one IFile segment per reduce partition, back to back;
``<file>.index`` holds per partition (startOffset, rawLength, partLength) as
three big-endian longs, followed by an 8-byte CRC32 of the index entries.
"""
from __future__ import annotations

import collections
import io
import struct
import threading
import zlib

from .vint import decode_vint, encode_vint

EOF_MARKER = -1
_EOF = encode_vint(EOF_MARKER) * 2


class IFileWriter:
    """Writes one IFile segment into an open binary stream."""

    def __init__(self, out, codec=None):
        self.out = out
        self.codec = codec
        self.start = out.tell()
        self.buf = io.BytesIO()
        self.raw_length = 0
        self.records = 0

    def append(self, kb: bytes, vb: bytes):
        self.buf.write(encode_vint(len(kb)))
        self.buf.write(encode_vint(len(vb)))
        self.buf.write(kb)
        self.buf.write(vb)
        self.records += 1

    def close(self):
        """Finish the segment; returns (start, raw_length, part_length)."""
        self.buf.write(_EOF)
        data = self.buf.getvalue()
        self.raw_length = len(data) + 4
        if self.codec is not None:
            data = self.codec.compress(data)
        crc = zlib.crc32(data) & 0xFFFFFFFF
        self.out.write(data)
        self.out.write(struct.pack(">I", crc))
        part = len(data) + 4
        return self.start, self.raw_length, part


def read_segment(data: bytes, codec=None, verify=True):
    """Parse one IFile segment (as stored, incl. CRC). Returns list of (k, v)."""
    # (a segment that never left this process — hbmr.mapred.sortbuf.
    # VerifiedSegment, or a memoryview into the in-memory map output store —
    # carries no CRC to check)
    if data.__class__ is memoryview:
        data, verify = data.tobytes(), False
    body, crc = data[:-4], struct.unpack(">I", data[-4:])[0]
    if verify and not getattr(data, "verified", False) and \
            (zlib.crc32(body) & 0xFFFFFFFF) != crc:
        raise IOError("IFile checksum error")
    if codec is not None:
        body = codec.decompress(body)
    out = []
    pos = 0
    n = len(body)
    while pos < n:
        kl, pos = decode_vint(body, pos)
        vl, pos = decode_vint(body, pos)
        if kl == EOF_MARKER and vl == EOF_MARKER:
            break
        out.append((body[pos:pos + kl], body[pos + kl:pos + kl + vl]))
        pos += kl + vl
    return out


def iter_segment(data: bytes, codec=None, verify=True):
    yield from read_segment(data, codec, verify)


class SpillRecord:
    ENTRY = struct.Struct(">qqq")

    def __init__(self, partitions: int = 0):
        self.entries = [(0, 0, 0)] * partitions

    def put(self, part, start, raw, plen):
        self.entries[part] = (start, raw, plen)

    def get(self, part):
        return self.entries[part]

    def __len__(self):
        return len(self.entries)

    def to_bytes(self) -> bytes:
        body = b"".join(self.ENTRY.pack(*e) for e in self.entries)
        return body + struct.pack(">q", zlib.crc32(body) & 0xFFFFFFFF)

    def write(self, path):
        with open(path, "wb") as f:
            f.write(self.to_bytes())
        _remember(path, self)

    @classmethod
    def from_bytes(cls, data: bytes) -> "SpillRecord":
        body, crc = data[:-8], struct.unpack(">q", data[-8:])[0]
        if (zlib.crc32(body) & 0xFFFFFFFF) != crc:
            raise IOError("spill index checksum error")
        r = cls(0)
        r.entries = [cls.ENTRY.unpack_from(body, i) for i in range(0, len(body), cls.ENTRY.size)]
        return r

    @classmethod
    def read(cls, path) -> "SpillRecord":
        got = _INDEX_CACHE.get(path)
        if got is not None:
            return got
        with open(path, "rb") as f:
            return cls.from_bytes(f.read())


# The spill indexes this process wrote, by path: a reduce in the same process
# as its maps (a tracker's reduce of its own maps' outputs) finds them here
# instead of re-reading each map's .index file (map output paths are unique
# per attempt and never rewritten in place).  Bounded by partition entries.
_INDEX_CACHE: "collections.OrderedDict[str, SpillRecord]" = collections.OrderedDict()
_INDEX_CACHE_ENTRIES = [0]
_INDEX_CACHE_MAX = 1 << 18
_INDEX_LOCK = threading.Lock()


def _remember(path, rec):
    n = len(rec.entries)
    if n > _INDEX_CACHE_MAX // 64:
        return
    with _INDEX_LOCK:
        old = _INDEX_CACHE.pop(path, None)
        if old is not None:
            _INDEX_CACHE_ENTRIES[0] -= len(old.entries)
        _INDEX_CACHE[path] = rec
        _INDEX_CACHE_ENTRIES[0] += n
        while _INDEX_CACHE_ENTRIES[0] > _INDEX_CACHE_MAX:
            _p, r = _INDEX_CACHE.popitem(last=False)
            _INDEX_CACHE_ENTRIES[0] -= len(r.entries)


def read_partition(path, index: SpillRecord, part: int, codec=None):
    start, _raw, plen = index.get(part)
    with open(path, "rb") as f:
        f.seek(start)
        data = f.read(plen)
    return read_segment(data, codec)
