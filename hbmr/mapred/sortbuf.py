"""Native map-output sort path (CPU tasks).

Batch partition / sort / group / IFile encode of serialised records in C++
(native/cpu/mapout.cc, ``hbmr/lib/libhbmr_cpu.so``), used by
:class:`hbmr.mapred.task.MapOutputBuffer` and ReduceTask when the job's map
output key is a Writable with a known raw comparator (Text, BytesWritable,
IntWritable, LongWritable) and no custom sort/grouping comparator is set —
the reference's MapOutputBuffer quick-sort over raw bytes
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/MapTask.java:1119-1130,
1396-1465) and Merger (Merger.java:236-365), done on whole spills.  Other jobs
keep the generic Python path (``hbmr.map.sort.native=false`` forces it).
"""
from __future__ import annotations

import ctypes
import logging
import os
import zlib
import struct

import numpy as np

log = logging.getLogger("hbmr.sortbuf")

_LIB = None
_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                         "libhbmr_cpu.so")
_P = ctypes.c_void_p
_I64 = ctypes.c_int64

TEXT, BYTES, INT, LONG = 0, 1, 2, 3


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_LIB_PATH):
            _LIB = False
            log.warning("%s missing (run native/build.py): map-output sort stays in Python",
                        _LIB_PATH)
            return None
        L = ctypes.CDLL(_LIB_PATH)
        L.hbmr_hash_partition.argtypes = [ctypes.c_int, _P, _P, _P, _I64, ctypes.c_int, _P]
        L.hbmr_sort_records.argtypes = [ctypes.c_int, _P, _P, _P, _I64, _P, _P]
        L.hbmr_group_runs.argtypes = [ctypes.c_int, _P, _P, _P, _P, _I64, _I64, _P]
        L.hbmr_group_runs.restype = _I64
        L.hbmr_ifile_encode.argtypes = [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P]
        L.hbmr_ifile_encode.restype = _I64
        L.hbmr_ifile_decode.argtypes = [_P, _I64, _I64, _P, _P, _P, _P]
        L.hbmr_ifile_decode.restype = _I64
        _LIB = L
    return _LIB or None


def key_kind(job):
    """Native comparator kind for this job's map output key, else None."""
    if not job.get_boolean("hbmr.map.sort.native", True):
        return None
    if job.get("mapred.output.key.comparator.class") or \
            job.get("mapred.output.value.groupfn.class"):
        return None
    from ..io.writable import BytesWritable, IntWritable, LongWritable, Text
    kinds = {Text: TEXT, BytesWritable: BYTES, IntWritable: INT, LongWritable: LONG}
    k = kinds.get(job.get_map_output_key_class())
    if k is None or lib() is None:
        return None
    return k


def hash_partitioned(job) -> bool:
    from .lib.basic import HashPartitioner
    return job.get_partitioner_class() is HashPartitioner


def _addr(a):
    return a.ctypes.data


class Batch:
    """Records as (pos, len) slices of two byte buffers."""

    __slots__ = ("kbuf", "kpos", "klen", "vbuf", "vpos", "vlen", "_karr", "_varr")

    def __init__(self, kbuf, kpos, klen, vbuf, vpos, vlen):
        self.kbuf, self.kpos, self.klen = kbuf, kpos, klen
        self.vbuf, self.vpos, self.vlen = vbuf, vpos, vlen
        self._karr = np.frombuffer(kbuf, dtype=np.uint8) if len(kbuf) else np.zeros(1, np.uint8)
        self._varr = np.frombuffer(vbuf, dtype=np.uint8) if len(vbuf) else np.zeros(1, np.uint8)

    @property
    def n(self):
        return len(self.kpos)

    @classmethod
    def from_lists(cls, keys: list, vals: list) -> "Batch":
        kl = np.fromiter(map(len, keys), dtype=np.int64, count=len(keys))
        vl = np.fromiter(map(len, vals), dtype=np.int64, count=len(vals))
        kp = np.zeros(len(keys), np.int64)
        vp = np.zeros(len(vals), np.int64)
        if len(keys) > 1:
            np.cumsum(kl[:-1], out=kp[1:])
            np.cumsum(vl[:-1], out=vp[1:])
        return cls(b"".join(keys), kp, kl, b"".join(vals), vp, vl)

    @classmethod
    def from_ifile_bodies(cls, bodies: list) -> "Batch":
        """Records of several (decompressed, CRC-stripped) IFile bodies, in order."""
        buf = b"".join(bodies)
        L = lib()
        kpos, klen, vpos, vlen = [], [], [], []
        base = 0
        arr = np.frombuffer(buf, dtype=np.uint8) if buf else np.zeros(1, np.uint8)
        for body in bodies:
            cap = max(1, len(body) // 2)
            kp = np.empty(cap, np.int64)
            kl = np.empty(cap, np.int64)
            vp = np.empty(cap, np.int64)
            vl = np.empty(cap, np.int64)
            nr = L.hbmr_ifile_decode(_addr(arr) + base, len(body), cap, _addr(kp), _addr(kl),
                                     _addr(vp), _addr(vl))
            if nr < 0:
                raise IOError("malformed IFile segment")
            kpos.append(kp[:nr] + base)
            klen.append(kl[:nr])
            vpos.append(vp[:nr] + base)
            vlen.append(vl[:nr])
            base += len(body)
        cat = (lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.int64))
        kp, vp = cat(kpos), cat(vpos)
        return cls(buf, kp, cat(klen), buf, vp, cat(vlen))

    @classmethod
    def for_reduce(cls, bodies: list) -> "Batch":
        """from_ifile_bodies for a reduce's sort and feed only (no re-encode):
        a partition of few large records — a Pipes K-Means block per map,
        ~1 MB each, 128 of them at config 3 — keeps its values where they
        are (views into the segments) and joins only the keys, instead of
        copying every value into one buffer first (134 MB, ~25 ms on the box
        before the feed could start).  Anything else: from_ifile_bodies."""
        total = sum(len(b) for b in bodies)
        if len(bodies) < 2 or total < (8 << 20):
            return cls.from_ifile_bodies(bodies)
        L = lib()
        segs = []
        n = 0
        for body in bodies:
            arr = np.frombuffer(body, dtype=np.uint8) if len(body) else np.zeros(1, np.uint8)
            cap = max(1, len(body) // 2)
            kp = np.empty(cap, np.int64)
            kl = np.empty(cap, np.int64)
            vp = np.empty(cap, np.int64)
            vl = np.empty(cap, np.int64)
            nr = L.hbmr_ifile_decode(_addr(arr), len(body), cap, _addr(kp), _addr(kl),
                                     _addr(vp), _addr(vl))
            if nr < 0:
                raise IOError("malformed IFile segment")
            n += nr
            if n > 65536 or (nr and total // max(1, n) < 4096):
                return cls.from_ifile_bodies(bodies)     # many small records
            segs.append((body, kp[:nr], kl[:nr], vp[:nr], vl[:nr]))
        keys, views = [], []
        for body, kp, kl, vp, vl in segs:
            mv = memoryview(body)
            for i in range(len(kp)):
                keys.append(bytes(mv[int(kp[i]):int(kp[i]) + int(kl[i])]))
                views.append(mv[int(vp[i]):int(vp[i]) + int(vl[i])])
        return _ViewBatch.build(keys, views)

    # -- kernels -------------------------------------------------------------------------
    def hash_partition(self, kind, R) -> np.ndarray:
        part = np.empty(self.n, np.int32)
        if self.n:
            lib().hbmr_hash_partition(kind, _addr(self._karr), _addr(self.kpos),
                                      _addr(self.klen), self.n, R, _addr(part))
        return part

    def sort(self, kind, part) -> np.ndarray:
        perm = np.empty(self.n, np.int64)
        if self.n:
            part = np.ascontiguousarray(part, dtype=np.int32)
            lib().hbmr_sort_records(kind, _addr(self._karr), _addr(self.kpos), _addr(self.klen),
                                    self.n, _addr(part), _addr(perm))
        return perm

    def group_ends(self, kind, perm, lo, hi) -> np.ndarray:
        if hi <= lo:
            return np.zeros(0, np.int64)
        ends = np.empty(hi - lo, np.int64)
        nr = lib().hbmr_group_runs(kind, _addr(self._karr), _addr(self.kpos), _addr(self.klen),
                                   _addr(perm), lo, hi, _addr(ends))
        return ends[:nr]

    def ifile_body(self, perm, lo, hi, view=False):
        """IFile segment body (records + EOF marker, no CRC) of perm[lo:hi]
        (``view``: a memoryview of the encode buffer, not a bytes copy)."""
        sel = perm[lo:hi]
        bound = int(self.klen[sel].sum() + self.vlen[sel].sum()) + 10 * (hi - lo) + 4
        out = np.empty(bound, np.uint8)
        n = lib().hbmr_ifile_encode(_addr(self._karr), _addr(self.kpos), _addr(self.klen),
                                    _addr(self._varr), _addr(self.vpos), _addr(self.vlen),
                                    _addr(perm), lo, hi, _addr(out))
        return memoryview(out)[:n] if view else out[:n].tobytes()

    def key(self, r) -> bytes:
        p = int(self.kpos[r])
        return self.kbuf[p:p + int(self.klen[r])]

    def value(self, r) -> bytes:
        p = int(self.vpos[r])
        return self.vbuf[p:p + int(self.vlen[r])]

    def value_view(self, r) -> memoryview:
        """value() without the copy (a view into the batch's buffer)."""
        p = int(self.vpos[r])
        return memoryview(self.vbuf)[p:p + int(self.vlen[r])]



class _ViewBatch(Batch):
    """Batch.for_reduce's form: keys in one buffer (sort, grouping), each
    value a view into the map output segment it arrived in."""

    __slots__ = ("views",)

    @classmethod
    def build(cls, keys: list, views: list) -> "_ViewBatch":
        kl = np.fromiter(map(len, keys), dtype=np.int64, count=len(keys))
        kp = np.zeros(len(keys), np.int64)
        if len(keys) > 1:
            np.cumsum(kl[:-1], out=kp[1:])
        vl = np.fromiter(map(len, views), dtype=np.int64, count=len(views))
        b = cls(b"".join(keys), kp, kl, b"", np.zeros(len(views), np.int64), vl)
        b.views = views
        return b

    def value(self, r) -> bytes:
        return bytes(self.views[r])

    def value_view(self, r) -> memoryview:
        return self.views[r]

    def ifile_body(self, perm, lo, hi, view=False):
        raise NotImplementedError("a reduce-side view batch is not re-encoded")


def write_segment(f, body: bytes, codec=None, crc=True):
    """Append one IFile segment (body [+codec] + CRC32) to f; returns
    (start, raw_length, part_length) for the SpillRecord.  ``crc`` False
    leaves the CRC word zero (an in-memory map output, read only as a
    VerifiedSegment; fill_crcs completes it if it goes to a file after all)."""
    start = f.tell()
    raw_len = len(body) + 4
    if codec is not None:
        body = codec.compress(body)
    f.write(body)
    f.write(struct.pack(">I", zlib.crc32(body) & 0xFFFFFFFF) if crc else b"\0\0\0\0")
    return start, raw_len, len(body) + 4


def fill_crcs(data: bytes, rec) -> bytes:
    """``data`` (a spill's segments written with crc=False) with every
    partition segment's CRC32 computed, per its SpillRecord ``rec``."""
    out = bytearray(data)
    mv = memoryview(out)
    for p in range(len(rec)):
        start, _raw, plen = rec.get(p)
        if plen >= 4:
            c = zlib.crc32(mv[start:start + plen - 4]) & 0xFFFFFFFF
            out[start + plen - 4:start + plen] = struct.pack(">I", c)
    return bytes(out)


class VerifiedSegment(bytes):
    """A map-output segment that never left this process (an in-memory map
    output, hbmr/mapred/mapoutput.py): no disk or wire between its writer and
    here, so the reduce skips the check (zlib's CRC runs ~1 GB/s: a 1 MB
    K-Means partials block per map made it most of the copy phase) — and its
    writer skips computing one (write_segment crc=False: the CRC word is 0)."""
    __slots__ = ()
    verified = True


def in_process(data) -> bool:
    """A segment that never left this process: a VerifiedSegment, or a
    memoryview into the in-memory map output store (MapOutputLocation.
    read_partition: no copy; every fetch from a file or the wire is bytes)."""
    return data.__class__ is VerifiedSegment or data.__class__ is memoryview


def segment_body(data: bytes, codec=None, verify=True) -> bytes:
    """Stored IFile segment (incl. CRC) → decompressed body."""
    body, crc = memoryview(data)[:-4], struct.unpack(">I", data[-4:])[0]
    if verify and not in_process(data) and \
            (zlib.crc32(body) & 0xFFFFFFFF) != crc:
        raise IOError("IFile checksum error")
    return codec.decompress(bytes(body)) if codec is not None else body
