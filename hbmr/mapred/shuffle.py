"""Reduce-side shuffle buffer with bounded memory: in-memory segments, direct
to-disk segments, background-style merges into sorted on-disk runs and a
final streaming k-way merge.

The reference's ReduceTask.ReduceCopier (hadoop-1.0.3/src/mapred/org/apache/
hadoop/mapred/ReduceTask.java): a fetched map output goes to memory when it is
at most 25% of the shuffle buffer (shuffleInMemory, :1646) and to a local
file otherwise (shuffleToDisk, :1775); the InMemFSMergeThread (:2692) merges
the in-memory segments into one on-disk run when the buffer passes
``mapred.job.shuffle.merge.percent`` or holds ``mapred.inmem.merge.threshold``
segments; the LocalFSMerger (:2585) merges ``io.sort.factor`` on-disk runs
into one when there are 2*factor-1 of them; createKVIterator (:2421) merges
what is left, in passes of at most ``io.sort.factor`` runs.

Order guarantee (what makes disk merges output-identical to the all-in-memory
path): runs are kept in arrival (map) order, every merge combines *adjacent*
runs and is stable, and the final merge breaks key ties by run order — so the
values of a key reach the reducer in exactly the order of the in-memory stable
sort of the concatenated map outputs.

Memory: ``hbmr.reduce.shuffle.memory.mb`` (default 256, the reduce heap the
reference sized with -Xmx) × ``mapred.job.shuffle.input.buffer.percent``
(0.70).  Disk runs are uncompressed IFile bodies + CRC32 in the attempt's
work directory.
"""
from __future__ import annotations

import heapq
import os
import struct
import zlib

import numpy as np

from ..io.ifile import EOF_MARKER, read_segment
from . import counters as C
from . import sortbuf

SHUFFLE_GROUP = "hbmr.ShuffleCounters"
_MAX_SINGLE = 0.25          # ReduceCopier.MAX_SINGLE_SHUFFLE_SEGMENT_FRACTION


def _read_vint(f):
    """Hadoop VInt from a buffered binary stream (WritableUtils.readVInt)."""
    b = f.read(1)
    if not b:
        raise EOFError("truncated IFile run")
    first = struct.unpack("b", b)[0]
    if first >= -112:
        return first
    neg = first < -120
    n = (-119 - first) if neg else (-111 - first)
    rest = f.read(n - 1)
    v = 0
    for c in rest:
        v = (v << 8) | c
    return ~v if neg else v


class _Run:
    """A sorted run: in memory (stored IFile segment bytes) or on disk (IFile
    body + CRC32 file)."""
    __slots__ = ("data", "path", "nbytes")

    def __init__(self, data=None, path=None, nbytes=0):
        self.data = data
        self.path = path
        self.nbytes = nbytes


def iter_disk_run(path, bufsize=1 << 20):
    """Stream (key, value) records of an on-disk run, verifying its CRC32."""
    size = os.path.getsize(path)
    with open(path, "rb", buffering=bufsize) as f:
        body_len = size - 4
        crc = 0
        # read the body through a CRC-tracking window
        start = f.tell()
        while f.tell() - start < body_len:
            kl = _read_vint(f)
            vl = _read_vint(f)
            if kl == EOF_MARKER and vl == EOF_MARKER:
                break
            kb = f.read(kl)
            vb = f.read(vl)
            yield kb, vb
        end = f.tell()
        f.seek(0)
        remaining = end
        while remaining > 0:
            chunk = f.read(min(bufsize, remaining))
            crc = zlib.crc32(chunk, crc)
            remaining -= len(chunk)
        f.seek(body_len)
        want = struct.unpack(">I", f.read(4))[0]
    if (crc & 0xFFFFFFFF) != want:
        raise IOError(f"IFile checksum error in {path}")


class ShuffleMerger:
    def __init__(self, job, work_dir, codec, sort_key, kind, reporter, check_killed=None):
        self.codec = codec
        self.sort_key = sort_key
        self.kind = kind
        self.rep = reporter
        self.check_killed = check_killed or (lambda: None)
        self.dir = os.path.join(work_dir, "shuffle")
        mem = job.get_int("hbmr.reduce.shuffle.memory.bytes",
                          job.get_int("hbmr.reduce.shuffle.memory.mb", 256) << 20)
        self.budget = max(1, int(mem * job.get_float("mapred.job.shuffle.input.buffer.percent",
                                                     0.70)))
        self.max_single = int(self.budget * _MAX_SINGLE)
        self.merge_at = int(self.budget * job.get_float("mapred.job.shuffle.merge.percent", 0.66))
        self.inmem_threshold = max(1, job.get_int("mapred.inmem.merge.threshold", 1000))
        self.factor = max(2, job.get_int("io.sort.factor", 10))
        self.runs: list[_Run] = []      # arrival order; in-memory runs only at the tail
        self.mem_bytes = 0
        self._seq = 0
        self.shuffled = 0

    # -- copy phase ------------------------------------------------------------------
    def add(self, data: bytes):
        """One fetched map-output segment (as stored: maybe compressed, + CRC)."""
        self.shuffled += len(data)
        if len(data) > self.max_single:
            # shuffleToDisk: keep order — flush the in-memory tail first
            self._merge_memory()
            path = self._new_path()
            body = sortbuf.segment_body(data, self.codec)
            self._write_body(path, body)
            self.runs.append(_Run(path=path, nbytes=len(body)))
            self.rep.incrCounter(SHUFFLE_GROUP, "SEGMENTS_SHUFFLED_TO_DISK", 1)
        else:
            self.runs.append(_Run(data=data, nbytes=len(data)))
            self.mem_bytes += len(data)
            self.rep.incrCounter(SHUFFLE_GROUP, "SEGMENTS_SHUFFLED_IN_MEMORY", 1)
            mem_runs = sum(1 for r in self.runs if r.data is not None)
            if self.mem_bytes >= self.merge_at or mem_runs >= self.inmem_threshold:
                self._merge_memory()
        ndisk = sum(1 for r in self.runs if r.path is not None)
        if ndisk >= 2 * self.factor - 1:
            self._merge_disk_prefix()

    @property
    def on_disk(self):
        return any(r.path is not None for r in self.runs)

    # -- merges ----------------------------------------------------------------------
    def _new_path(self):
        os.makedirs(self.dir, exist_ok=True)
        self._seq += 1
        return os.path.join(self.dir, f"run{self._seq:05d}.ifile")

    @staticmethod
    def _write_body(path, body):
        from ..fs import STATS
        with open(path, "wb") as f:
            f.write(body)
            f.write(struct.pack(">I", zlib.crc32(body) & 0xFFFFFFFF))
        STATS.add("file", written=len(body) + 4)

    def _records(self, run):
        if run.data is not None:
            return iter(read_segment(run.data, self.codec))
        return iter_disk_run(run.path)

    def _merge_to_disk(self, runs):
        """Stable merge of adjacent runs into one on-disk run."""
        self.check_killed()
        path = self._new_path()
        n = 0
        if self.kind is not None and all(r.data is not None for r in runs):
            # in-memory merge in C++: stable sort of the concatenation
            b = sortbuf.Batch.from_ifile_bodies([sortbuf.segment_body(r.data, self.codec)
                                                 for r in runs])
            perm = b.sort(self.kind, np.zeros(b.n, np.int32))
            body = b.ifile_body(perm, 0, b.n)
            self._write_body(path, body)
            n = b.n
            nbytes = len(body)
        else:
            from ..io.ifile import IFileWriter
            with open(path, "wb") as f:
                w = IFileWriter(f, None)
                for kb, vb in self._merge_iter(runs):
                    w.append(kb, vb)
                    n += 1
                w.close()
            nbytes = os.path.getsize(path)
        for r in runs:
            if r.path is not None:
                os.remove(r.path)
        self.rep.incrCounter(C.TASK_GROUP, C.SPILLED_RECORDS, n)
        return _Run(path=path, nbytes=nbytes)

    def _merge_memory(self):
        """InMemFSMergeThread: the in-memory tail → one on-disk run."""
        i = len(self.runs)
        while i > 0 and self.runs[i - 1].data is not None:
            i -= 1
        tail = self.runs[i:]
        if not tail:
            return
        merged = self._merge_to_disk(tail)
        self.runs[i:] = [merged]
        self.mem_bytes = 0
        self.rep.incrCounter(SHUFFLE_GROUP, "INMEM_MERGES", 1)

    def _merge_disk_prefix(self):
        """LocalFSMerger: merge the first ``factor`` adjacent on-disk runs."""
        j = 0
        while j < len(self.runs) and self.runs[j].path is not None and j < self.factor:
            j += 1
        if j >= 2:
            self.runs[:j] = [self._merge_to_disk(self.runs[:j])]
            self.rep.incrCounter(SHUFFLE_GROUP, "ONDISK_MERGES", 1)

    def _merge_iter(self, runs):
        """k-way merge; ties go to the earlier run (stable)."""
        sk = self.sort_key

        def deco(ri, it):
            for si, (kb, vb) in enumerate(it):
                yield sk(kb), ri, si, kb, vb
        for _k, _ri, _si, kb, vb in heapq.merge(*[deco(i, self._records(r))
                                                   for i, r in enumerate(runs)]):
            yield kb, vb

    # -- sort phase (createKVIterator) -------------------------------------------------
    def memory_bodies(self):
        """All runs are in memory: their decompressed IFile bodies (native path)."""
        return [sortbuf.segment_body(r.data, self.codec) for r in self.runs]

    def memory_records(self):
        return [[(self.sort_key(kb), kb, vb) for kb, vb in read_segment(r.data, self.codec)]
                for r in self.runs]

    def final_iter(self):
        """Records of the merged partition as (sort key, key, value): in-memory
        runs are first written out so the reduce holds ≤ ``factor`` streams
        (mapred.job.reduce.input.buffer.percent = 0), then adjacent runs are
        merged in passes of ``factor`` until one pass remains."""
        self._merge_memory()
        while len(self.runs) > self.factor:
            out = []
            for i in range(0, len(self.runs), self.factor):
                grp = self.runs[i:i + self.factor]
                out.append(grp[0] if len(grp) == 1 else self._merge_to_disk(grp))
            self.runs = out
            self.rep.incrCounter(SHUFFLE_GROUP, "ONDISK_MERGES", 1)
        sk = self.sort_key
        for kb, vb in self._merge_iter(self.runs):
            yield sk(kb), kb, vb

    def cleanup(self):
        for r in self.runs:
            if r.path is not None and os.path.exists(r.path):
                os.remove(r.path)
        self.runs = []
