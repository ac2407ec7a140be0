"""Many small files per map task (hadoop-1.0.3 mapred/lib/{CombineFileInputFormat,
CombineFileSplit,CombineFileRecordReader}.java, mapred/MultiFileInputFormat.java,
MultiFileSplit.java).

CombineFileInputFormat packs file chunks into splits of at most
``mapred.max.split.size`` bytes (node/rack grouping collapses to one node
here); its record reader opens a per-chunk reader of ``getRecordReaderClass()``
in turn.  MultiFileInputFormat groups whole files into ``numSplits`` splits of
about equal total size.
"""
from __future__ import annotations

import io
import struct

from ...io.writable import Text
from .. import formats as F
from ..api import InputSplit, RecordReader


class CombineFileSplit(InputSplit):
    def __init__(self, paths, starts, lengths, locations=()):
        self.paths, self.starts, self.lengths = list(paths), list(starts), list(lengths)
        self.locations = list(locations)

    def getLength(self):  # noqa: N802
        return sum(self.lengths)

    def getNumPaths(self):  # noqa: N802
        return len(self.paths)

    def getPath(self, i):  # noqa: N802
        return self.paths[i]

    def getOffset(self, i):  # noqa: N802
        return self.starts[i]

    def getLength_i(self, i):  # noqa: N802
        return self.lengths[i]

    def getLocations(self):  # noqa: N802
        return self.locations

    def serialize(self):
        out = [struct.pack(">i", len(self.paths))]
        for p, s, n in zip(self.paths, self.starts, self.lengths):
            out += [Text(p).serialize(), struct.pack(">qq", s, n)]
        return b"".join(out)

    @classmethod
    def deserialize(cls, raw):
        b = io.BytesIO(raw)
        n = struct.unpack(">i", b.read(4))[0]
        ps, ss, ls = [], [], []
        for _ in range(n):
            t = Text()
            t.readFields(b)
            s, ln = struct.unpack(">qq", b.read(16))
            ps.append(str(t))
            ss.append(s)
            ls.append(ln)
        return cls(ps, ss, ls)


class MultiFileSplit(CombineFileSplit):
    pass


class CombineFileRecordReader(RecordReader):
    """Reads chunk after chunk with a per-chunk reader built by
    ``make(job, FileSplit) -> RecordReader``."""

    def __init__(self, job, split: CombineFileSplit, make):
        self.job, self.split, self.make = job, split, make
        self.i = -1
        self.cur = None
        self.done_bytes = 0

    def _advance(self):
        if self.cur is not None:
            self.cur.close()
            self.done_bytes += self.split.lengths[self.i]
        self.i += 1
        if self.i >= len(self.split.paths):
            self.cur = None
            return False
        fs = F.FileSplit(self.split.paths[self.i], self.split.starts[self.i],
                         self.split.lengths[self.i])
        self.cur = self.make(self.job, fs)
        return True

    def next(self):
        while True:
            if self.cur is None and not self._advance():
                return None
            kv = self.cur.next()
            if kv is not None:
                return kv
            if not self._advance():
                return None

    def getProgress(self):  # noqa: N802
        total = self.split.getLength() or 1
        return min(1.0, self.done_bytes / total)

    def close(self):
        if self.cur is not None:
            self.cur.close()


class CombineFileInputFormat(F.FileInputFormat):
    """Subclasses set ``record_reader`` (a ``make(job, FileSplit)`` callable) or
    override getRecordReader."""

    record_reader = staticmethod(F.LineRecordReader)

    def getSplits(self, job, num_splits):  # noqa: N802
        max_size = job.get_long("mapred.max.split.size", 0)
        chunks = []
        for f in self.list_status(job):
            if f.length == 0:
                continue
            if max_size and self.is_splitable(None, f.path):
                off = 0
                while off < f.length:
                    n = min(max_size, f.length - off)
                    chunks.append((f.path, off, n))
                    off += n
            else:
                chunks.append((f.path, 0, f.length))
        out, cur, size = [], [], 0
        for c in chunks:
            if cur and max_size and size + c[2] > max_size:
                out.append(CombineFileSplit(*zip(*cur)))
                cur, size = [], 0
            cur.append(c)
            size += c[2]
        if cur:
            out.append(CombineFileSplit(*zip(*cur)))
        return out

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return CombineFileRecordReader(job, split, type(self).record_reader)


class MultiFileInputFormat(F.FileInputFormat):
    """Whole files grouped into ``num_splits`` splits of similar total length."""

    record_reader = staticmethod(F.LineRecordReader)

    def getSplits(self, job, num_splits):  # noqa: N802
        files = [f for f in self.list_status(job)]
        if not files:
            return []
        n = max(1, min(num_splits or 1, len(files)))
        total = sum(f.length for f in files)
        goal = total / n
        out, cur, size = [], [], 0
        for f in files:
            cur.append((f.path, 0, f.length))
            size += f.length
            if size >= goal and len(out) < n - 1:
                out.append(MultiFileSplit(*zip(*cur)))
                cur, size = [], 0
        if cur:
            out.append(MultiFileSplit(*zip(*cur)))
        return out

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return CombineFileRecordReader(job, split, type(self).record_reader)
