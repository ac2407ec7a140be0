"""CompositeInputFormat and CompositeInputSplit: map-side joins
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/join/CompositeInputFormat.java,
CompositeInputSplit.java).

A job sets ``mapred.input.format.class`` to CompositeInputFormat and
``mapred.join.expr`` to an expression over sources that are sorted by key and
partitioned identically (e.g. the outputs of jobs with the same number of
reduces and partitioner).  Each map then reads the i-th split of every source
and receives (key, TupleWritable) records — no shuffle is needed to join them
(examples/Join.java:144-145)."""
from __future__ import annotations

import io

from ...io.vint import encode_vint, read_vint
from ...io.writable import Text
from ...utils.reflection import class_name, load_class
from ..api import InputFormat, InputSplit
from .parser import parse


class CompositeInputSplit(InputSplit):
    """The i-th split of every join source."""

    def __init__(self, splits=()):
        self.splits = list(splits)

    def add(self, s):
        self.splits.append(s)

    def get(self, i):
        return self.splits[i]

    def getLength(self, i=None):  # noqa: N802
        if i is not None:
            return self.splits[i].getLength()
        return sum(s.getLength() for s in self.splits)

    def getLocations(self):  # noqa: N802
        seen = []
        for s in self.splits:
            for h in s.getLocations() or []:
                if h not in seen:
                    seen.append(h)
        return seen

    def serialize(self) -> bytes:
        """vint count, then (class name, vint length, bytes) per child split."""
        out = io.BytesIO()
        out.write(encode_vint(len(self.splits)))
        for s in self.splits:
            Text.writeString(out, class_name(s))
            raw = s.serialize()
            out.write(encode_vint(len(raw)))
            out.write(raw)
        return out.getvalue()

    @classmethod
    def deserialize(cls, raw: bytes) -> "CompositeInputSplit":
        b = io.BytesIO(raw)
        n = read_vint(b)
        splits = []
        for _ in range(n):
            scls = load_class(Text.readString(b))
            m = read_vint(b)
            splits.append(scls.deserialize(b.read(m)))
        return cls(splits)

    def __repr__(self):
        return "CompositeInputSplit(" + ", ".join(repr(s) for s in self.splits) + ")"


class CompositeInputFormat(InputFormat):
    """InputFormat over a join expression (``mapred.join.expr``)."""

    def __init__(self):
        self.root = None

    def configure(self, job):
        pass

    def setFormat(self, job):  # noqa: N802
        self.root = parse(job.get("mapred.join.expr"), job)

    def getSplits(self, job, num_splits):  # noqa: N802
        self.setFormat(job)
        from ..jobconf import JobConf
        c = JobConf(job)
        # one split per source file: the i-th files of the sources are the
        # i-th partitions and must stay whole (CompositeInputFormat.getSplits)
        c.set_long("mapred.min.split.size", 2 ** 63 - 1)
        return self.root.getSplits(c, num_splits)

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        self.setFormat(job)
        return self.root.getRecordReader(split, job, reporter)

    # -- expression builders (CompositeInputFormat.compose) ----------------------------
    @staticmethod
    def compose(*args) -> str:
        """compose(inf, path) -> 'tbl(inf,"path")';
        compose(op, inf, path1, path2, ...) -> 'op(tbl(inf,"p1"),tbl(inf,"p2"),...)'."""
        if len(args) == 2:
            inf, path = args
            return f'tbl({class_name(inf)},"{path}")'
        op, inf, *paths = args
        return f"{op}(" + ",".join(f'tbl({class_name(inf)},"{p}")' for p in paths) + ")"
