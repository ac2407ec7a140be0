"""TupleWritable: the value type of a map-side join — one slot per join
source, each either written (the source had the key) or empty.

Wire format as the reference's (hadoop-1.0.3/src/mapred/org/apache/hadoop/
mapred/join/TupleWritable.java:163-195): vint slot count, vlong bitmask of the
written slots, the class name of every slot's value (Text.writeString), then
the written values themselves."""
from __future__ import annotations

import io

from ...io.vint import encode_vlong, read_vlong
from ...io.writable import Text, Writable, class_for_java_name, register_writable


class TupleWritable(Writable):
    JAVA_NAME = "org.apache.hadoop.mapred.join.TupleWritable"

    def __init__(self, values=None):
        self.values = list(values or [])
        self.written = 0
        for i, v in enumerate(self.values):
            if v is not None:
                self.written |= 1 << i

    # -- reference API ---------------------------------------------------------------
    def has(self, i: int) -> bool:
        return bool(self.written >> i & 1)

    def get(self, i: int):
        return self.values[i]

    def size(self) -> int:
        return len(self.values)

    def setWritten(self, i: int):  # noqa: N802
        self.written |= 1 << i

    def clearWritten(self, i: int | None = None):  # noqa: N802
        if i is None:
            self.written = 0
        else:
            self.written &= ~(1 << i)

    def __iter__(self):
        """The written values, in slot order (TupleWritable.iterator)."""
        return (v for i, v in enumerate(self.values) if self.has(i))

    def __len__(self):
        return len(self.values)

    def __eq__(self, other):
        if not isinstance(other, TupleWritable) or self.size() != other.size() or \
                self.written != other.written:
            return False
        return all(self.values[i] == other.values[i] for i in range(self.size()) if self.has(i))

    def __hash__(self):
        return self.written

    def __str__(self):
        return "[" + ",".join(str(v) if self.has(i) else "" for i, v in
                              enumerate(self.values)) + "]"

    __repr__ = __str__

    # -- Writable ----------------------------------------------------------------------
    def serialize(self) -> bytes:
        out = io.BytesIO()
        out.write(encode_vlong(len(self.values)))
        out.write(encode_vlong(self.written))
        for v in self.values:
            cls = type(v) if v is not None else Text
            Text.writeString(out, cls.java_name())
        for i, v in enumerate(self.values):
            if self.has(i):
                out.write(v.serialize())
        return out.getvalue()

    def readFields(self, inp):  # noqa: N802
        n = read_vlong(inp)
        self.written = read_vlong(inp)
        classes = [class_for_java_name(Text.readString(inp)) for _ in range(n)]
        self.values = []
        for i, cls in enumerate(classes):
            v = cls()
            if self.written >> i & 1:
                v.readFields(inp)
            self.values.append(v)


register_writable(TupleWritable, TupleWritable.JAVA_NAME)
