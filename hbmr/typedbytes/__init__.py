"""Typed bytes: a self-describing binary encoding of basic values, the
interchange format of Streaming's ``-io typedbytes`` and of
DumpTypedBytes / LoadTypedBytes (hadoop-1.0.3
src/contrib/streaming/src/java/org/apache/hadoop/typedbytes/{Type,
TypedBytesInput,TypedBytesOutput,TypedBytesWritable,TypedBytesWritableInput,
TypedBytesWritableOutput}.java).

Wire format: one type-code byte, then the payload, big-endian:

  0 BYTES  int32 length + bytes      6 DOUBLE  8 bytes
  1 BYTE   1 byte                    7 STRING  int32 length + UTF-8
  2 BOOL   1 byte (0/1)              8 VECTOR  int32 count + items
  3 INT    4 bytes                   9 LIST    items, then MARKER (255)
  4 LONG   8 bytes                  10 MAP     int32 count + key/value items
  5 FLOAT  4 bytes              50..200 application types: int32 length + bytes

Python values map as: ``Buffer`` (bytes payload of code 0 or 50..200),
``Byte``, int (INT if it fits in 32 bits, else LONG; ``Long`` forces LONG),
bool, ``Float`` (FLOAT) / float (DOUBLE), str, tuple (VECTOR), list (LIST)
and dict (MAP).
"""
from __future__ import annotations

import io
import struct

from ..io.writable import (BooleanWritable, BytesWritable, DoubleWritable, FloatWritable,
                           IntWritable, LongWritable, MapWritable, NullWritable, Text, VIntWritable,
                           VLongWritable, Writable, WritableComparable, _java, hash_bytes)

BYTES, BYTE, BOOL, INT, LONG, FLOAT, DOUBLE, STRING, VECTOR, LIST, MAP = range(11)
WRITABLE = 50
MARKER = 255


class Buffer(bytes):
    """A BYTES payload (record.Buffer in the reference); ``code`` keeps an
    application type code 50..200."""

    def __new__(cls, b=b"", code=BYTES):
        o = super().__new__(cls, b)
        o.code = code
        return o


class Byte(int):
    """A BYTE (signed 8-bit) value."""


class Long(int):
    """An int written as LONG even when it fits in 32 bits."""


class Float(float):
    """A float written as FLOAT (32-bit)."""


class TypedBytesOutput:
    """TypedBytesOutput: typed-bytes writer over a binary stream."""

    def __init__(self, out):
        self.out = out

    def write(self, obj) -> None:
        w = self.out.write
        if isinstance(obj, Buffer):
            w(struct.pack(">Bi", obj.code, len(obj)) + bytes(obj))
        elif isinstance(obj, (bytes, bytearray, memoryview)):
            b = bytes(obj)
            w(struct.pack(">Bi", BYTES, len(b)) + b)
        elif isinstance(obj, bool):
            w(struct.pack(">B?", BOOL, obj))
        elif isinstance(obj, Byte):
            w(struct.pack(">Bb", BYTE, obj))
        elif isinstance(obj, int):
            if not isinstance(obj, Long) and -2 ** 31 <= obj < 2 ** 31:
                w(struct.pack(">Bi", INT, obj))
            else:
                w(struct.pack(">Bq", LONG, obj))
        elif isinstance(obj, Float):
            w(struct.pack(">Bf", FLOAT, obj))
        elif isinstance(obj, float):
            w(struct.pack(">Bd", DOUBLE, obj))
        elif isinstance(obj, str):
            b = obj.encode("utf-8")
            w(struct.pack(">Bi", STRING, len(b)) + b)
        elif isinstance(obj, tuple):
            w(struct.pack(">Bi", VECTOR, len(obj)))
            for x in obj:
                self.write(x)
        elif isinstance(obj, list):
            w(bytes((LIST,)))
            for x in obj:
                self.write(x)
            w(bytes((MARKER,)))
        elif isinstance(obj, dict):
            w(struct.pack(">Bi", MAP, len(obj)))
            for k, v in obj.items():
                self.write(k)
                self.write(v)
        else:
            raise TypeError(f"cannot write objects of type {type(obj).__name__} as typed bytes")

    def write_raw(self, raw: bytes) -> None:
        self.out.write(raw)


class _Marker:
    pass


_END = _Marker()


class TypedBytesInput:
    """TypedBytesInput: ``read()`` returns the next value (None at end of
    stream); ``read_raw()`` the next value's bytes including its code."""

    def __init__(self, inp):
        self.inp = inp

    def _n(self, n) -> bytes:
        b = self.inp.read(n)
        if len(b) != n:
            raise EOFError("truncated typed bytes sequence")
        return b

    def read(self):
        c = self.inp.read(1)
        if not c:
            return None
        v = self._value(c[0])
        return None if v is _END else v

    def _value(self, code):
        if code == BYTES or 50 <= code <= 200:
            n = struct.unpack(">i", self._n(4))[0]
            return Buffer(self._n(n), code)
        if code == BYTE:
            return Byte(struct.unpack(">b", self._n(1))[0])
        if code == BOOL:
            return self._n(1)[0] != 0
        if code == INT:
            return struct.unpack(">i", self._n(4))[0]
        if code == LONG:
            return Long(struct.unpack(">q", self._n(8))[0])
        if code == FLOAT:
            return Float(struct.unpack(">f", self._n(4))[0])
        if code == DOUBLE:
            return struct.unpack(">d", self._n(8))[0]
        if code == STRING:
            n = struct.unpack(">i", self._n(4))[0]
            return self._n(n).decode("utf-8")
        if code == VECTOR:
            n = struct.unpack(">i", self._n(4))[0]
            return tuple(self._item() for _ in range(n))
        if code == LIST:
            out = []
            while True:
                v = self._item(allow_end=True)
                if v is _END:
                    return out
                out.append(v)
        if code == MAP:
            n = struct.unpack(">i", self._n(4))[0]
            d = {}
            for _ in range(n):
                k = self._item()
                d[_hashable(k)] = self._item()
            return d
        if code == MARKER:
            return _END
        raise ValueError(f"unknown typed bytes type code {code}")

    def _item(self, allow_end=False):
        c = self._n(1)[0]
        v = self._value(c)
        if v is _END and not allow_end:
            raise ValueError("unexpected typed bytes list marker")
        return v

    def read_raw(self) -> bytes | None:
        """The next value's raw bytes (type code included); None at end."""
        c = self.inp.read(1)
        if not c:
            return None
        buf = io.BytesIO()
        buf.write(c)
        self._copy(c[0], buf)
        return buf.getvalue()

    def _copy(self, code, buf):
        if code in (BYTES, STRING) or 50 <= code <= 200:
            nb = self._n(4)
            buf.write(nb + self._n(struct.unpack(">i", nb)[0]))
        elif code in (BYTE, BOOL):
            buf.write(self._n(1))
        elif code in (INT, FLOAT):
            buf.write(self._n(4))
        elif code in (LONG, DOUBLE):
            buf.write(self._n(8))
        elif code in (VECTOR, MAP):
            nb = self._n(4)
            buf.write(nb)
            for _ in range(struct.unpack(">i", nb)[0] * (2 if code == MAP else 1)):
                c = self._n(1)
                buf.write(c)
                self._copy(c[0], buf)
        elif code == LIST:
            while True:
                c = self._n(1)
                buf.write(c)
                if c[0] == MARKER:
                    return
                self._copy(c[0], buf)
        elif code != MARKER:
            raise ValueError(f"unknown typed bytes type code {code}")


def _hashable(k):
    if isinstance(k, list):
        return tuple(k)
    if isinstance(k, dict):
        return tuple(sorted(k.items()))
    return k


def dumps(obj) -> bytes:
    b = io.BytesIO()
    TypedBytesOutput(b).write(obj)
    return b.getvalue()


def loads(raw: bytes):
    return TypedBytesInput(io.BytesIO(raw)).read()


def iter_values(inp):
    """Every value of a typed-bytes stream."""
    tin = TypedBytesInput(inp)
    while True:
        c = inp.read(1)
        if not c:
            return
        yield tin._value(c[0])


@_java("org.apache.hadoop.typedbytes.TypedBytesWritable")
class TypedBytesWritable(BytesWritable):
    """TypedBytesWritable: a BytesWritable holding one raw typed-bytes value
    (serialised like BytesWritable: int32 length + the raw bytes)."""

    __slots__ = ()

    @classmethod
    def of(cls, value):
        return cls(dumps(value))

    def get_value(self):
        return loads(self.bytes) if self.bytes else None

    def get_type(self) -> int | None:
        return self.bytes[0] if self.bytes else None

    def hash_code(self):
        return hash_bytes(self.bytes)

    def __str__(self):
        v = self.get_value()
        if isinstance(v, (bytes, Buffer)):
            return " ".join(f"{b:02x}" for b in v)
        return str(v)


# --------------------------------------------------------------------- Writables
def from_writable(w):
    """TypedBytesWritableOutput.write: a Writable as its natural typed value."""
    if isinstance(w, TypedBytesWritable):
        return w.get_value()
    if isinstance(w, Text):
        return w.bytes.decode("utf-8", errors="replace")
    if isinstance(w, BytesWritable):
        return Buffer(w.bytes)
    if isinstance(w, BooleanWritable):
        return bool(w.value)
    if isinstance(w, (VLongWritable,)):
        return Long(int(w.value))
    if isinstance(w, (IntWritable, VIntWritable)):
        return int(w.value)
    if isinstance(w, LongWritable):
        return Long(int(w.value))
    if isinstance(w, FloatWritable):
        return Float(w.value)
    if isinstance(w, DoubleWritable):
        return float(w.value)
    if isinstance(w, NullWritable):
        return Buffer(b"")
    if isinstance(w, MapWritable):
        return {from_writable(k): from_writable(v) for k, v in w.d.items()}
    if isinstance(w, Writable):
        # any other Writable: its serialised bytes under the WRITABLE code
        return Buffer(w.serialize(), WRITABLE)
    return w


def to_writable(v) -> Writable:
    """TypedBytesWritableInput.readWritable: a typed value as a Writable."""
    if isinstance(v, Buffer):
        return BytesWritable(bytes(v))
    if isinstance(v, bool):
        return BooleanWritable(v)
    if isinstance(v, Byte):
        return IntWritable(int(v))
    if isinstance(v, Long):
        return LongWritable(int(v))
    if isinstance(v, int):
        return IntWritable(v) if -2 ** 31 <= v < 2 ** 31 else LongWritable(v)
    if isinstance(v, Float):
        return FloatWritable(float(v))
    if isinstance(v, float):
        return DoubleWritable(v)
    if isinstance(v, str):
        return Text(v)
    return TypedBytesWritable.of(v)


__all__ = ["BYTES", "BYTE", "BOOL", "INT", "LONG", "FLOAT", "DOUBLE", "STRING", "VECTOR", "LIST",
           "MAP", "MARKER", "WRITABLE", "Buffer", "Byte", "Long", "Float", "TypedBytesInput",
           "TypedBytesOutput", "TypedBytesWritable", "dumps", "loads", "iter_values",
           "from_writable", "to_writable", "WritableComparable"]
