"""Writable record types (wire-compatible with org.apache.hadoop.io.*).

Each type serialises exactly like its Hadoop counterpart (big-endian
DataOutput encoding; Text = VInt length + UTF-8) so SequenceFiles written here
are readable by stock Hadoop and vice versa.  ``hash_code`` reproduces Java's
``hashCode`` so :class:`hbmr.mapred.lib.HashPartitioner` routes keys to the same
reducer as Hadoop's ``(hashCode & MAX_INT) % R``
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/lib/HashPartitioner.java:31-34,
src/core/org/apache/hadoop/io/WritableComparator.java:138-142).

``raw_sort_key(raw)`` maps serialised bytes to a Python value whose ordering
equals the type's RawComparator, which is what the map-side sort uses.
"""
from __future__ import annotations

import io
import struct
from functools import total_ordering

import numpy as np

from .vint import decode_vint, encode_vint, read_vint

# one-byte VInt encodings of 0..127 (the common Text length), for serialize()
_VINT1 = [bytes((i,)) for i in range(128)]

_JAVA_NAME_TO_CLASS: dict[str, type] = {}


def _java(name):
    def deco(cls):
        cls.JAVA_NAME = name
        _JAVA_NAME_TO_CLASS[name] = cls
        return cls
    return deco


def java_int(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - 0x100000000 if x & 0x80000000 else x


def hash_bytes(b: bytes) -> int:
    """WritableComparator.hashBytes: h = 31*h + (signed byte), h0 = 1."""
    h = 1
    for x in b:
        h = (31 * h + (x - 256 if x > 127 else x)) & 0xFFFFFFFF
    return java_int(h)


class Writable:
    JAVA_NAME = None

    def write(self, out) -> None:
        out.write(self.serialize())

    def readFields(self, inp) -> None:  # noqa: N802 (Hadoop API name)
        raise NotImplementedError

    def serialize(self) -> bytes:
        raise NotImplementedError

    @classmethod
    def deserialize(cls, raw: bytes):
        obj = cls()
        obj.readFields(io.BytesIO(raw))
        return obj

    @classmethod
    def java_name(cls) -> str:
        return cls.JAVA_NAME or f"{cls.__module__}:{cls.__qualname__}"


@total_ordering
class WritableComparable(Writable):
    def _cmp_key(self):
        return type(self).raw_sort_key(self.serialize())

    @classmethod
    def raw_sort_key(cls, raw: bytes):
        return raw

    def __lt__(self, other):
        return self._cmp_key() < other._cmp_key()

    def __eq__(self, other):
        return type(self) is type(other) and self.serialize() == other.serialize()

    def __hash__(self):
        return self.hash_code()

    def hash_code(self) -> int:
        return hash_bytes(self.serialize())


@_java("org.apache.hadoop.io.Text")
class Text(WritableComparable):
    __slots__ = ("bytes",)

    def __init__(self, value=b""):
        self.set(value)

    def set(self, value):
        if isinstance(value, Text):
            self.bytes = value.bytes
        elif isinstance(value, str):
            self.bytes = value.encode("utf-8")
        else:
            self.bytes = bytes(value)

    def __str__(self):
        return self.bytes.decode("utf-8", errors="replace")

    toString = __str__  # noqa: N815

    def __repr__(self):
        return f"Text({str(self)!r})"

    def getLength(self):  # noqa: N802
        return len(self.bytes)

    def serialize(self) -> bytes:
        b = self.bytes
        n = len(b)
        return (_VINT1[n] if n < 128 else encode_vint(n)) + b

    def readFields(self, inp):  # noqa: N802
        n = read_vint(inp)
        self.bytes = inp.read(n)

    @classmethod
    def deserialize(cls, raw: bytes):
        obj = cls.__new__(cls)
        obj.bytes = raw[1:] if raw[0] < 128 else raw[decode_vint(raw, 0)[1]:]
        return obj

    @classmethod
    def raw_sort_key(cls, raw: bytes):
        _, pos = decode_vint(raw, 0)
        return raw[pos:]

    def hash_code(self) -> int:
        return hash_bytes(self.bytes)

    @staticmethod
    def writeString(out, s: str):  # noqa: N802
        b = s.encode("utf-8")
        out.write(encode_vint(len(b)) + b)

    @staticmethod
    def readString(inp) -> str:  # noqa: N802
        n = read_vint(inp)
        return inp.read(n).decode("utf-8")


class _FixedNum(WritableComparable):
    FMT = ">i"
    __slots__ = ("value",)

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        cls._ST = struct.Struct(cls.FMT)

    def __init__(self, value=0):
        self.value = value

    def get(self):
        return self.value

    def set(self, v):
        self.value = v

    def serialize(self) -> bytes:
        return self._ST.pack(self.value)

    @classmethod
    def deserialize(cls, raw: bytes):
        if cls.readFields is not _FixedNum.readFields:
            return super().deserialize(raw)
        obj = cls.__new__(cls)
        obj.value = cls._ST.unpack(raw)[0]
        return obj

    def readFields(self, inp):  # noqa: N802
        sz = struct.calcsize(self.FMT)
        self.value = struct.unpack(self.FMT, inp.read(sz))[0]

    @classmethod
    def raw_sort_key(cls, raw: bytes):
        return struct.unpack(cls.FMT, raw)[0]

    def __str__(self):
        return str(self.value)

    def __repr__(self):
        return f"{type(self).__name__}({self.value!r})"


@_java("org.apache.hadoop.io.IntWritable")
class IntWritable(_FixedNum):
    FMT = ">i"

    def hash_code(self):
        return java_int(self.value)


@_java("org.apache.hadoop.io.LongWritable")
class LongWritable(_FixedNum):
    FMT = ">q"

    def hash_code(self):
        v = self.value & 0xFFFFFFFFFFFFFFFF
        return java_int(v ^ (v >> 32))


@_java("org.apache.hadoop.io.FloatWritable")
class FloatWritable(_FixedNum):
    FMT = ">f"

    def hash_code(self):
        return java_int(struct.unpack(">I", struct.pack(">f", self.value))[0])


@_java("org.apache.hadoop.io.DoubleWritable")
class DoubleWritable(_FixedNum):
    FMT = ">d"

    def hash_code(self):
        v = struct.unpack(">Q", struct.pack(">d", self.value))[0]
        return java_int(v ^ (v >> 32))


@_java("org.apache.hadoop.io.BooleanWritable")
class BooleanWritable(_FixedNum):
    FMT = ">?"

    def hash_code(self):
        return 1 if self.value else 0


@_java("org.apache.hadoop.io.VIntWritable")
class VIntWritable(_FixedNum):
    def serialize(self):
        return encode_vint(self.value)

    def readFields(self, inp):  # noqa: N802
        self.value = read_vint(inp)

    @classmethod
    def raw_sort_key(cls, raw):
        return decode_vint(raw, 0)[0]

    def hash_code(self):
        return java_int(self.value)


@_java("org.apache.hadoop.io.VLongWritable")
class VLongWritable(VIntWritable):
    def hash_code(self):
        v = self.value & 0xFFFFFFFFFFFFFFFF
        return java_int(v ^ (v >> 32))


@_java("org.apache.hadoop.io.NullWritable")
class NullWritable(WritableComparable):
    _inst = None

    def __new__(cls):
        if cls._inst is None:
            cls._inst = super().__new__(cls)
        return cls._inst

    @classmethod
    def get(cls):
        return cls()

    def serialize(self):
        return b""

    def readFields(self, inp):  # noqa: N802
        pass

    @classmethod
    def raw_sort_key(cls, raw):
        return 0

    def hash_code(self):
        return 0

    def __str__(self):
        return "(null)"


@_java("org.apache.hadoop.io.BytesWritable")
class BytesWritable(WritableComparable):
    __slots__ = ("bytes",)

    def __init__(self, value=b""):
        self.bytes = bytes(value)

    def get(self):
        return self.bytes

    getBytes = get  # noqa: N815

    def getLength(self):  # noqa: N802
        return len(self.bytes)

    def serialize(self):
        return struct.pack(">i", len(self.bytes)) + self.bytes

    def readFields(self, inp):  # noqa: N802
        n = struct.unpack(">i", inp.read(4))[0]
        self.bytes = inp.read(n)

    @classmethod
    def raw_sort_key(cls, raw):
        return raw[4:]

    def hash_code(self):
        return hash_bytes(self.bytes)

    def __str__(self):
        return " ".join(f"{b:02x}" for b in self.bytes)


@_java("org.apache.hadoop.io.ArrayWritable")
class ArrayWritable(Writable):
    value_class = Text

    def __init__(self, values=(), value_class=None):
        if value_class is not None:
            self.value_class = value_class
        self.values = list(values)

    def serialize(self):
        return struct.pack(">i", len(self.values)) + b"".join(v.serialize() for v in self.values)

    def readFields(self, inp):  # noqa: N802
        n = struct.unpack(">i", inp.read(4))[0]
        self.values = []
        for _ in range(n):
            v = self.value_class()
            v.readFields(inp)
            self.values.append(v)


@_java("org.apache.hadoop.io.MapWritable")
class MapWritable(Writable):
    """Simplified MapWritable: Text keys/values only (class-id table omitted)."""

    def __init__(self, d=None):
        self.d = dict(d or {})

    def serialize(self):
        out = io.BytesIO()
        out.write(struct.pack(">i", len(self.d)))
        for k, v in self.d.items():
            Text(k).write(out)
            Text(v).write(out)
        return out.getvalue()

    def readFields(self, inp):  # noqa: N802
        n = struct.unpack(">i", inp.read(4))[0]
        self.d = {}
        for _ in range(n):
            k = Text()
            k.readFields(inp)
            v = Text()
            v.readFields(inp)
            self.d[str(k)] = str(v)


@_java("hbmr.io.FloatVectorWritable")
class FloatVectorWritable(WritableComparable):
    """Dense float32 vector: int32 BE count + count big-endian float32s.

    The K-Means and matmul record type.  ``numpy()`` returns a native float32
    view; bulk readers in :mod:`hbmr.gpu.split_cache` decode whole splits at once.
    """
    __slots__ = ("vec",)

    def __init__(self, vec=()):
        self.vec = np.asarray(vec, dtype=np.float32)

    def numpy(self):
        return self.vec

    def serialize(self):
        v = np.ascontiguousarray(self.vec, dtype=">f4")
        return struct.pack(">i", v.size) + v.tobytes()

    def readFields(self, inp):  # noqa: N802
        n = struct.unpack(">i", inp.read(4))[0]
        self.vec = np.frombuffer(inp.read(4 * n), dtype=">f4").astype(np.float32)

    @classmethod
    def raw_sort_key(cls, raw):
        return tuple(np.frombuffer(raw[4:], dtype=">f4").tolist())

    def __str__(self):
        return ",".join(f"{x:g}" for x in self.vec.tolist())


def class_for_java_name(name: str) -> type:
    if name in _JAVA_NAME_TO_CLASS:
        return _JAVA_NAME_TO_CLASS[name]
    if ":" in name:
        from ..utils.reflection import load_class
        return load_class(name)
    raise KeyError(f"unknown Writable class {name!r}")


def register_writable(cls, java_name: str | None = None):
    name = java_name or cls.java_name()
    cls.JAVA_NAME = name
    _JAVA_NAME_TO_CLASS[name] = cls
    return cls


def writable_from(value):
    """Wrap a plain Python value as the natural Writable."""
    if isinstance(value, Writable):
        return value
    if isinstance(value, bool):
        return BooleanWritable(value)
    if isinstance(value, int):
        return LongWritable(value) if not -2**31 <= value < 2**31 else IntWritable(value)
    if isinstance(value, float):
        return DoubleWritable(value)
    if isinstance(value, (str, bytes)):
        return Text(value)
    if value is None:
        return NullWritable()
    if isinstance(value, np.ndarray):
        return FloatVectorWritable(value)
    raise TypeError(f"cannot wrap {type(value)} as a Writable")


_I32 = struct.Struct(">i")


def _text_payload(raw: bytes) -> bytes:
    n = len(raw)
    return (_VINT1[n] if n < 128 else encode_vint(n)) + raw


def _bytes_payload(raw: bytes) -> bytes:
    return _I32.pack(len(raw)) + raw


def serialize_in_place(ser, raw, room=8):
    """``ser(raw)`` without copying a large payload: ``raw`` a memoryview
    that starts ``room`` bytes into its own bytearray (the Pipes uplink's
    large values, UplinkReader._value) gets its serialisation prefix written
    into that room and comes back as a view of prefix + payload."""
    if raw.__class__ is memoryview:
        buf = raw.obj
        if buf.__class__ is bytearray and len(buf) == len(raw) + room:
            pre = _prefix_of(ser, len(raw))
            if pre is not None and len(pre) <= room:
                start = room - len(pre)
                buf[start:room] = pre
                return memoryview(buf)[start:]
        return ser(bytes(raw))
    return ser(raw)


def _prefix_of(ser, n):
    if ser is _bytes_payload:
        return _I32.pack(n)
    if ser is _text_payload:
        return _VINT1[n] if n < 128 else encode_vint(n)
    return None


def payload_serializer(cls):
    """raw payload bytes -> ``cls``'s serialised form, for the classes whose
    Pipes wire form is the bare payload (Text, BytesWritable; BinaryProtocol.
    writeObject, BinaryProtocol.java:349-369), so a Pipes child's output can be
    collected without building Writables; None for any other class."""
    if cls is Text:
        return _text_payload
    if cls is BytesWritable:
        return _bytes_payload
    return None

