"""Pluggable serialization framework (``io.serializations``).

Behaviour from hadoop-1.0.3/src/core/org/apache/hadoop/io/serializer/
(SerializationFactory.java, Serialization/Serializer/Deserializer,
WritableSerialization.java, JavaSerialization.java): a job may use map-output
key/value types that are not Writables; the factory walks the classes named
in ``io.serializations`` and picks the first whose ``accept(cls)`` is true.

hbmr serializations:

* ``WritableSerialization`` — Writables (their own wire format).
* ``MsgpackSerialization`` — plain Python values (int, float, str, bytes,
  bool, None, tuple, list, dict): the JavaSerialization analogue, but a typed
  data format instead of executable object streams, so map outputs never
  unpickle anything.  Keys sort by their decoded value.
* ``JsonSerialization`` — the same types as UTF-8 JSON (human-readable spills).

``adapter_for(cls, conf)`` returns a class that the MapReduce runtime can use
like a Writable class (``deserialize``/``raw_sort_key``; ``isinstance`` of a
raw value against it checks the underlying type), and :func:`to_bytes`
serialises either kind of object.
"""
from __future__ import annotations

import json

import msgpack

from ..utils.reflection import load_class
from .writable import Writable, hash_bytes

DEFAULT_SERIALIZATIONS = ("hbmr.io.serializer:WritableSerialization,"
                          "hbmr.io.serializer:MsgpackSerialization")
_PLAIN = (int, float, str, bytes, bool, type(None), tuple, list, dict)


class Serialization:
    def accept(self, cls) -> bool:
        raise NotImplementedError

    def serialize(self, obj) -> bytes:
        raise NotImplementedError

    def deserialize(self, raw: bytes, cls):
        raise NotImplementedError

    def sort_key(self, raw: bytes, cls):
        return self.deserialize(raw, cls)


class WritableSerialization(Serialization):
    def accept(self, cls):
        return isinstance(cls, type) and issubclass(cls, Writable)

    def serialize(self, obj):
        return obj.serialize()

    def deserialize(self, raw, cls):
        return cls.deserialize(raw)

    def sort_key(self, raw, cls):
        return cls.raw_sort_key(raw)


class MsgpackSerialization(Serialization):
    def accept(self, cls):
        return cls in _PLAIN

    def serialize(self, obj):
        return msgpack.packb(obj, use_bin_type=True)

    def deserialize(self, raw, cls):
        return msgpack.unpackb(raw, raw=False, use_list=cls is list, strict_map_key=False)


class JsonSerialization(Serialization):
    def accept(self, cls):
        return cls in (int, float, str, bool, type(None), list, dict)

    def serialize(self, obj):
        return json.dumps(obj, separators=(",", ":"), sort_keys=True).encode()

    def deserialize(self, raw, cls):
        return json.loads(raw)


class SerializationFactory:
    def __init__(self, conf=None):
        names = (conf.get("io.serializations", DEFAULT_SERIALIZATIONS) if conf is not None
                 else DEFAULT_SERIALIZATIONS)
        self.serializations = [load_class(n.strip())() for n in names.split(",") if n.strip()]

    def get_serialization(self, cls) -> Serialization:
        for s in self.serializations:
            if s.accept(cls):
                return s
        raise TypeError(f"no serialization in io.serializations accepts {cls!r}")

    getSerialization = get_serialization  # noqa: N815


class _AdapterMeta(type):
    def __instancecheck__(cls, obj):
        return isinstance(obj, cls.underlying)


def adapter_for(cls, conf=None):
    """A Writable-like class for a non-Writable key/value type."""
    if cls is None or (isinstance(cls, type) and issubclass(cls, Writable)):
        return cls
    ser = SerializationFactory(conf).get_serialization(cls)
    if isinstance(ser, WritableSerialization):
        return cls
    ns = {"underlying": cls, "serialization": ser, "hbmr_serialized": True,
          "deserialize": staticmethod(lambda raw: ser.deserialize(raw, cls)),
          "raw_sort_key": staticmethod(lambda raw: ser.sort_key(raw, cls)),
          "encode": staticmethod(ser.serialize)}
    return _AdapterMeta(f"Serialized[{cls.__name__}]", (), ns)


def to_bytes(obj, adapter=None) -> bytes:
    """Serialise a Writable, or a plain value through its adapter (msgpack by default)."""
    if isinstance(obj, Writable):
        return obj.serialize()
    if adapter is not None and getattr(adapter, "hbmr_serialized", False):
        return adapter.encode(obj)
    return msgpack.packb(obj, use_bin_type=True)


def hash_code(obj) -> int:
    """Partitioning hash: Writable.hashCode, else hashBytes of the serialised form."""
    if hasattr(obj, "hash_code"):
        return obj.hash_code()
    return hash_bytes(to_bytes(obj))
