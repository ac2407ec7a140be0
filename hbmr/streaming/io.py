"""Streaming's pluggable record encodings between the framework and the
streaming process (hadoop-1.0.3 contrib/streaming .../streaming/io/*.java).

An *identifier* names a pair (InputWriter, OutputReader) plus the key/value
classes the OutputReader produces (IdentifierResolver.java):

* ``text``: ``key<sep>value\\n`` lines; output lines are split at the N-th
  separator (``stream.num.{map,reduce}.output.key.fields``,
  ``stream.{map,reduce}.output.field.separator``) — Text/Text;
* ``rawbytes``: each of key and value as int32 length + bytes —
  BytesWritable/BytesWritable;
* ``typedbytes``: each of key and value as one typed-bytes value
  (hbmr.typedbytes) — TypedBytesWritable/TypedBytesWritable.

``-io ID`` sets ``stream.{map,reduce}.{input,output}`` to ID; the resolver
class is ``stream.io.identifier.resolver.class`` (subclass IdentifierResolver
to add identifiers).
"""
from __future__ import annotations

import struct

from ..io.writable import BytesWritable, Text, Writable
from ..typedbytes import TypedBytesInput, TypedBytesWritable, dumps, from_writable

TEXT_ID, RAW_BYTES_ID, TYPED_BYTES_ID = "text", "rawbytes", "typedbytes"


def _sep(job, key, default="\t") -> bytes:
    v = job.get(key)
    if v is None or v == "":
        v = default
    return v.encode("utf-8")


class InputWriter:
    """Writes (key, value) records to the process's stdin (InputWriter.java).
    ``role`` is "map" or "reduce"."""

    def initialize(self, job, role, out):
        self.job, self.role, self.out = job, role, out

    def write_key(self, key):
        raise NotImplementedError

    def write_value(self, value):
        raise NotImplementedError


class OutputReader:
    """Reads (key, value) records from the process's stdout (OutputReader.java)."""

    def initialize(self, job, role, inp):
        self.job, self.role, self.inp = job, role, inp

    def read_key_value(self):
        """The next (key, value), or None at end of stream."""
        raise NotImplementedError


def _utf8(obj) -> bytes:
    if isinstance(obj, (Text, BytesWritable)):
        return obj.bytes
    if isinstance(obj, (bytes, bytearray)):
        return bytes(obj)
    return str(obj).encode("utf-8")


class TextInputWriter(InputWriter):
    def initialize(self, job, role, out):
        super().initialize(job, role, out)
        self.sep = _sep(job, f"stream.{role}.input.field.separator")

    def write_key(self, key):
        self.out.write(_utf8(key) + self.sep)

    def write_value(self, value):
        self.out.write(_utf8(value) + b"\n")


class TextOutputReader(OutputReader):
    def initialize(self, job, role, inp):
        super().initialize(job, role, inp)
        self.sep = _sep(job, f"stream.{role}.output.field.separator")
        self.nkeys = max(1, job.get_int(f"stream.num.{role}.output.key.fields", 1))
        self.last = b""

    def read_key_value(self):
        line = self.inp.readline()
        if not line:
            return None
        if line.endswith(b"\n"):
            line = line[:-1]
            if line.endswith(b"\r"):
                line = line[:-1]
        self.last = line
        return split_key_value(line, self.sep, self.nkeys)


def split_key_value(line: bytes, sep: bytes, nkeys: int = 1):
    """TextOutputReader.splitKeyVal: the key is everything before the
    ``nkeys``-th separator; without that many separators the whole line is
    the key and the value is empty."""
    pos = line.find(sep)
    for _ in range(1, nkeys):
        if pos < 0:
            break
        pos = line.find(sep, pos + len(sep))
    if pos < 0:
        return Text(line), Text(b"")
    return Text(line[:pos]), Text(line[pos + len(sep):])


def _raw(obj) -> bytes:
    if isinstance(obj, (BytesWritable, Text)):
        return obj.bytes
    if isinstance(obj, Writable):
        return obj.serialize()
    return _utf8(obj)


class RawBytesInputWriter(InputWriter):
    def write_key(self, key):
        b = _raw(key)
        self.out.write(struct.pack(">i", len(b)) + b)

    write_value = write_key


class RawBytesOutputReader(OutputReader):
    def _chunk(self):
        n = self.inp.read(4)
        if len(n) < 4:
            return None
        (ln,) = struct.unpack(">i", n)
        b = self.inp.read(ln)
        if len(b) != ln:
            raise EOFError("truncated rawbytes record from the streaming process")
        return b

    def read_key_value(self):
        k = self._chunk()
        if k is None:
            return None
        v = self._chunk()
        if v is None:
            raise EOFError("rawbytes key without a value from the streaming process")
        return BytesWritable(k), BytesWritable(v)


class TypedBytesInputWriter(InputWriter):
    def write_key(self, key):
        if isinstance(key, TypedBytesWritable):
            self.out.write(key.bytes)
        else:
            self.out.write(dumps(from_writable(key)))

    write_value = write_key


class TypedBytesOutputReader(OutputReader):
    def initialize(self, job, role, inp):
        super().initialize(job, role, inp)
        self.tin = TypedBytesInput(inp)

    def read_key_value(self):
        k = self.tin.read_raw()
        if k is None:
            return None
        v = self.tin.read_raw()
        if v is None:
            raise EOFError("typed bytes key without a value from the streaming process")
        return TypedBytesWritable(k), TypedBytesWritable(v)


class IdentifierResolver:
    """IdentifierResolver.java: identifier → writer / reader / key / value classes."""

    TABLE = {
        TEXT_ID: (TextInputWriter, TextOutputReader, Text, Text),
        RAW_BYTES_ID: (RawBytesInputWriter, RawBytesOutputReader, BytesWritable, BytesWritable),
        TYPED_BYTES_ID: (TypedBytesInputWriter, TypedBytesOutputReader, TypedBytesWritable,
                         TypedBytesWritable),
    }

    def resolve(self, ident: str):
        ent = self.TABLE.get((ident or TEXT_ID).lower())
        if ent is None:
            raise ValueError(f"unknown streaming io identifier {ident!r} "
                             f"(known: {', '.join(sorted(self.TABLE))})")
        (self.input_writer_class, self.output_reader_class, self.output_key_class,
         self.output_value_class) = ent
        return self
