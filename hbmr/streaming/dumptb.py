"""DumpTypedBytes / LoadTypedBytes (hadoop-1.0.3 contrib/streaming
DumpTypedBytes.java, LoadTypedBytes.java).

  hbmr dumptb <path>   every (key, value) of the files under <path> (SequenceFiles
                       or text, AutoInputFormat) to stdout as typed bytes
  hbmr loadtb <path>   typed-bytes (key, value) pairs from stdin into the
                       SequenceFile <path> (TypedBytesWritable keys and values)
"""
from __future__ import annotations

import sys

from .. import fs as F
from ..io import sequencefile as seqf
from ..mapred.formats import FileSplit
from ..typedbytes import (TypedBytesInput, TypedBytesOutput, TypedBytesWritable, dumps,
                          from_writable)
from .formats import AutoInputFormat


def _files(path):
    if F.isdir(path):
        return sorted(f for f in (path.rstrip("/") + "/" + n for n in F.listdir(path))
                      if not F.hidden(f.rsplit("/", 1)[-1]) and not F.isdir(f))
    return [path]


def _size(path) -> int:
    return F.get_fs(path).get_file_status(path).length


def dump_typed_bytes(path, out) -> int:
    """Writes every record as two typed-bytes values; returns the record count."""
    fmt = AutoInputFormat()
    tout = TypedBytesOutput(out)
    n = 0
    for f in _files(path):
        rr = fmt.getRecordReader(FileSplit(f, 0, _size(f)), None, None)
        try:
            while True:
                kv = rr.next()
                if kv is None:
                    break
                for w in kv:
                    if isinstance(w, TypedBytesWritable):
                        tout.write_raw(w.bytes)
                    else:
                        tout.write_raw(dumps(from_writable(w)))
                n += 1
        finally:
            rr.close()
    return n


def load_typed_bytes(path, inp) -> int:
    """Reads typed-bytes (key, value) pairs until EOF into a SequenceFile."""
    tin = TypedBytesInput(inp)
    n = 0
    with seqf.Writer(path, TypedBytesWritable, TypedBytesWritable) as w:
        while True:
            k = tin.read_raw()
            if k is None:
                break
            v = tin.read_raw()
            if v is None:
                raise EOFError("typed bytes key without a value")
            w.append(TypedBytesWritable(k), TypedBytesWritable(v))
            n += 1
    return n


def dump_main(argv) -> int:
    if len(argv) != 1:
        print("Usage: hbmr dumptb <path>", file=sys.stderr)
        return 1
    dump_typed_bytes(argv[0], sys.stdout.buffer)
    sys.stdout.buffer.flush()
    return 0


def load_main(argv) -> int:
    if len(argv) != 1:
        print("Usage: hbmr loadtb <path>", file=sys.stderr)
        return 1
    load_typed_bytes(argv[0], sys.stdin.buffer)
    return 0
