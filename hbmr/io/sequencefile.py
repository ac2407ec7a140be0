"""SequenceFile version 6 reader/writer, byte-compatible with Hadoop 1.0.3.

Layout (hadoop-1.0.3/src/core/org/apache/hadoop/io/SequenceFile.java:191-203
header constants, Writer.writeFileHeader, Reader.init, sync handling):

    'SEQ' 0x06 | Text keyClass | Text valueClass | bool compressed |
    bool blockCompressed | [Text codecClass] | Metadata(int n, n×(Text,Text)) |
    16-byte sync
    records:  [int -1, sync]  int recLen  int keyLen  key  value
    blocks :  int -1, sync, VInt nrec, 4 × (VInt len, compressed buffer)
              (key lengths, keys, value lengths, values)

Sync markers are emitted at most every SYNC_INTERVAL (2000) bytes so readers
can start inside a file (``sync(pos)``), which is how FileInputFormat splits
are honoured by :class:`SequenceFileRecordReader`.
"""
from __future__ import annotations

import hashlib
import io
import os
import struct
import time
import uuid

from .compress import get_codec
from .vint import decode_vint, encode_vint, read_vint
from .writable import Text, Writable, class_for_java_name

VERSION = 6
SYNC_ESCAPE = -1
SYNC_HASH_SIZE = 16
SYNC_SIZE = 4 + SYNC_HASH_SIZE
SYNC_INTERVAL = 100 * SYNC_SIZE
BLOCK_SIZE_DEFAULT = 1_000_000  # io.seqfile.compress.blocksize

NONE, RECORD, BLOCK = "NONE", "RECORD", "BLOCK"


def _cls_name(c) -> str:
    if isinstance(c, str):
        return c
    return c.java_name() if hasattr(c, "java_name") else f"{c.__module__}:{c.__qualname__}"


class Metadata:
    def __init__(self, d=None):
        self.d = dict(d or {})

    def write(self, out):
        out.write(struct.pack(">i", len(self.d)))
        for k in sorted(self.d):
            Text(k).write(out)
            Text(self.d[k]).write(out)

    @classmethod
    def read(cls, inp):
        n = struct.unpack(">i", inp.read(4))[0]
        d = {}
        for _ in range(n):
            k, v = Text(), Text()
            k.readFields(inp)
            v.readFields(inp)
            d[str(k)] = str(v)
        return cls(d)


class _PosFile:
    """Buffered binary file that tracks its logical position."""

    def __init__(self, f):
        self.f = f
        self.pos = f.tell()

    def write(self, b):
        self.f.write(b)
        self.pos += len(b)

    def tell(self):
        return self.pos

    def flush(self):
        self.f.flush()

    def close(self):
        self.f.close()


class Writer:
    def __init__(self, path, key_class, value_class, compression: str = NONE, codec=None,
                 metadata: dict | None = None, block_size: int = BLOCK_SIZE_DEFAULT, fs=None):
        self.path = str(path)
        self.key_class = key_class
        self.value_class = value_class
        self.compression = (compression or NONE).upper()
        if self.compression not in (NONE, RECORD, BLOCK):
            raise ValueError(f"bad compression type {compression}")
        self.codec = get_codec(codec or "default") if self.compression != NONE else None
        self.block_size = block_size
        from .. import fs as F
        d = os.path.dirname(self.path)
        if d:
            F.makedirs(d)
        self.out = _PosFile(F.fopen(self.path, "wb"))
        self.sync = hashlib.md5(f"{uuid.uuid4()}@{time.time_ns()}".encode()).digest()
        self.last_sync_pos = 0
        self._blk_keys = io.BytesIO()
        self._blk_vals = io.BytesIO()
        self._blk_klens = io.BytesIO()
        self._blk_vlens = io.BytesIO()
        self._blk_n = 0
        self._write_header(Metadata(metadata))

    def _write_header(self, meta: Metadata):
        o = self.out
        o.write(b"SEQ" + bytes([VERSION]))
        Text.writeString(o, _cls_name(self.key_class))
        Text.writeString(o, _cls_name(self.value_class))
        o.write(bytes([self.compression != NONE, self.compression == BLOCK]))
        if self.codec is not None:
            Text.writeString(o, self.codec.JAVA_NAME)
        meta.write(o)
        o.write(self.sync)

    def _check_and_write_sync(self):
        if self.out.tell() >= self.last_sync_pos + SYNC_INTERVAL:
            self._write_sync()

    def _write_sync(self):
        if self.last_sync_pos != self.out.tell():
            self.out.write(struct.pack(">i", SYNC_ESCAPE))
            self.out.write(self.sync)
            self.last_sync_pos = self.out.tell()

    def append(self, key, value):
        kb = key.serialize() if isinstance(key, Writable) else bytes(key)
        vb = value.serialize() if isinstance(value, Writable) else bytes(value)
        self.append_raw(kb, vb)

    def append_raw(self, kb: bytes, vb: bytes):
        if self.compression == BLOCK:
            self._blk_klens.write(encode_vint(len(kb)))
            self._blk_keys.write(kb)
            self._blk_vlens.write(encode_vint(len(vb)))
            self._blk_vals.write(vb)
            self._blk_n += 1
            if self._blk_keys.tell() + self._blk_vals.tell() >= self.block_size:
                self._flush_block()
            return
        if self.compression == RECORD:
            vb = self.codec.compress(vb)
        self._check_and_write_sync()
        self.out.write(struct.pack(">ii", len(kb) + len(vb), len(kb)))
        self.out.write(kb)
        self.out.write(vb)

    def _flush_block(self):
        if self._blk_n == 0:
            return
        self._write_sync()
        self.out.write(encode_vint(self._blk_n))
        for buf in (self._blk_klens, self._blk_keys, self._blk_vlens, self._blk_vals):
            c = self.codec.compress(buf.getvalue())
            self.out.write(encode_vint(len(c)))
            self.out.write(c)
            buf.seek(0)
            buf.truncate()
        self._blk_n = 0

    def get_length(self):
        return self.out.tell()

    getLength = get_length  # noqa: N815

    def sync_now(self):
        if self.compression == BLOCK:
            self._flush_block()
        else:
            self._write_sync()

    def close(self):
        if self.out is None:
            return
        if self.compression == BLOCK:
            self._flush_block()
        self.out.close()
        self.out = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Reader:
    def __init__(self, path, fs=None, buffer_size: int = 1 << 20):
        from .. import fs as F
        self.path = str(path)
        self.f = F.fopen(self.path, "rb", buffering=buffer_size)
        if F.is_dfs(self.path):
            self.file_len = F.get_fs(self.path).get_file_status(self.path).length
        else:
            self.file_len = os.fstat(self.f.fileno()).st_size
        magic = self.f.read(3)
        if magic != b"SEQ":
            raise IOError(f"{self.path} is not a SequenceFile")
        self.version = self.f.read(1)[0]
        if self.version < 5:
            raise IOError(f"unsupported SequenceFile version {self.version}")
        self.key_class_name = Text.readString(self.f)
        self.value_class_name = Text.readString(self.f)
        flags = self.f.read(2)
        self.decompress = bool(flags[0])
        self.block_compressed = bool(flags[1])
        self.codec = None
        if self.decompress:
            self.codec = get_codec(Text.readString(self.f))
        self.metadata = Metadata.read(self.f).d
        self.sync = self.f.read(SYNC_HASH_SIZE)
        self.header_end = self.f.tell()
        self.sync_seen = False
        self._blk = []          # buffered (k, v) of the current block
        self._blk_i = 0

    # -- classes -----------------------------------------------------------
    @property
    def key_class(self):
        return class_for_java_name(self.key_class_name)

    @property
    def value_class(self):
        return class_for_java_name(self.value_class_name)

    getKeyClass = key_class  # noqa: N815
    getValueClass = value_class  # noqa: N815

    @property
    def compression(self):
        return BLOCK if self.block_compressed else (RECORD if self.decompress else NONE)

    # -- positioning -------------------------------------------------------
    def get_position(self) -> int:
        return self.f.tell()

    getPosition = get_position  # noqa: N815

    def seek(self, pos: int):
        self.f.seek(pos)
        self._blk = []
        self._blk_i = 0

    def sync_to(self, position: int):
        """Seek to the first sync marker at or after ``position`` (Reader.sync)."""
        if position + SYNC_SIZE >= self.file_len:
            self.seek(self.file_len)
            return
        if position < self.header_end:
            self.seek(self.header_end)
            self.sync_seen = True
            return
        self.f.seek(position + 4)  # skip the escape int
        window = self.f.read(SYNC_HASH_SIZE)
        pos = position + 4
        while len(window) == SYNC_HASH_SIZE:
            if window == self.sync:
                # position at the escape int preceding the hash
                self.seek(pos - 4)
                return
            nxt = self.f.read(1)
            if not nxt:
                break
            window = window[1:] + nxt
            pos += 1
        self.seek(self.file_len)

    def _read_int(self):
        b = self.f.read(4)
        if len(b) < 4:
            return None
        return struct.unpack(">i", b)[0]

    # -- record iteration --------------------------------------------------
    def next_raw(self):
        """Return (key_bytes, value_bytes) or None at EOF."""
        self.sync_seen = False
        if self.block_compressed:
            if self._blk_i >= len(self._blk):
                if not self._read_block():
                    return None
            kv = self._blk[self._blk_i]
            self._blk_i += 1
            return kv
        length = self._read_int()
        if length is None:
            return None
        if length == SYNC_ESCAPE:
            h = self.f.read(SYNC_HASH_SIZE)
            if h != self.sync:
                raise IOError(f"{self.path}: sync check failure")
            self.sync_seen = True
            length = self._read_int()
            if length is None:
                return None
        klen = self._read_int()
        kb = self.f.read(klen)
        vb = self.f.read(length - klen)
        if self.decompress:
            vb = self.codec.decompress(vb)
        return kb, vb

    def _read_block(self):
        esc = self._read_int()
        if esc is None:
            return False
        if esc != SYNC_ESCAPE:
            raise IOError(f"{self.path}: expected sync before block")
        if self.f.read(SYNC_HASH_SIZE) != self.sync:
            raise IOError(f"{self.path}: sync check failure")
        self.sync_seen = True
        n = read_vint(self.f)
        bufs = []
        for _ in range(4):
            ln = read_vint(self.f)
            bufs.append(self.codec.decompress(self.f.read(ln)))
        klens, keys, vlens, vals = bufs
        out = []
        kp = vp = kl = vl = 0
        for _ in range(n):
            a, kl = decode_vint(klens, kl)
            b, vl = decode_vint(vlens, vl)
            out.append((keys[kp:kp + a], vals[vp:vp + b]))
            kp += a
            vp += b
        self._blk = out
        self._blk_i = 0
        return True

    def next(self, key=None, value=None):
        raw = self.next_raw()
        if raw is None:
            return False if key is not None else None
        kb, vb = raw
        if key is not None:
            key.readFields(io.BytesIO(kb))
            if value is not None:
                value.readFields(io.BytesIO(vb))
            return True
        return self.key_class.deserialize(kb), self.value_class.deserialize(vb)

    def __iter__(self):
        kc, vc = self.key_class, self.value_class
        while True:
            raw = self.next_raw()
            if raw is None:
                return
            yield kc.deserialize(raw[0]), vc.deserialize(raw[1])

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def createWriter(path, key_class, value_class, compression=NONE, codec=None, metadata=None,  # noqa: N802
                 **kw):
    return Writer(path, key_class, value_class, compression, codec, metadata, **kw)


class Sorter:
    """SequenceFile.Sorter (hadoop-1.0.3/src/core/org/apache/hadoop/io/
    SequenceFile.java:2269): sort the records of SequenceFiles by key into one
    SequenceFile, or merge already-sorted ones.

    ``sort`` reads the inputs in order, cuts them into runs of at most
    ``io.sort.mb`` (``hbmr.io.sort.bytes``) raw bytes, sorts each run in memory
    (stable, by the key type's raw comparator — ``key_class.raw_sort_key`` or a
    given ``comparator`` over raw key bytes) and writes it as a temporary
    SequenceFile; ``merge`` combines sorted files ``io.sort.factor`` at a time
    (multi-pass) with a streaming k-way merge whose ties go to the earlier
    input, so equal keys keep their input order.  Output compression defaults
    to NONE (``compression``/``codec`` as for :class:`Writer`)."""

    def __init__(self, key_class, value_class, conf=None, comparator=None,
                 compression: str = NONE, codec=None, tmp_dir=None):
        self.kcls, self.vcls = key_class, value_class
        get = (lambda k, d: conf.get_int(k, d)) if conf is not None else (lambda k, d: d)
        self.memory = get("hbmr.io.sort.bytes", get("io.sort.mb", 100) << 20)
        self.factor = max(2, get("io.sort.factor", 10))
        self.sort_key = comparator or key_class.raw_sort_key
        self.compression, self.codec = compression, codec
        self.tmp_dir = tmp_dir
        self.runs_written = 0
        self.merge_passes = 0

    def _writer(self, path):
        return Writer(path, self.kcls, self.vcls, self.compression, self.codec)

    def _tmp(self, out_path, i):
        d = self.tmp_dir or (str(out_path) + ".sort-tmp")
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, f"run-{i:05d}.seq")

    @staticmethod
    def _records(path):
        with Reader(path) as r:
            while True:
                raw = r.next_raw()
                if raw is None:
                    return
                yield raw

    def sort(self, in_paths, out_path, delete_input=False) -> int:
        """Sort the records of ``in_paths`` into ``out_path``; returns the count."""
        if isinstance(in_paths, (str, os.PathLike)):
            in_paths = [in_paths]
        runs, buf, size, total = [], [], 0, 0
        sk = self.sort_key

        def flush():
            nonlocal buf, size
            if not buf and runs:
                return
            buf.sort(key=lambda r: sk(r[0]))          # stable
            path = self._tmp(out_path, len(runs))
            with self._writer(path) as w:
                for kb, vb in buf:
                    w.append_raw(kb, vb)
            runs.append(path)
            self.runs_written += 1
            buf, size = [], 0
        for p in in_paths:
            for kb, vb in self._records(str(p)):
                buf.append((kb, vb))
                size += len(kb) + len(vb) + 16
                total += 1
                if size >= self.memory:
                    flush()
        flush()
        if len(runs) == 1:
            os.replace(runs[0], str(out_path))
        else:
            self.merge(runs, out_path, delete_input=True)
        tmp = self.tmp_dir or (str(out_path) + ".sort-tmp")
        if os.path.isdir(tmp) and not os.listdir(tmp):
            os.rmdir(tmp)
        if delete_input:
            for p in in_paths:
                os.remove(str(p))
        return total

    def _merge_iter(self, paths):
        import heapq
        sk = self.sort_key

        def deco(i, it):
            for j, (kb, vb) in enumerate(it):
                yield sk(kb), i, j, kb, vb
        for _k, _i, _j, kb, vb in heapq.merge(*[deco(i, self._records(str(p)))
                                                for i, p in enumerate(paths)]):
            yield kb, vb

    def merge(self, in_paths, out_path, delete_input=False) -> int:
        """Merge sorted ``in_paths`` into ``out_path`` (multi-pass at
        ``io.sort.factor``); returns the number of records."""
        paths = [str(p) for p in in_paths]
        owned: set = set()
        gen = 0
        while len(paths) > self.factor:
            nxt = []
            for i in range(0, len(paths), self.factor):
                grp = paths[i:i + self.factor]
                if len(grp) == 1:
                    nxt.append(grp[0])
                    continue
                tmp = self._tmp(out_path, 100000 + gen)
                gen += 1
                with self._writer(tmp) as w:
                    for kb, vb in self._merge_iter(grp):
                        w.append_raw(kb, vb)
                for g in grp:
                    if g in owned or delete_input:
                        os.remove(g)
                owned.add(tmp)
                nxt.append(tmp)
            paths = nxt
            self.merge_passes += 1
        n = 0
        with self._writer(str(out_path)) as w:
            for kb, vb in self._merge_iter(paths):
                w.append_raw(kb, vb)
                n += 1
        self.merge_passes += 1
        for g in paths:
            if g in owned or delete_input:
                os.remove(g)
        return n
