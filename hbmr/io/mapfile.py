"""Sorted, indexed containers on top of SequenceFile: MapFile, ArrayFile,
SetFile and BloomMapFile.

Behaviour of hadoop-1.0.3/src/core/org/apache/hadoop/io/MapFile.java (694),
ArrayFile.java, SetFile.java and BloomMapFile.java, re-designed in Python:

* a MapFile is a directory with ``data`` (a SequenceFile whose keys must be
  appended in non-decreasing order, else ``IOError("key out of order")``,
  MapFile.java:159-170) and ``index`` (a SequenceFile key → LongWritable data
  offset written every ``io.map.index.interval`` = 128 entries, :141-156);
* the Reader loads the index (every ``io.map.index.skip``+1-th entry) once,
  binary-searches it and scans the data forward (``seek``/``get``/
  ``getClosest(before=)``/``midKey``/``finalKey``, :391-560);
* ``fix()`` rebuilds a missing index from the data file (:640-694);
* keys compare by their Writable raw sort key, so no deserialisation is needed
  while scanning;
* block-compressed data gets a sync (block boundary) before every indexed
  entry, so an index offset always starts a block.

BloomMapFile keeps a Bloom filter of the keys in ``bloom`` so a ``get`` of an
absent key usually never touches the data file.  hbmr's filter is a plain bit
array with k double-hashed MD5 probes (JSON header + bits), not Hadoop's
DynamicBloomFilter serialisation.
"""
from __future__ import annotations

import bisect
import hashlib
import json
import math
import os
import shutil
import struct

from . import sequencefile as SF
from .writable import LongWritable, NullWritable

DATA = "data"
INDEX = "index"
BLOOM = "bloom"


def _raw(key):
    return key.serialize()


class MapFileWriter:
    def __init__(self, dirname, key_class, value_class, compression=SF.NONE, codec=None,
                 index_interval=128, conf=None):
        self.dir = str(dirname)
        if conf is not None:
            index_interval = conf.get_int("io.map.index.interval", index_interval)
        os.makedirs(self.dir, exist_ok=True)
        self.key_class = key_class
        self.interval = max(1, index_interval)
        self.data = SF.Writer(os.path.join(self.dir, DATA), key_class, value_class,
                              compression, codec)
        self.index = SF.Writer(os.path.join(self.dir, INDEX), key_class, LongWritable,
                               SF.BLOCK if compression == SF.BLOCK else SF.NONE, codec)
        self.size = 0
        self._last = None
        self._last_index_pos = -1

    def get_index_interval(self):
        return self.interval

    def set_index_interval(self, n):
        self.interval = max(1, int(n))

    def _check_key(self, kb):
        sk = self.key_class.raw_sort_key(kb)
        if self._last is not None and sk < self._last:
            raise IOError(f"key out of order: {self.key_class.deserialize(kb)!r} after "
                          f"previous key")
        self._last = sk

    def append(self, key, value):
        kb = _raw(key)
        vb = value.serialize()
        self._check_key(kb)
        if self.size % self.interval == 0:
            if self.data.compression == SF.BLOCK:
                self.data.sync_now()          # index offsets start a block
            pos = self.data.get_length()
            if pos != self._last_index_pos:
                self.index.append_raw(kb, LongWritable(pos).serialize())
                self._last_index_pos = pos
        self.data.append_raw(kb, vb)
        self.size += 1

    def close(self):
        self.data.close()
        self.index.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class MapFileReader:
    def __init__(self, dirname, conf=None, index_skip=0):
        self.dir = str(dirname)
        if conf is not None:
            index_skip = conf.get_int("io.map.index.skip", index_skip)
        self.data = SF.Reader(os.path.join(self.dir, DATA))
        self.key_class = self.data.key_class
        self.value_class = self.data.value_class
        self._skip = max(0, index_skip)
        self._keys: list | None = None      # raw sort keys of the loaded index
        self._raw_keys: list = []
        self._pos: list = []
        self._first_pos = self.data.get_position()
        self._next_key_raw = None

    def _load_index(self):
        if self._keys is not None:
            return
        keys, raws, pos = [], [], []
        ip = os.path.join(self.dir, INDEX)
        if os.path.exists(ip):
            with SF.Reader(ip) as r:
                i = 0
                while True:
                    kv = r.next_raw()
                    if kv is None:
                        break
                    if i % (self._skip + 1) == 0:
                        p = LongWritable.deserialize(kv[1]).get()
                        if pos and p <= pos[-1]:
                            raise IOError(f"{ip}: index positions not increasing")
                        keys.append(self.key_class.raw_sort_key(kv[0]))
                        raws.append(kv[0])
                        pos.append(p)
                    i += 1
        self._keys, self._raw_keys, self._pos = keys, raws, pos

    # -- sequential access ------------------------------------------------------
    def reset(self):
        self.data.seek(self._first_pos)

    def next(self, key=None, value=None):
        kv = self.data.next_raw()
        if kv is None:
            return False if key is not None else None
        if key is not None:
            key.readFields(_bio(kv[0]))
            if value is not None:
                value.readFields(_bio(kv[1]))
            return True
        return self.key_class.deserialize(kv[0]), self.value_class.deserialize(kv[1])

    def __iter__(self):
        self.reset()
        while True:
            kv = self.next()
            if kv is None:
                return
            yield kv

    # -- keyed access -------------------------------------------------------------
    def _seek_internal(self, key, before=False):
        """Position the data reader at the first entry ≥ key (or, with
        ``before``, the last entry ≤ key).  Returns (cmp, raw_kv) with cmp = 0
        for an exact match, or None when nothing qualifies."""
        self._load_index()
        target = self.key_class.raw_sort_key(_raw(key))
        i = bisect.bisect_right(self._keys, target) - 1
        # equal keys may span index entries: start at the first index key < target
        while i > 0 and self._keys[i] == target:
            i -= 1
        self.data.seek(self._pos[i] if i >= 0 else self._first_pos)
        prev = None
        prev_pos = None
        while True:
            here = self.data.get_position()
            blk_here = (self.data._blk, self.data._blk_i) if self.data.block_compressed else None
            kv = self.data.next_raw()
            if kv is None:
                break
            sk = self.key_class.raw_sort_key(kv[0])
            if sk >= target:
                if before and sk > target:
                    if prev is None:
                        return None
                    self._restore(prev_pos)
                    return (-1, prev)
                self._restore((here, blk_here))
                return (0 if sk == target else 1, kv)
            prev, prev_pos = kv, (here, blk_here)
        if before and prev is not None:
            self._restore(prev_pos)
            return (-1, prev)
        return None

    def _restore(self, state):
        pos, blk = state
        if blk is not None:
            self.data.f.seek(pos)
            self.data._blk, self.data._blk_i = blk
        else:
            self.data.seek(pos)

    def seek(self, key) -> bool:
        """Position at ``key``; True iff it exists (MapFile.Reader.seek)."""
        r = self._seek_internal(key)
        return r is not None and r[0] == 0

    def get(self, key, value=None):
        r = self._seek_internal(key)
        if r is None or r[0] != 0:
            return None
        self.data.next_raw()
        if value is not None:
            value.readFields(_bio(r[1][1]))
            return value
        return self.value_class.deserialize(r[1][1])

    def get_closest(self, key, value=None, before=False):
        """Key of the entry at or after ``key`` (before=True: at or before);
        fills ``value``; None if there is none."""
        r = self._seek_internal(key, before=before)
        if r is None:
            return None
        self.data.next_raw()
        if value is not None:
            value.readFields(_bio(r[1][1]))
        return self.key_class.deserialize(r[1][0])

    getClosest = get_closest  # noqa: N815

    def mid_key(self):
        self._load_index()
        if not self._raw_keys:
            return None
        return self.key_class.deserialize(self._raw_keys[(len(self._raw_keys) - 1) // 2])

    midKey = mid_key  # noqa: N815

    def final_key(self):
        self._load_index()
        start = self._pos[-1] if self._pos else self._first_pos
        save = self.data.get_position()
        self.data.seek(start)
        last = None
        while True:
            kv = self.data.next_raw()
            if kv is None:
                break
            last = kv[0]
        self.data.seek(save)
        return None if last is None else self.key_class.deserialize(last)

    finalKey = final_key  # noqa: N815

    def close(self):
        self.data.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _bio(b):
    import io
    return io.BytesIO(b)


class MapFile:
    Writer = MapFileWriter
    Reader = MapFileReader
    DATA_FILE_NAME = DATA
    INDEX_FILE_NAME = INDEX

    @staticmethod
    def rename(old, new):
        os.rename(old, new)

    @staticmethod
    def delete(name):
        shutil.rmtree(name, ignore_errors=True)

    @staticmethod
    def fix(dirname, key_class=None, value_class=None, dry_run=False, index_interval=128):
        """Rebuild ``index`` from ``data``; returns the number of entries
        (MapFile.fix).  Does nothing (returns -1) if the index exists."""
        ip = os.path.join(str(dirname), INDEX)
        if os.path.exists(ip):
            return -1
        n = 0
        with SF.Reader(os.path.join(str(dirname), DATA)) as r:
            kc = key_class or r.key_class
            w = None if dry_run else SF.Writer(ip, kc, LongWritable)
            last_pos = -1
            while True:
                pos = r.get_position()
                blk_start = r.block_compressed and r._blk_i >= len(r._blk)
                kv = r.next_raw()
                if kv is None:
                    break
                if w is not None and n % index_interval == 0:
                    # block-compressed: only block starts are addressable
                    if (not r.block_compressed or blk_start) and pos != last_pos:
                        w.append_raw(kv[0], LongWritable(pos).serialize())
                        last_pos = pos
                n += 1
            if w is not None:
                w.close()
        return n


# -- ArrayFile: dense LongWritable keys 0..n-1 -----------------------------------------
class ArrayFileWriter(MapFileWriter):
    def __init__(self, dirname, value_class, compression=SF.NONE, codec=None, conf=None):
        super().__init__(dirname, LongWritable, value_class, compression, codec, conf=conf)
        self._n = 0

    def append(self, value):  # noqa: D401 - ArrayFile.Writer.append(Writable)
        super().append(LongWritable(self._n), value)
        self._n += 1


class ArrayFileReader(MapFileReader):
    def seek(self, n) -> bool:  # noqa: D401
        return super().seek(LongWritable(int(n)))

    def get(self, n, value=None):
        return super().get(LongWritable(int(n)), value)

    def next(self, value=None):
        kv = super().next()
        if kv is None:
            return None
        if value is not None:
            value.readFields(_bio(kv[1].serialize()))
            return value
        return kv[1]

    def key(self):
        """Index of the next value (ArrayFile.Reader.key)."""
        pos = self.data.get_position()
        blk = (self.data._blk, self.data._blk_i) if self.data.block_compressed else None
        kv = self.data.next_raw()
        self._restore((pos, blk))
        return None if kv is None else LongWritable.deserialize(kv[0]).get()


class ArrayFile:
    Writer = ArrayFileWriter
    Reader = ArrayFileReader


# -- SetFile: keys only ------------------------------------------------------------------
class SetFileWriter(MapFileWriter):
    def __init__(self, dirname, key_class, compression=SF.NONE, codec=None, conf=None):
        super().__init__(dirname, key_class, NullWritable, compression, codec, conf=conf)

    def append(self, key):  # noqa: D401
        super().append(key, NullWritable())


class SetFileReader(MapFileReader):
    def seek(self, key) -> bool:
        return super().seek(key)

    def contains(self, key) -> bool:
        return super().seek(key)

    def next(self, key=None):
        kv = super().next()
        if kv is None:
            return None
        return kv[0]

    def get(self, key):
        """The stored key equal to ``key`` or None (SetFile.Reader.get)."""
        return key if super().seek(key) else None


class SetFile:
    Writer = SetFileWriter
    Reader = SetFileReader


# -- BloomMapFile ----------------------------------------------------------------------
class BloomFilter:
    def __init__(self, nbits, k):
        self.nbits = max(8, int(nbits))
        self.k = max(1, int(k))
        self.bits = bytearray((self.nbits + 7) // 8)

    @classmethod
    def for_capacity(cls, n, error_rate=0.005):
        n = max(1, n)
        m = math.ceil(-n * math.log(error_rate) / (math.log(2) ** 2))
        k = max(1, round(m / n * math.log(2)))
        return cls(m, k)

    def _probes(self, raw: bytes):
        h = hashlib.md5(raw).digest()
        a, b = struct.unpack("<QQ", h)
        b |= 1
        for i in range(self.k):
            yield (a + i * b) % self.nbits

    def add(self, raw: bytes):
        for p in self._probes(raw):
            self.bits[p >> 3] |= 1 << (p & 7)

    def might_contain(self, raw: bytes) -> bool:
        return all(self.bits[p >> 3] & (1 << (p & 7)) for p in self._probes(raw))

    def save(self, path):
        with open(path, "wb") as f:
            hdr = json.dumps({"nbits": self.nbits, "k": self.k}).encode()
            f.write(struct.pack(">I", len(hdr)) + hdr + bytes(self.bits))

    @classmethod
    def load(cls, path):
        with open(path, "rb") as f:
            (n,) = struct.unpack(">I", f.read(4))
            hdr = json.loads(f.read(n))
            bf = cls(hdr["nbits"], hdr["k"])
            bf.bits = bytearray(f.read())
        return bf


class BloomMapFileWriter(MapFileWriter):
    def __init__(self, dirname, key_class, value_class, compression=SF.NONE, codec=None,
                 conf=None, expected_keys=None, error_rate=None):
        super().__init__(dirname, key_class, value_class, compression, codec, conf=conf)
        if conf is not None:
            expected_keys = expected_keys or conf.get_int("io.mapfile.bloom.size", 1024 * 1024)
            error_rate = error_rate or conf.get_float("io.mapfile.bloom.error.rate", 0.005)
        self.bloom = BloomFilter.for_capacity(expected_keys or 1024 * 1024, error_rate or 0.005)

    def append(self, key, value):
        super().append(key, value)
        self.bloom.add(_raw(key))

    def close(self):
        super().close()
        self.bloom.save(os.path.join(self.dir, BLOOM))


class BloomMapFileReader(MapFileReader):
    def __init__(self, dirname, conf=None):
        super().__init__(dirname, conf)
        self.bloom = BloomFilter.load(os.path.join(self.dir, BLOOM))

    def probably_has_key(self, key) -> bool:
        return self.bloom.might_contain(_raw(key))

    probablyHasKey = probably_has_key  # noqa: N815

    def get(self, key, value=None):
        if not self.probably_has_key(key):
            return None
        return super().get(key, value)


class BloomMapFile:
    Writer = BloomMapFileWriter
    Reader = BloomMapFileReader
