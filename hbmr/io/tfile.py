"""TFile: a sorted (or unsorted) key/value container with block compression,
a block index and named meta blocks.

Behaviour from hadoop-1.0.3/src/core/org/apache/hadoop/io/file/tfile/
(TFile.java, BCFile.java, Utils.java): records are appended as
``VInt klen, key, VInt vlen, value`` into data blocks of at least
``min_block_size`` raw bytes, each compressed on its own (``none`` / ``gz``);
a sorted TFile ("memcmp" comparator) rejects out-of-order keys, records the
first key of every block in the ``TFile.index`` meta block and supports
``Scanner`` ranges, ``seekTo(key)`` (exact), ``lowerBound`` / ``upperBound``
with a binary search over the index then one block decode; user meta blocks
are written and read by name; a fixed trailer (meta-index offset, version,
magic) ends the file.  The layout follows the BCFile idea (data blocks, then
meta blocks, then a meta index) but is hbmr's own encoding, not byte
compatible with Java TFiles.
"""
from __future__ import annotations

import bisect
import io
import struct
import zlib

from .vint import encode_vlong, read_vlong

MAGIC = b"hbmr.TFile.v1\x00\x00\x00"          # 16 bytes
VERSION = (1, 0)
_TRAILER = struct.Struct(">QHH16s")
COMPRESSIONS = ("none", "gz")


def _compress(data: bytes, algo: str) -> bytes:
    return zlib.compress(data, 6) if algo == "gz" else data


def _decompress(data: bytes, algo: str) -> bytes:
    return zlib.decompress(data) if algo == "gz" else data


def _vint(b: io.BytesIO, n: int):
    b.write(encode_vlong(n))


def _read_vint(b) -> int:
    return read_vlong(b)


class Writer:
    def __init__(self, path_or_file, min_block_size=256 * 1024, compression="none",
                 comparator="memcmp"):
        if compression not in COMPRESSIONS:
            raise ValueError(f"unsupported compression {compression!r}")
        if comparator not in ("memcmp", None, ""):
            raise ValueError("only the memcmp comparator (or unsorted) is supported")
        self.f = open(path_or_file, "wb") if isinstance(path_or_file, str) else path_or_file
        self.min_block = min_block_size
        self.algo = compression
        self.sorted = bool(comparator)
        self.comparator = comparator or ""
        self.block = io.BytesIO()
        self.block_entries = 0
        self.block_first = None
        self.last_key = None
        self.index = []          # (first key, offset, compressed len, raw len, entries)
        self.entries = 0
        self.meta = {}
        self.closed = False

    def append(self, key: bytes, value: bytes):
        key, value = bytes(key), bytes(value)
        if self.sorted and self.last_key is not None and key < self.last_key:
            raise ValueError("keys must be appended in memcmp order to a sorted TFile")
        if self.block_first is None:
            self.block_first = key
        _vint(self.block, len(key))
        self.block.write(key)
        _vint(self.block, len(value))
        self.block.write(value)
        self.block_entries += 1
        self.entries += 1
        self.last_key = key
        if self.block.tell() >= self.min_block:
            self._flush_block()

    def _flush_block(self):
        if not self.block_entries:
            return
        raw = self.block.getvalue()
        comp = _compress(raw, self.algo)
        off = self.f.tell()
        self.f.write(comp)
        self.index.append((self.block_first, off, len(comp), len(raw), self.block_entries))
        self.block = io.BytesIO()
        self.block_entries = 0
        self.block_first = None

    def prepare_meta_block(self, name: str, data: bytes):
        if name.startswith("TFile."):
            raise ValueError("TFile.* meta block names are reserved")
        if name in self.meta:
            raise ValueError(f"meta block {name!r} already exists")
        self.meta[name] = bytes(data)

    prepareMetaBlock = prepare_meta_block  # noqa: N815

    def close(self):
        if self.closed:
            return
        self._flush_block()
        idx = io.BytesIO()
        _vint(idx, len(self.index))
        for first, off, clen, rlen, n in self.index:
            _vint(idx, len(first))
            idx.write(first)
            for x in (off, clen, rlen, n):
                _vint(idx, x)
        info = io.BytesIO()
        for s in (self.algo.encode(), self.comparator.encode()):
            _vint(info, len(s))
            info.write(s)
        _vint(info, self.entries)
        blocks = {"TFile.index": idx.getvalue(), "TFile.meta": info.getvalue(), **self.meta}
        locs = []
        for name, data in blocks.items():
            off = self.f.tell()
            self.f.write(data)
            locs.append((name, off, len(data)))
        mi_off = self.f.tell()
        mi = io.BytesIO()
        _vint(mi, len(locs))
        for name, off, n in locs:
            nb = name.encode()
            _vint(mi, len(nb))
            mi.write(nb)
            _vint(mi, off)
            _vint(mi, n)
        self.f.write(mi.getvalue())
        self.f.write(_TRAILER.pack(mi_off, VERSION[0], VERSION[1], MAGIC))
        self.f.close()
        self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Reader:
    def __init__(self, path_or_file):
        self.f = open(path_or_file, "rb") if isinstance(path_or_file, str) else path_or_file
        self.f.seek(0, 2)
        size = self.f.tell()
        if size < _TRAILER.size:
            raise IOError("not a TFile (too short)")
        self.f.seek(size - _TRAILER.size)
        mi_off, major, _minor, magic = _TRAILER.unpack(self.f.read(_TRAILER.size))
        if magic != MAGIC:
            raise IOError("not a TFile (bad magic)")
        if major != VERSION[0]:
            raise IOError(f"incompatible TFile version {major}")
        self.f.seek(mi_off)
        mi = io.BytesIO(self.f.read(size - _TRAILER.size - mi_off))
        self.meta_locs = {}
        for _ in range(_read_vint(mi)):
            name = mi.read(_read_vint(mi)).decode()
            self.meta_locs[name] = (_read_vint(mi), _read_vint(mi))
        info = io.BytesIO(self.get_meta_block("TFile.meta"))
        self.algo = info.read(_read_vint(info)).decode()
        self.comparator = info.read(_read_vint(info)).decode()
        self.entries = _read_vint(info)
        idx = io.BytesIO(self.get_meta_block("TFile.index"))
        self.index = []
        for _ in range(_read_vint(idx)):
            first = idx.read(_read_vint(idx))
            self.index.append((first, *(_read_vint(idx) for _ in range(4))))
        self.first_keys = [b[0] for b in self.index]
        self._cache = (None, None)

    def is_sorted(self):
        return bool(self.comparator)

    isSorted = is_sorted  # noqa: N815

    def get_entry_count(self):
        return self.entries

    getEntryCount = get_entry_count  # noqa: N815

    def get_meta_block(self, name):
        if name not in self.meta_locs:
            raise KeyError(f"no meta block {name!r}")
        off, n = self.meta_locs[name]
        self.f.seek(off)
        return self.f.read(n)

    getMetaBlock = get_meta_block  # noqa: N815

    def _block(self, i):
        if self._cache[0] == i:
            return self._cache[1]
        _, off, clen, _, n = self.index[i]
        self.f.seek(off)
        raw = _decompress(self.f.read(clen), self.algo)
        b = io.BytesIO(raw)
        recs = []
        for _ in range(n):
            k = b.read(_read_vint(b))
            v = b.read(_read_vint(b))
            recs.append((k, v))
        self._cache = (i, recs)
        return recs

    def get_first_key(self):
        return self.first_keys[0] if self.index else None

    def get_last_key(self):
        return self._block(len(self.index) - 1)[-1][0] if self.index else None

    getFirstKey, getLastKey = get_first_key, get_last_key  # noqa: N815

    def _locate(self, key, upper=False):
        """(block, record) of the first entry >= key (> key when upper)."""
        if not self.is_sorted():
            raise ValueError("seeking needs a sorted TFile")
        key = bytes(key)
        i = max(0, bisect.bisect_right(self.first_keys, key) - 1)
        while i < len(self.index):
            recs = self._block(i)
            keys = [k for k, _ in recs]
            j = bisect.bisect_right(keys, key) if upper else bisect.bisect_left(keys, key)
            if j < len(recs):
                return i, j
            i += 1
        return len(self.index), 0

    def create_scanner(self, begin_key=None, end_key=None):
        """Entries with begin_key <= key < end_key (whole file by default)."""
        return Scanner(self, begin_key, end_key)

    createScanner = create_scanner  # noqa: N815

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Scanner:
    def __init__(self, reader: Reader, begin_key=None, end_key=None):
        self.r = reader
        self.end_key = bytes(end_key) if end_key is not None else None
        self.pos = reader._locate(begin_key) if begin_key is not None else (0, 0)

    def seek_to(self, key) -> bool:
        """Position at key; True iff an entry with exactly that key exists."""
        self.pos = self.r._locate(key)
        e = self.entry()
        return e is not None and e[0] == bytes(key)

    def lower_bound(self, key):
        self.pos = self.r._locate(key)

    def upper_bound(self, key):
        self.pos = self.r._locate(key, upper=True)

    seekTo, lowerBound, upperBound = seek_to, lower_bound, upper_bound  # noqa: N815

    def at_end(self) -> bool:
        return self.entry() is None

    atEnd = at_end  # noqa: N815

    def entry(self):
        i, j = self.pos
        if i >= len(self.r.index):
            return None
        recs = self.r._block(i)
        if j >= len(recs):
            return None
        k, v = recs[j]
        if self.end_key is not None and k >= self.end_key:
            return None
        return k, v

    def advance(self) -> bool:
        i, j = self.pos
        if i >= len(self.r.index):
            return False
        j += 1
        if j >= self.r.index[i][4]:
            i, j = i + 1, 0
        self.pos = (i, j)
        return not self.at_end()

    def __iter__(self):
        while True:
            e = self.entry()
            if e is None:
                return
            yield e
            self.advance()
