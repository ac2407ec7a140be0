"""Text / WordCount primitives (native/kernels/text.hip) and their CPU twins.

A word table travels as ``(blob, counts)``: ``blob`` is a uint8 tensor
``b"w1\\nw2\\n..."`` of distinct words and ``counts`` an int64 tensor with one
count per word, in blob order.  The same layout is the map output, the
shuffle payload (one contiguous run per reduce partition) and the reduce
input, so every stage is tokenize → exact hash-aggregate → (partition) → pack.

On a GPU the native library must load (no silent fallback); the CPU versions
back CPU map slots and the tests' references.
"""
from __future__ import annotations

import collections

import torch

from . import _lib
from ..io.writable import hash_bytes

_TABLE_MAX = 1 << 28
INITIAL_TABLE = 1 << 21     # first word-table size tried (slots)


def _ptr(t):
    return None if t is None else t.data_ptr()


def _st(stream):
    return _lib.stream_handle(stream)


def _call(name, *args):
    lib = _lib.load()
    _lib.check(getattr(lib, name)(*args), name)


# --------------------------------------------------------------------------- GPU
def tokenize(buf: torch.Tensor, stream=None):
    """Word (start, len) int32 pairs of a uint8 device buffer, in order."""
    n = buf.numel()
    dev = buf.device
    lib = _lib.load()
    tiles = lib.hbmr_wc_tiles(n)
    if tiles == 0:
        z = torch.empty(0, dtype=torch.int32, device=dev)
        return z, z
    tc = torch.empty(tiles, dtype=torch.int32, device=dev)
    _call("hbmr_wc_tokenize_count", _ptr(buf), n, _ptr(tc), _st(stream))
    base = torch.zeros(tiles, dtype=torch.int64, device=dev)
    csum = torch.cumsum(tc.to(torch.int64), 0)
    base[1:] = csum[:-1]
    nw = int(csum[-1])
    starts = torch.empty(nw, dtype=torch.int32, device=dev)
    lens = torch.empty(nw, dtype=torch.int32, device=dev)
    if nw:
        _call("hbmr_wc_tokenize_write", _ptr(buf), n, _ptr(base), _ptr(starts), _ptr(lens),
              _st(stream))
    return starts, lens


def _pow2(x):
    return 1 << max(10, int(x - 1).bit_length())


def aggregate(buf, starts, lens, weights=None, R=1, stream=None):
    """Exact per-word totals: (ustart, ulen, ucount int64, upart int32), unordered.
    ``upart`` = (Text.hashCode() & INT_MAX) % R (Hadoop's HashPartitioner)."""
    dev = buf.device
    nw = starts.numel()
    n = buf.numel()
    # distinct words are usually far fewer than words: start at ≤ 2M slots
    # (32 MiB of keys + counts) and grow on overflow (bounded probe runs)
    full = min(_pow2(2 * max(nw, 1)), _TABLE_MAX)
    cap = min(full, INITIAL_TABLE)
    while True:
        tkeys = torch.zeros(cap, dtype=torch.int64, device=dev)
        tcounts = torch.zeros(cap, dtype=torch.int64, device=dev)
        ovf = torch.zeros(1, dtype=torch.int32, device=dev)
        if nw:
            _call("hbmr_wc_insert", _ptr(buf), n, _ptr(starts), _ptr(lens), _ptr(weights), nw,
                  _ptr(tkeys), _ptr(tcounts), cap, _ptr(ovf), _st(stream))
        if int(ovf) == 0:
            break
        if cap >= full:
            raise RuntimeError(f"word table overflow at {cap} slots for {nw} words")
        cap = min(cap * 4, full)
    ustart = torch.empty(min(cap, max(nw, 1)), dtype=torch.int32, device=dev)
    ulen = torch.empty_like(ustart)
    ucount = torch.empty(ustart.numel(), dtype=torch.int64, device=dev)
    upart = torch.empty(ustart.numel(), dtype=torch.int32, device=dev)
    counter = torch.zeros(1, dtype=torch.int32, device=dev)
    if nw:
        _call("hbmr_wc_compact", _ptr(buf), n, _ptr(tkeys), _ptr(tcounts), cap, int(R),
              _ptr(ustart), _ptr(ulen), _ptr(ucount), _ptr(upart), _ptr(counter), _st(stream))
    nu = int(counter)
    return ustart[:nu], ulen[:nu], ucount[:nu], upart[:nu]


def pack(buf, ustart, ulen, order=None, stream=None):
    """``b"w\\n"`` blob of the words (in ``order`` if given)."""
    nu = ustart.numel()
    sizes = (ulen if order is None else ulen[order]).to(torch.int64) + 1
    off = torch.zeros(nu, dtype=torch.int64, device=buf.device)
    if nu > 1:
        off[1:] = torch.cumsum(sizes, 0)[:-1]
    total = int(sizes.sum()) if nu else 0
    out = torch.empty(total, dtype=torch.uint8, device=buf.device)
    if nu:
        _call("hbmr_wc_pack", _ptr(buf), _ptr(ustart), _ptr(ulen),
              _ptr(None if order is None else order.contiguous()), nu, _ptr(off), _ptr(out),
              _st(stream))
    return out


def _aligned(buf):
    """The tokenizer reads 16-byte vectors: copy a misaligned view."""
    return buf if buf.data_ptr() % 16 == 0 else buf.clone()


def count_words(buf: torch.Tensor, stream=None):
    """Map + combine of one text split → (blob, counts)."""
    if buf.device.type != "cuda":
        return count_words_cpu(bytes(buf.numpy()))
    buf = _aligned(buf)
    starts, lens = tokenize(buf, stream)
    us, ul, uc, _ = aggregate(buf, starts, lens, None, 1, stream)
    return pack(buf, us, ul, None, stream), uc


def merge_tables(blob: torch.Tensor, counts: torch.Tensor, R: int = 1, stream=None):
    """Sum a concatenation of word tables.  Returns (blob, counts, part_bytes,
    part_words): the merged table with partition p's words contiguous, in
    partition order, and the per-partition byte / word counts (for the
    all-to-all-v of the shuffle)."""
    if blob.device.type != "cuda":
        return merge_tables_cpu(bytes(blob.numpy()), counts, R)
    blob = _aligned(blob)
    starts, lens = tokenize(blob, stream)
    if starts.numel() != counts.numel():
        raise ValueError(f"word table mismatch: {starts.numel()} words, {counts.numel()} counts")
    us, ul, uc, up = aggregate(blob, starts, lens, counts.contiguous(), R, stream)
    order = torch.argsort(up, stable=True)
    out = pack(blob, us, ul, order, stream)
    up_o = up[order].to(torch.int64)
    part_words = torch.bincount(up_o, minlength=R)
    part_bytes = torch.bincount(up_o, weights=(ul[order].to(torch.float64) + 1),
                                minlength=R).to(torch.int64)
    return out, uc[order], part_bytes.tolist(), part_words.tolist()


# --------------------------------------------------------------------------- CPU twins
def _table_from(counter):
    words = list(counter.keys())
    blob = b"".join(w + b"\n" for w in words)
    return (torch.frombuffer(bytearray(blob), dtype=torch.uint8) if blob else
            torch.empty(0, dtype=torch.uint8),
            torch.tensor([counter[w] for w in words], dtype=torch.int64))


def count_words_cpu(data: bytes):
    return _table_from(collections.Counter(data.split()))


def parse_table(blob: bytes, counts) -> list:
    words = blob.split(b"\n")[:-1] if blob else []
    cs = counts.tolist() if hasattr(counts, "tolist") else list(counts)
    if len(words) != len(cs):
        raise ValueError(f"word table mismatch: {len(words)} words, {len(cs)} counts")
    return list(zip(words, cs))


def partition_of(word: bytes, R: int) -> int:
    return (hash_bytes(word) & 0x7FFFFFFF) % R


def merge_tables_cpu(blob: bytes, counts, R: int = 1):
    c = collections.Counter()
    for w, n in parse_table(blob, counts):
        c[w] += int(n)
    parts = [[] for _ in range(R)]
    for w, n in c.items():
        parts[partition_of(w, R) if R > 1 else 0].append((w, n))
    words = [w for p in parts for w, _ in p]
    out = b"".join(w + b"\n" for w in words)
    blob_t = torch.frombuffer(bytearray(out), dtype=torch.uint8) if out else \
        torch.empty(0, dtype=torch.uint8)
    counts_t = torch.tensor([n for p in parts for _, n in p], dtype=torch.int64)
    return (blob_t, counts_t, [sum(len(w) + 1 for w, _ in p) for p in parts],
            [len(p) for p in parts])


def sorted_items(blob: torch.Tensor, counts: torch.Tensor) -> list:
    """(word, count) pairs in Text key order (unsigned lexicographic bytes)."""
    b = bytes(blob.cpu().numpy()) if blob.numel() else b""
    return sorted(parse_table(b, counts.cpu()))



