"""GPU sort / shuffle primitives (native/kernels/sort.hip) and their CPU twins.

* :func:`radix_sort_pairs` — stable LSD radix sort of uint64 keys (held in
  int64 tensors, compared unsigned) carrying uint32 values.
* TeraSort record ops: :func:`teragen` (Hadoop 1.0.3 TeraGen records bit for
  bit, on the device), :func:`tera_keys`, :func:`sort_records`,
  :func:`gather_records`, :func:`split_offsets`, :func:`count_unsorted`.

CPU versions (numpy) back CPU map slots and the tests' references; on a GPU
the native library must load (no silent fallback).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib

RECORD = 100
KEY = 10
# HBMR_TERA_SORT80=1: always the full 10-pass 80-bit key sort (A/B of the
# hi-only sort + tie fix-up)
_SORT80 = __import__("os").environ.get("HBMR_TERA_SORT80") == "1"


# TeraSort reduce v4: the radix sort covers hi >> TIE_SHIFT (the low bits of hi
# and lo are ordered by the in-place tie fix); HBMR_TERA_TIE_SHIFT overrides
TIE_SHIFT = int(os.environ.get("HBMR_TERA_TIE_SHIFT", "16"))
# bits of hi the v4 reduce radix-sorts below a group's common key prefix (the
# group is a key range: its splitters fix the top bits).  40 = 5 passes of 8
# bits: equal 40-bit prefixes come in pairs or triples among the ~2.5e8 keys of
# a group even for TeraGen's printable bytes (95 values of 256), ordered by the
# in-place tie fix — 0.229-0.231 s per 100 GB vs 0.237-0.242 s with 48 bits
# (profiles/r05_terasort_1gpu.json).  A 32-bit window leaves runs of equal
# prefixes longer than the tie fix takes and the group falls back to the
# full-key path: 0.76 s (profiles/r03_terasort_window.json)
SORT_BITS = int(os.environ.get("HBMR_TERA_SORT_BITS", "40"))


def sort_window(hi_range=None):
    """[begin, end) bits of hi the v4 reduce sorts.  Without a range: the top
    64 - TIE_SHIFT bits.  With the group's inclusive (low, high) hi bounds (as
    unsigned ints): the bits above their highest differing bit are the same in
    every key of the group, so the sort takes the SORT_BITS below that (ties on
    the sorted prefix are ordered by the full key afterwards)."""
    if hi_range is None or SORT_BITS <= 0:
        return TIE_SHIFT, 64
    lo, up = hi_range
    end = max(8, min(64, (int(lo) ^ int(up)).bit_length()))
    return max(0, end - SORT_BITS), end

def _ptr(t):
    return None if t is None else t.data_ptr()


def _on_gpu(t):
    return t.device.type == "cuda"


# --------------------------------------------------------------------------- radix sort
def radix_sort_pairs(keys: torch.Tensor, vals: torch.Tensor, begin_bit: int = 0,
                     end_bit: int = 64, stream=None) -> None:
    """In place: sort ``keys`` (int64 storage of uint64) and permute ``vals`` (int32)
    by key bits [begin_bit, end_bit).  Stable."""
    n = keys.numel()
    if vals.numel() != n or keys.dtype != torch.int64 or vals.dtype != torch.int32:
        raise ValueError("keys int64[n], vals int32[n] required")
    if n <= 1:
        return
    if not _on_gpu(keys):
        k = keys.numpy().view(np.uint64)
        mask = np.uint64(((1 << (end_bit - begin_bit)) - 1) if end_bit - begin_bit < 64
                         else 0xFFFFFFFFFFFFFFFF)
        dig = (k >> np.uint64(begin_bit)) & mask
        order = np.argsort(dig, kind="stable")
        keys.copy_(torch.from_numpy(k[order].view(np.int64).copy()))
        vals.copy_(vals[torch.from_numpy(order)])
        return
    lib = _lib.load()
    tk = torch.empty_like(keys)
    tv = torch.empty_like(vals)
    wsb = int(lib.hbmr_radix_sort_workspace_bytes(n))
    ws = torch.empty(wsb, dtype=torch.uint8, device=keys.device)
    rc = lib.hbmr_radix_sort_pairs_u64(_ptr(keys), _ptr(vals), _ptr(tk), _ptr(tv), n, begin_bit,
                                       end_bit, _ptr(ws), wsb, _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_radix_sort_pairs_u64")


ONESWEEP_MAX = 1 << 30
# per (device, stream): the onesweep look-back status words, zeroed once and
# tagged with a fresh epoch per pass (no memset before every pass), and the
# epoch counter the native side advances.  Calls on one stream run in order,
# so one status array per stream is never used by two sorts at once.
_ONESWEEP_STATUS: dict = {}


def _onesweep_status(device, nbytes, stream):
    key = (str(device), _lib.stream_handle(stream))
    ent = _ONESWEEP_STATUS.get(key)
    if ent is None or ent[0].numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        ent = _ONESWEEP_STATUS[key] = (buf, ctypes.c_uint(0))   # 0: zeroed on first use
    return ent


def radix_sort_keys(keys: torch.Tensor, begin_bit: int = 0, end_bit: int = 64, stream=None,
                    err: torch.Tensor | None = None, inplace: bool = True) -> torch.Tensor:
    """In place: sort ``keys`` (int64 storage of uint64) by bits [begin_bit,
    end_bit), keys only, stable — the onesweep kernels (one histogram read for
    every digit, a decoupled look-back scatter per digit).  ``err`` (int32[1],
    device) is set non-zero if a look-back timed out (the order check of the
    caller then fails); n < 2^30.  Returns the sorted tensor: ``keys``, or
    with ``inplace=False`` whichever of keys and its scratch twin the last
    pass wrote (no copy back after an odd number of passes)."""
    n = keys.numel()
    if keys.dtype != torch.int64:
        raise ValueError("keys int64[n] required")
    if n <= 1:
        return keys
    if not _on_gpu(keys):
        k = keys.numpy().view(np.uint64)
        w = end_bit - begin_bit
        mask = np.uint64((1 << w) - 1 if w < 64 else 0xFFFFFFFFFFFFFFFF)
        order = np.argsort((k >> np.uint64(begin_bit)) & mask, kind="stable")
        keys.copy_(torch.from_numpy(k[order].view(np.int64).copy()))
        return keys
    if n >= ONESWEEP_MAX:
        raise ValueError("onesweep radix sort: n must be below 2^30")
    lib = _lib.load()
    tk = torch.empty_like(keys)
    wsb = int(lib.hbmr_radix_onesweep_workspace_bytes(n))
    ws = torch.empty(wsb, dtype=torch.uint8, device=keys.device)
    if err is None:
        err = torch.zeros(1, dtype=torch.int32, device=keys.device)
    status, epoch = _onesweep_status(keys.device, int(lib.hbmr_radix_onesweep_status_bytes(n)),
                                     stream)
    rc = lib.hbmr_radix_sort_keys_u64(_ptr(keys), _ptr(tk), n, begin_bit, end_bit, _ptr(ws), wsb,
                                      _ptr(status), status.numel(), ctypes.byref(epoch),
                                      _ptr(err), int(inplace), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_radix_sort_keys_u64")
    passes = (end_bit - begin_bit + 7) // 8
    return tk if (not inplace and passes % 2) else keys


def argsort_u64(keys: torch.Tensor, stream=None):
    """(sorted keys, int32 permutation) without modifying ``keys``."""
    k = keys.clone()
    v = torch.arange(keys.numel(), dtype=torch.int32, device=keys.device)
    radix_sort_pairs(k, v, stream=stream)
    return k, v


# --------------------------------------------------------------------------- TeraGen
_A, _C, _M = 3141592621, 663896637, 0xFFFFFFFF


def _lcg_jump_np(steps: np.ndarray) -> np.ndarray:
    """State after ``steps`` LCG iterations from 0 (vectorised affine powering)."""
    steps = steps.astype(np.uint64)
    ra = np.ones_like(steps)
    rc = np.zeros_like(steps)
    ma = np.uint64(_A)
    mc = np.uint64(_C)
    m = np.uint64(_M)
    s = steps.copy()
    while s.any():
        bit = (s & np.uint64(1)).astype(bool)
        rc = np.where(bit, (ma * rc + mc) & m, rc)
        ra = np.where(bit, (ma * ra) & m, ra)
        mc = (ma * mc + mc) & m
        ma = (ma * ma) & m
        s >>= np.uint64(1)
    return rc  # x0 = 0


def teragen_keys_cpu(first_row: int, nrows: int) -> np.ndarray:
    """Only the 10-byte keys of TeraGen rows (uint8 [n, 10]), vectorised — what
    TeraSort's sampler reads (TeraInputFormat.java:101-141)."""
    rows = np.arange(first_row, first_row + nrows, dtype=np.int64)
    s = _lcg_jump_np(rows.astype(np.uint64) * np.uint64(3))
    kb = np.empty((nrows, 12), dtype=np.uint8)
    for q in range(3):
        s = (np.uint64(_A) * s + np.uint64(_C)) & np.uint64(_M)
        temp = s // np.uint64(52)
        for pos in (3, 2, 1, 0):
            kb[:, pos + 4 * q] = (32 + temp % np.uint64(95)).astype(np.uint8)
            temp = temp // np.uint64(95)
    return kb[:, :10].copy()


def teragen_cpu(first_row: int, nrows: int) -> np.ndarray:
    """Reference TeraGen (TeraGen.java RandomGenerator / SortGenMapper) → uint8 [n, 100]."""
    rows = np.arange(first_row, first_row + nrows, dtype=np.int64)
    out = np.empty((nrows, RECORD), dtype=np.uint8)
    s = _lcg_jump_np(rows.astype(np.uint64) * np.uint64(3))
    kb = np.empty((nrows, 12), dtype=np.uint8)
    for q in range(3):
        s = (np.uint64(_A) * s + np.uint64(_C)) & np.uint64(_M)
        temp = s // np.uint64(52)
        for pos in (3, 2, 1, 0):
            kb[:, pos + 4 * q] = (32 + temp % np.uint64(95)).astype(np.uint8)
            temp = temp // np.uint64(95)
    out[:, :10] = kb[:, :10]
    rid = rows.astype(np.int32)   # Java (int) rowId
    for i in range(nrows):
        t = str(int(rid[i])).encode()[:10]
        out[i, 10:20] = np.frombuffer(b" " * (10 - len(t)) + t, dtype=np.uint8)
    fb = (rows * 8) % 26
    for q in range(7):
        out[:, 20 + 10 * q:30 + 10 * q] = (65 + (fb + q) % 26).astype(np.uint8)[:, None]
    out[:, 90:98] = (65 + (fb + 7) % 26).astype(np.uint8)[:, None]
    out[:, 98] = 13
    out[:, 99] = 10
    return out


def teragen(first_row: int, nrows: int, device="cuda", stream=None) -> torch.Tensor:
    dev = torch.device(device)
    if dev.type != "cuda":
        return torch.from_numpy(teragen_cpu(first_row, nrows))
    out = torch.empty(nrows, RECORD, dtype=torch.uint8, device=dev)
    rc = _lib.load().hbmr_teragen(first_row, nrows, _ptr(out), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_teragen")
    return out


# --------------------------------------------------------------------------- records
def tera_keys(records: torch.Tensor, stream=None):
    """(hi, lo) int64 tensors: key bytes 0-7 and 8-9 as big-endian unsigned ints."""
    n, stride = records.shape
    if _on_gpu(records):
        hi = torch.empty(n, dtype=torch.int64, device=records.device)
        lo = torch.empty(n, dtype=torch.int64, device=records.device)
        rc = _lib.load().hbmr_tera_keys(_ptr(records), n, stride, _ptr(hi), _ptr(lo),
                                         _lib.stream_handle(stream))
        _lib.check(rc, "hbmr_tera_keys")
        return hi, lo
    r = records.numpy()
    hi = np.zeros(n, dtype=np.uint64)
    for j in range(8):
        hi = (hi << np.uint64(8)) | r[:, j].astype(np.uint64)
    lo = (r[:, 8].astype(np.uint64) << np.uint64(8)) | r[:, 9].astype(np.uint64)
    return torch.from_numpy(hi.view(np.int64)), torch.from_numpy(lo.view(np.int64))


def gather_records(records: torch.Tensor, perm: torch.Tensor, stream=None) -> torch.Tensor:
    n, rb = records.shape
    if not _on_gpu(records):
        return records[perm.long()]
    out = torch.empty_like(records)
    rc = _lib.load().hbmr_gather_records(_ptr(records), _ptr(perm), n, rb, _ptr(out),
                                          _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_gather_records")
    return out


def sort_keys(hi: torch.Tensor, lo: torch.Tensor, stream=None):
    """Permutation ordering records by (hi, lo) unsigned; returns (perm, hi_sorted, lo_sorted)."""
    n = hi.numel()
    if not _on_gpu(hi):
        h = hi.numpy().view(np.uint64)
        lw = lo.numpy().view(np.uint64)
        order = np.lexsort((lw, h)).astype(np.int32)
        return (torch.from_numpy(order), torch.from_numpy(h[order].view(np.int64).copy()),
                torch.from_numpy(lw[order].view(np.int64).copy()))
    lib = _lib.load()
    if not _SORT80:
        # 8 passes over hi only, lo gathered, then runs of equal hi (rare: hi
        # holds 8 of the 10 key bytes) ordered by lo in place; a run longer
        # than the fix-up handles falls back to the full 80-bit sort below
        perm = torch.arange(n, dtype=torch.int32, device=hi.device)
        hi_k = hi.clone()
        radix_sort_pairs(hi_k, perm, 0, 64, stream=stream)
        lo_s = torch.empty_like(lo)
        rc = lib.hbmr_gather_u64(_ptr(lo), _ptr(perm), n, _ptr(lo_s), _lib.stream_handle(stream))
        _lib.check(rc, "hbmr_gather_u64")
        flag = torch.zeros(1, dtype=torch.int32, device=hi.device)
        rc = lib.hbmr_tera_tie_fix(_ptr(hi_k), _ptr(lo_s), _ptr(perm), n, _ptr(flag),
                                   _lib.stream_handle(stream))
        _lib.check(rc, "hbmr_tera_tie_fix")
        if not int(flag.item()):
            return perm, hi_k, lo_s
        del perm, hi_k, lo_s
    # LSD: 2 passes over the low 16 bits, then 8 over the high 64 (stable)
    lo_k = lo.clone()
    perm = torch.arange(n, dtype=torch.int32, device=hi.device)
    radix_sort_pairs(lo_k, perm, 0, 16, stream=stream)
    hi_k = torch.empty_like(hi)
    rc = lib.hbmr_gather_u64(_ptr(hi), _ptr(perm), n, _ptr(hi_k), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_gather_u64")
    radix_sort_pairs(hi_k, perm, 0, 64, stream=stream)
    lo_s = torch.empty_like(lo)
    rc = lib.hbmr_gather_u64(_ptr(lo), _ptr(perm), n, _ptr(lo_s), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_gather_u64")
    return perm, hi_k, lo_s


def sort_records(records: torch.Tensor, stream=None):
    """Sort 100-byte records by their 10-byte key → (sorted records, hi, lo)."""
    hi, lo = tera_keys(records, stream=stream)
    perm, hs, ls = sort_keys(hi, lo, stream=stream)
    return gather_records(records, perm, stream=stream), hs, ls


def split_offsets(hi: torch.Tensor, lo: torch.Tensor, split_hi: torch.Tensor,
                  split_lo: torch.Tensor, stream=None) -> torch.Tensor:
    """For sorted (hi, lo): offsets[R+1] of the R range partitions defined by the
    R-1 splitters (partition p holds keys in [split[p-1], split[p]))."""
    n = hi.numel()
    nparts = split_hi.numel() + 1
    if not _on_gpu(hi):
        h = hi.numpy().view(np.uint64)
        lw = lo.numpy().view(np.uint64)
        sh = split_hi.numpy().view(np.uint64)
        sl = split_lo.numpy().view(np.uint64)
        out = np.zeros(nparts + 1, dtype=np.int64)
        out[nparts] = n
        for p in range(1, nparts):
            a, b = 0, n
            while a < b:
                m = (a + b) // 2
                if h[m] < sh[p - 1] or (h[m] == sh[p - 1] and lw[m] < sl[p - 1]):
                    a = m + 1
                else:
                    b = m
            out[p] = a
        return torch.from_numpy(out)
    out = torch.empty(nparts + 1, dtype=torch.int64, device=hi.device)
    rc = _lib.load().hbmr_split_offsets(_ptr(hi), _ptr(lo), n, _ptr(split_hi), _ptr(split_lo),
                                         nparts, _ptr(out), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_split_offsets")
    return out


def count_unsorted(hi: torch.Tensor, lo: torch.Tensor, stream=None) -> int:
    """Number of adjacent out-of-order key pairs (TeraValidate's check)."""
    n = hi.numel()
    if n <= 1:
        return 0
    if not _on_gpu(hi):
        h = hi.numpy().view(np.uint64)
        lw = lo.numpy().view(np.uint64)
        bad = (h[:-1] > h[1:]) | ((h[:-1] == h[1:]) & (lw[:-1] > lw[1:]))
        return int(bad.sum())
    bad = torch.zeros(1, dtype=torch.int64, device=hi.device)
    rc = _lib.load().hbmr_check_sorted(_ptr(hi), _ptr(lo), n, _ptr(bad),
                                        _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_check_sorted")
    return int(bad.item())


def keys_from_bytes(keys: list) -> tuple[torch.Tensor, torch.Tensor]:
    """10-byte keys (bytes) → (hi, lo) int64 tensors (host)."""
    hi = np.array([int.from_bytes(k[:8].ljust(8, b"\0"), "big") for k in keys], dtype=np.uint64)
    lo = np.array([int.from_bytes(k[8:10].ljust(2, b"\0"), "big") for k in keys], dtype=np.uint64)
    return torch.from_numpy(hi.view(np.int64)), torch.from_numpy(lo.view(np.int64))


# --------------------------------------------------------------------------- range-partitioned TeraSort
def tera_keys_part(records: torch.Tensor, split_hi: torch.Tensor, split_lo: torch.Tensor,
                   stream=None):
    """(hi, lo, pid) of every record: key words and its range partition (the
    number of splitters <= key; splitters sorted, at most 4096)."""
    n, stride = records.shape
    ns = split_hi.numel()
    if _on_gpu(records):
        if ns > 4096:
            raise ValueError("at most 4096 splitters (4097 partitions)")
        hi = torch.empty(n, dtype=torch.int64, device=records.device)
        lo = torch.empty(n, dtype=torch.int64, device=records.device)
        pid = torch.empty(n, dtype=torch.int64, device=records.device)
        sh = split_hi.to(records.device)
        sl = split_lo.to(records.device)
        rc = _lib.load().hbmr_tera_keys_part(_ptr(records), n, stride, _ptr(sh) if ns else None,
                                              _ptr(sl) if ns else None, ns, _ptr(hi), _ptr(lo),
                                              _ptr(pid), _lib.stream_handle(stream))
        _lib.check(rc, "hbmr_tera_keys_part")
        return hi, lo, pid
    hi, lo = tera_keys(records)
    h = hi.numpy().view(np.uint64)
    lw = lo.numpy().view(np.uint64)
    sh = split_hi.numpy().view(np.uint64)
    sl = split_lo.numpy().view(np.uint64)
    # pid = #splitters <= key (lexicographic (hi, lo))
    pid = np.searchsorted(sh, h, side="left").astype(np.int64)
    for j in range(ns):      # ties on hi: decide by lo
        tie = h == sh[j]
        pid[tie & (lw >= sl[j])] = np.maximum(pid[tie & (lw >= sl[j])], j + 1)
    return hi, lo, torch.from_numpy(pid)


_SPLITTERS_DEV: dict = {}


def _splitters_on(dev, split_hi, split_lo):
    """(hi, lo) of a job's splitters on ``dev``, uploaded once per splitter
    set (every map of a job partitions by the same ones)."""
    if split_hi.device == dev:
        return split_hi, split_lo
    hb = split_hi.numpy().tobytes()
    key = (str(dev), hb, split_lo.numpy().tobytes())
    got = _SPLITTERS_DEV.get(key)
    if got is None:
        if len(_SPLITTERS_DEV) > 16:
            _SPLITTERS_DEV.clear()
        got = _SPLITTERS_DEV[key] = tuple(
            t.pin_memory().to(dev, non_blocking=True) for t in (split_hi, split_lo))
    return got


def tera_partition(records: torch.Tensor, split_hi: torch.Tensor, split_lo: torch.Tensor,
                   stream=None, kbytes=False):
    """Range-partition a split: (hi, lo, row, offsets) — key words and record
    numbers in partition order (order inside a partition unspecified) and
    offsets[R+1] of the R = #splitters + 1 partitions (int64, on the records'
    device).  On the GPU: one key/partition/count kernel, an on-device scan and
    one tile-ranked scatter (no sort, no gathers).  ``kbytes``: also an
    int64[2] on the device — the OR of every key's high-word bytes (the key
    alphabet [0, 2^bits(OR)) the reduce's dense window needs) and the split's
    key checksum sum(hi + lo) mod 2^64."""
    n, stride = records.shape
    ns = split_hi.numel()
    nparts = ns + 1
    if not _on_gpu(records):
        hi, lo, pid = tera_keys_part(records, split_hi, split_lo)
        order = torch.from_numpy(np.argsort(pid.numpy(), kind="stable"))
        counts = torch.bincount(pid, minlength=nparts)
        offs = torch.zeros(nparts + 1, dtype=torch.int64)
        torch.cumsum(counts, 0, out=offs[1:])
        if kbytes:
            orb = int(np.bitwise_or.reduce(records[:, :8].numpy(), axis=None)) if n else 0
            kmm = torch.stack([torch.tensor(orb, dtype=torch.int64), hi.sum() + lo.sum()])
            return hi[order], lo[order], order.to(torch.int32), offs, kmm
        return hi[order], lo[order], order.to(torch.int32), offs
    if ns > 4096:
        raise ValueError("at most 4096 splitters (4097 partitions)")
    dev = records.device
    lib = _lib.load()
    hi = torch.empty(n, dtype=torch.int64, device=dev)
    lo = torch.empty(n, dtype=torch.int64, device=dev)
    row = torch.empty(n, dtype=torch.int32, device=dev)
    offs = torch.empty(nparts + 1, dtype=torch.int64, device=dev)
    wsb = int(lib.hbmr_tera_partition_workspace_bytes(n, nparts))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    sh, sl = _splitters_on(dev, split_hi, split_lo)
    kmm = torch.zeros(2, dtype=torch.int64, device=dev) if kbytes else None
    rc = lib.hbmr_tera_partition(_ptr(records), n, stride, _ptr(sh) if ns else None,
                                 _ptr(sl) if ns else None, ns, _ptr(hi), _ptr(lo), _ptr(row),
                                 _ptr(offs), _ptr(kmm), _ptr(ws), wsb, _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_tera_partition")
    if kbytes:
        return hi, lo, row, offs, kmm
    return hi, lo, row, offs


def merge_runs(runs, stream=None):
    """K8: merge sorted runs [(hi, lo, val)] (keys uint64 in int64 storage, val
    int32; each run sorted by (hi, lo)) into one sorted (hi, lo, val) — a
    pairwise merge-path tree, log2(#runs) passes; stable (earlier runs first
    on equal keys)."""
    runs = [r for r in runs if r[0].numel()]
    if not runs:
        return (torch.empty(0, dtype=torch.int64), torch.empty(0, dtype=torch.int64),
                torch.empty(0, dtype=torch.int32))
    if not _on_gpu(runs[0][0]):
        h = torch.cat([r[0] for r in runs]).numpy().view(np.uint64)
        lw = torch.cat([r[1] for r in runs]).numpy().view(np.uint64)
        v = torch.cat([r[2] for r in runs])
        order = np.lexsort((np.arange(h.size), lw, h))     # stable: run order on ties
        o = torch.from_numpy(order)
        return (torch.from_numpy(h[order].view(np.int64).copy()),
                torch.from_numpy(lw[order].view(np.int64).copy()), v[o])
    lib = _lib.load()
    while len(runs) > 1:
        nxt = []
        for i in range(0, len(runs) - 1, 2):
            (ah, al, av), (bh, bl, bv) = runs[i], runs[i + 1]
            n = ah.numel() + bh.numel()
            oh = torch.empty(n, dtype=torch.int64, device=ah.device)
            ol = torch.empty(n, dtype=torch.int64, device=ah.device)
            ov = torch.empty(n, dtype=torch.int32, device=ah.device)
            rc = lib.hbmr_merge_path(_ptr(ah), _ptr(al), _ptr(av), ah.numel(), _ptr(bh), _ptr(bl),
                                     _ptr(bv), bh.numel(), _ptr(oh), _ptr(ol), _ptr(ov),
                                     _lib.stream_handle(stream))
            _lib.check(rc, "hbmr_merge_path")
            nxt.append((oh, ol, ov))
        if len(runs) % 2:
            nxt.append(runs[-1])
        runs = nxt
    return runs[0]


_PTR_TABLES: dict = {}


def _h2d_i64(values, device):
    """int64 values on the device without a blocking copy: a pinned staging
    tensor and an asynchronous copy on the current stream (a pageable copy
    waits for the device to drain everything queued before it)."""
    h = torch.as_tensor(np.asarray(values, dtype=np.int64))
    if device.type != "cuda":
        return h.to(device)
    return h.pin_memory().to(device, non_blocking=True)


def _ptr_table(ts, device):
    """Device table of the tensors' base addresses, cached by the addresses
    (a TeraSort reduce passes the same map outputs for every group)."""
    key = (str(device), tuple(t.data_ptr() for t in ts))
    tab = _PTR_TABLES.get(key)
    if tab is None:
        if len(_PTR_TABLES) > 64:
            _PTR_TABLES.clear()
        tab = _PTR_TABLES[key] = _h2d_i64(key[1], device)
    return tab


def tera_collect(his, los, rows, starts, lens, with_keys=True, stream=None):
    """Concatenate pieces [starts[s], starts[s]+lens[s]) of per-split (hi, lo,
    row) arrays → (hi, lo, split, row) (hi/lo None unless ``with_keys``)."""
    S = len(rows)
    n = int(sum(lens))
    dev = rows[0].device
    if not _on_gpu(rows[0]):
        sel = [slice(int(a), int(a) + int(m)) for a, m in zip(starts, lens)]
        split = torch.cat([torch.full((int(m),), s, dtype=torch.int32) for s, m in enumerate(lens)])
        row = torch.cat([r[sl] for r, sl in zip(rows, sel)])
        if not with_keys:
            return None, None, split, row
        return (torch.cat([h[sl] for h, sl in zip(his, sel)]),
                torch.cat([lw[sl] for lw, sl in zip(los, sel)]), split, row)
    prefix = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(np.asarray(lens, dtype=np.int64), out=prefix[1:])
    meta = _h2d_i64(np.concatenate([np.asarray(starts, dtype=np.int64), prefix]), dev)
    split = torch.empty(n, dtype=torch.int32, device=dev)
    row = torch.empty(n, dtype=torch.int32, device=dev)
    ohi = torch.empty(n, dtype=torch.int64, device=dev) if with_keys else None
    olo = torch.empty(n, dtype=torch.int64, device=dev) if with_keys else None
    th = _ptr_table(his, dev) if with_keys else None
    tl = _ptr_table(los, dev) if with_keys else None
    tr = _ptr_table(rows, dev)
    rc = _lib.load().hbmr_tera_collect(_ptr(th), _ptr(tl), _ptr(tr), _ptr(meta),
                                        _ptr(meta) + 8 * S, S, n, _ptr(ohi), _ptr(olo),
                                        _ptr(split), _ptr(row), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_tera_collect")
    return ohi, olo, split, row


NO_SPLIT = 0xFFFFFFFF


def tera_collect_slots(rows, starts: torch.Tensor, pre: torch.Tensor, cap: int, stream=None):
    """Static-shape shuffle send layout: (split, row) int32 [W * cap] — slot d
    holds destination d's pieces in split order (piece s = rows[s][starts[s, d]
    + i] for i < pre[d, s+1] - pre[d, s], at pre[d, s] + i), entries past
    min(pre[d, S], cap) carry split = NO_SPLIT (gather_records_multi leaves
    those records unwritten).  ``starts`` [S, W] and ``pre`` [W, S+1] (int64)
    stay on the device: nothing here waits for the maps that produced them."""
    S = len(rows)
    W = pre.shape[0]
    dev = rows[0].device
    if not _on_gpu(rows[0]):
        split = torch.full((W * cap,), -1, dtype=torch.int32)   # NO_SPLIT's bits
        row = torch.zeros(W * cap, dtype=torch.int32)
        st, pr = starts.tolist(), pre.tolist()
        for d in range(W):
            for s in range(S):
                a, b = pr[d][s], min(pr[d][s + 1], cap)
                if b <= a:
                    continue
                split[d * cap + a:d * cap + b] = s
                row[d * cap + a:d * cap + b] = rows[s][st[s][d]:st[s][d] + (b - a)]
        return split, row
    split = torch.empty(W * cap, dtype=torch.int32, device=dev)
    row = torch.empty(W * cap, dtype=torch.int32, device=dev)
    starts = starts.to(dev, torch.int64).contiguous()
    pre = pre.to(dev, torch.int64).contiguous()
    tr = _ptr_table(rows, dev)
    rc = _lib.load().hbmr_tera_collect_slots(_ptr(tr), _ptr(starts), _ptr(pre), S, W, cap,
                                              _ptr(split), _ptr(row), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_tera_collect_slots")
    return split, row


GID_MAX_SPLITS = 256
GID_MAX_ROWS = 1 << 24


PACK_GROUP_MAX = 1 << 24  # records per packed-key group: bounds the tie runs of a 32-bit window


class KeyWindow:
    """The order-preserving dense map of a key's high word h used by the
    packed reduce (native KeyWindow): v(h) = h's 8 bytes as base-R digits
    (every key byte in [m, m + R)), window = (v(h) - vlo) >> sh.  For a group
    with keys' v in [vlo, vup] (its splitters), sh makes the window fit in 32
    bits.  m = 0, R = 256, vlo = 0 is the plain shift h >> sh."""

    def __init__(self, m=0, R=256, vlo=0, sh=0):
        self.m, self.R, self.vlo, self.sh = int(m), int(R), int(vlo), int(sh)

    def v(self, h: int) -> int:
        x = 0
        for b in range(7, -1, -1):
            x = x * self.R + (((h >> (8 * b)) & 0xFF) - self.m)
        return x

    @classmethod
    def for_group(cls, m, R, lo_hi=None, up_hi=None, bits=32):
        """lo_hi / up_hi: the group's bounding splitter high words (None: the
        first / last group — the alphabet's ends)."""
        w = cls(m, R)
        vlo = 0 if lo_hi is None else w.v(int(lo_hi))
        vup = R ** 8 - 1 if up_hi is None else w.v(int(up_hi))
        span = max(1, vup - vlo + 1)
        return cls(m, R, vlo, max(0, span.bit_length() - bits))

    def apply_np(self, h: np.ndarray) -> np.ndarray:
        v = np.zeros(h.shape, dtype=np.uint64)
        for b in range(7, -1, -1):
            d = ((h >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.int64) - self.m
            v = v * np.uint64(self.R) + d.astype(np.uint64)
        return (v - np.uint64(self.vlo & 0xFFFFFFFFFFFFFFFF)) >> np.uint64(self.sh)


def tera_collect_gid(his, rows, starts, lens, stream=None, window: KeyWindow | None = None):
    """Pieces [starts[s], +lens[s]) of per-split (hi, row) arrays → (hi, gid)
    with gid = s << 24 | row (int32 storage): the record ids the v4 reduce
    sorts and gathers by (at most 256 splits of < 2^24 records).  With
    ``window``: (packed, None) — one sortable int64 per record, the key's
    32-bit window above the record's id."""
    S = len(rows)
    if S > GID_MAX_SPLITS:
        raise ValueError(f"at most {GID_MAX_SPLITS} map outputs per packed-id collect")
    n = int(sum(lens))
    dev = rows[0].device
    if not _on_gpu(rows[0]):
        sel = [slice(int(a), int(a) + int(m)) for a, m in zip(starts, lens)]
        gid = torch.cat([(r[sl].to(torch.int64) | (s << 24)).to(torch.int32)
                         for s, (r, sl) in enumerate(zip(rows, sel))])
        hi = torch.cat([h[sl] for h, sl in zip(his, sel)])
        if window is None:
            return hi, gid
        w = window.apply_np(hi.numpy().view(np.uint64)) & np.uint64(0xFFFFFFFF)
        pk = (w << np.uint64(32)) | gid.numpy().view(np.uint32).astype(np.uint64)
        return torch.from_numpy(pk.view(np.int64).copy()), None
    prefix = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(np.asarray(lens, dtype=np.int64), out=prefix[1:])
    meta = _h2d_i64(np.concatenate([np.asarray(starts, dtype=np.int64), prefix]), dev)
    ohi = torch.empty(n, dtype=torch.int64, device=dev)
    gid = None if window is not None else torch.empty(n, dtype=torch.int32, device=dev)
    th, tr = _ptr_table(his, dev), _ptr_table(rows, dev)
    kw = window or KeyWindow()
    rc = _lib.load().hbmr_tera_collect_gid(_ptr(th), _ptr(tr), _ptr(meta), _ptr(meta) + 8 * S, S,
                                            n, int(window is not None),
                                            kw.vlo & 0xFFFFFFFFFFFFFFFF, kw.m, kw.R, kw.sh,
                                            _ptr(ohi), _ptr(gid), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_tera_collect_gid")
    return ohi, gid


def gather_records_gid(bases, gid: torch.Tensor, stream=None, keys=None,
                       win: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = bases[g >> 24][g & 0xFFFFFF] (100-byte records) with g =
    gid[i]: int32 ids, or int64 packed keys whose low 32 bits are the ids.
    ``keys`` = (hi, lo) int64 [n] tensors also receive the gathered records'
    keys (as tera_keys would read them back), on the GPU in the same pass; hi
    may be the packed keys themselves (each record's id is read before its
    key is written over it).  ``win`` (int32 [n], packed ids only) receives
    each record's sort window (the packed key's high half) for the tie fix."""
    n = gid.numel()
    rb = bases[0].shape[1]
    packed = gid.dtype == torch.int64
    if not _on_gpu(gid):
        g = gid.to(torch.int64) & 0xFFFFFFFF
        s, r = g >> 24, g & 0xFFFFFF
        res = torch.empty(n, rb, dtype=torch.uint8)
        for j, b in enumerate(bases):
            m = s == j
            if m.any():
                res[m] = b[r[m]]
        if keys is not None:
            h, lo = tera_keys(res)
            keys[0].copy_(h)
            keys[1].copy_(lo)
        return res
    res = torch.empty(n, rb, dtype=torch.uint8, device=gid.device)
    tb = _ptr_table(bases, gid.device)
    kh, kl = keys if keys is not None else (None, None)
    rc = _lib.load().hbmr_gather_records_gid(_ptr(tb), None if packed else _ptr(gid),
                                              _ptr(gid) if packed else None, n, rb, _ptr(res),
                                              _ptr(kh), _ptr(kl), _ptr(win),
                                              _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_gather_records_gid")
    return res


def sort_gathered(his, rows, starts, lens, bases, stream=None, hi_range=None, defer=False,
                  alphabet=None, bounds=None):
    """TeraSort reduce v4 for one group: (hi, gid) collect, radix passes over
    a window of hi, ONE record gather, the low key words read back from the
    sorted records, and runs of an equal sorted prefix ordered by the full key
    in place.  Returns (records, hi, lo), or None when such a run is too long
    for the in-place fix-up (the caller takes the full-key path).
    ``hi_range`` (the group's hi bounds) places the window just below the
    group's common prefix.

    Groups below PACK_GROUP_MAX records, given the job's key ``alphabet``
    (m, R) and the group's splitter high words ``bounds`` (lo, up; None at
    the ends), sort packed keys — the key's dense 32-bit window (KeyWindow)
    above the 32-bit record id in one int64, keys only, by the onesweep
    kernels: 4 passes of 8 bytes per record and one histogram read, against 5
    passes of 12 bytes plus a histogram read each for (hi, gid) pairs over 40
    bits.  Equal windows (well under 1 % of a 12M-record group) are ordered
    by the tie fix.  Otherwise the pairs.

    ``defer``: no host read — returns (records, hi, lo, flag) with flag a
    device int32[1] the caller checks once for all groups (non-zero: this
    group's order is not final and must be redone on the full-key path)."""
    n = int(sum(lens))
    begin, end = sort_window(hi_range)
    kw = KeyWindow(sh=begin)
    if n < PACK_GROUP_MAX and alphabet is not None and bounds is not None:
        lo_b, up_b = bounds
        if (lo_b is None or up_b is None) and n:
            # an end group: its own smallest / largest high word bound the
            # window (the alphabet's ends would widen it many times over)
            # (uint64 order through int64: flip the sign bit both ways)
            pieces = [h[int(a):int(a) + int(m)] ^ _SIGN for h, a, m in zip(his, starts, lens)
                      if int(m)]
            mm = torch.stack([torch.stack([p.min(), p.max()]) for p in pieces]) ^ _SIGN
            if _on_gpu(mm):
                mm = mm.cpu()
            mu = mm.numpy().view(np.uint64)
            lo_b = int(mu[:, 0].min()) if lo_b is None else lo_b
            up_b = int(mu[:, 1].max()) if up_b is None else up_b
        kw = KeyWindow.for_group(alphabet[0], alphabet[1], lo_b, up_b)
        h, _ = tera_collect_gid(his, rows, starts, lens, stream=stream, window=kw)
        radix_sort_keys(h, 32, 64, stream=stream)
        lo = torch.empty_like(h)
        win = torch.empty(n, dtype=torch.int32, device=h.device) if _on_gpu(h) else None
        # each record's id is read from its packed word before the gather
        # writes the record's full hi key over it (and its window into win)
        recs = gather_records_gid(bases, h, stream=stream, keys=(h, lo), win=win)
    else:
        win = None
        h, gid = tera_collect_gid(his, rows, starts, lens, stream=stream)
        radix_sort_pairs(h, gid, begin, end, stream=stream)
        # the sorted keys come with the gather (lo is new; h is rewritten with
        # the same values): no second pass over the records
        lo = torch.empty_like(h)
        recs = gather_records_gid(bases, gid, stream=stream, keys=(h, lo))
        del gid
    if not _on_gpu(recs):
        order = np.lexsort((lo.numpy().view(np.uint64), h.numpy().view(np.uint64)))
        o = torch.from_numpy(order)
        if defer:
            return recs[o], h[o], lo[o], torch.zeros(1, dtype=torch.int32)
        return recs[o], h[o], lo[o]
    flag = torch.zeros(1, dtype=torch.int32, device=recs.device)
    lib = _lib.load()
    # moved records of the tie runs go through a compact scratch: room for a
    # quarter of the group (a few percent move with a 32-bit window)
    cap = max(4096, recs.shape[0] // 4)
    scratch = torch.empty(int(lib.hbmr_tera_tie_fix_scratch_bytes(cap, recs.shape[1])),
                          dtype=torch.uint8, device=recs.device)
    rc = lib.hbmr_tera_tie_fix_records(_ptr(h), _ptr(lo), _ptr(recs), recs.shape[0],
                                       recs.shape[1], kw.vlo & 0xFFFFFFFFFFFFFFFF, kw.m, kw.R,
                                       kw.sh, _ptr(win), _ptr(flag), _ptr(scratch), cap,
                                       _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_tera_tie_fix_records")
    if defer:
        return recs, h, lo, flag
    if int(flag.item()):
        return None
    return recs, h, lo


def gather_records_multi(bases, split: torch.Tensor, row: torch.Tensor, perm=None,
                         out=None, stream=None) -> torch.Tensor:
    """out[i] = bases[split[k]][row[k]], k = perm[i] (or i): 100-byte records
    gathered from several split tensors in one pass."""
    n = split.numel()
    rb = bases[0].shape[1]
    if not _on_gpu(split):
        k = perm.long() if perm is not None else torch.arange(n)
        s, r = split[k].long(), row[k].long()
        res = torch.empty(n, rb, dtype=torch.uint8) if out is None else out
        for j, b in enumerate(bases):
            m = s == j
            if m.any():
                res[m] = b[r[m]]
        return res
    res = torch.empty(n, rb, dtype=torch.uint8, device=split.device) if out is None else out
    tb = _ptr_table(bases, split.device)
    rc = _lib.load().hbmr_gather_records_multi(_ptr(tb), _ptr(split), _ptr(row), _ptr(perm), n, rb,
                                                _ptr(res), _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_gather_records_multi")
    return res


def gather_u64(src: torch.Tensor, perm: torch.Tensor, stream=None) -> torch.Tensor:
    """dst[i] = src[perm[i]] for int64 storage (perm int32)."""
    if not _on_gpu(src):
        return src[perm.long()]
    dst = torch.empty(perm.numel(), dtype=src.dtype, device=src.device)
    rc = _lib.load().hbmr_gather_u64(_ptr(src), _ptr(perm), perm.numel(), _ptr(dst),
                                      _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_gather_u64")
    return dst


def count_unsorted_dev(hi: torch.Tensor, lo: torch.Tensor, stream=None) -> torch.Tensor:
    """count_unsorted as a 0-d int64 device tensor (no host sync)."""
    n = hi.numel()
    if n <= 1 or not _on_gpu(hi):
        return torch.tensor(count_unsorted(hi, lo), dtype=torch.int64, device=hi.device)
    bad = torch.zeros(1, dtype=torch.int64, device=hi.device)
    rc = _lib.load().hbmr_check_sorted(_ptr(hi), _ptr(lo), n, _ptr(bad),
                                        _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_check_sorted")
    return bad[0]


_SIGN = -0x8000000000000000
GROUP_STATS_LEN = 2 + 2 * 1024


def tera_group_stats(hi: torch.Tensor, lo: torch.Tensor, prev, acc: torch.Tensor, stream=None):
    """acc[:2] (int64[GROUP_STATS_LEN], the keys' device; the rest is the
    kernel's scratch) += (records out of order — record 0 against ``prev``,
    the previous group's last (hi, lo) 1-element tensors, or None — and
    sum(hi + lo) mod 2^64), with no host read."""
    n = hi.numel()
    if n == 0:
        return
    if not _on_gpu(hi):
        bad = count_unsorted(hi, lo)
        if prev is not None:
            bad += int(pair_greater(prev, (hi[:1], lo[:1])))
        s = (hi.sum() + lo.sum()).reshape(())
        acc[:2] += torch.stack([torch.tensor(bad, dtype=torch.int64), s])
        return
    ph, pl = (prev[0], prev[1]) if prev is not None else (None, None)
    rc = _lib.load().hbmr_tera_group_stats(_ptr(hi), _ptr(lo), n, _ptr(ph), _ptr(pl), _ptr(acc),
                                            _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_tera_group_stats")


def pair_greater(a, b) -> torch.Tensor:
    """1 if key a > key b (a, b: (hi, lo) 1-element int64 tensors holding uint64),
    as a 0-d int64 tensor on their device (no host sync)."""
    ah, al = a[0] ^ _SIGN, a[1]
    bh, bl = b[0] ^ _SIGN, b[1]
    return ((ah > bh) | ((ah == bh) & (al > bl))).to(torch.int64).reshape(())
