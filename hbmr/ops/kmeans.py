"""K-Means map/combine/reduce ops on MI355X (HIP kernels in native/kernels/kmeans.hip).

Data layout contract (built by :class:`hbmr.gpu.split_cache.SplitCache`):

* points: ``bf16 [n, dp]`` with ``dp`` in {64, 128, 256} (feature dim zero-padded),
* centroids: fp32 master copy ``[k, d]`` plus a bf16 image ``[k_pad, dp]`` and
  ``chalf = -||c||²/2`` (fp32, ``[k_pad]``); padded clusters carry -1e30 so they
  never win the arg-max,
* partial sums: **int64 fixed point** ``[k, dp]`` (``Σ round(x·2^fx_shift)``) and
  int64 counts ``[k]`` — exact and order-independent, so K-Means results are
  bitwise reproducible for any placement of map tasks over CPUs/GPUs and any
  GPU count (integer RCCL all-reduce is exact too).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from . import _lib
from ..utils.trace import TRACE

SUPPORTED_DP = (64, 128, 256)


def _nullctx():
    import contextlib
    return contextlib.nullcontext()
FX_SHIFT = 24  # fixed-point fraction bits of the partial sums
# exact mode's Elkan scan: neighbours listed per centroid (past them the scan
# checks every centroid); HBMR_KMEANS_NBR_L overrides
NBR_L = 256


def padded_dim(d: int) -> int:
    for dp in SUPPORTED_DP:
        if d <= dp:
            return dp
    raise ValueError(f"feature dim {d} > {SUPPORTED_DP[-1]} not supported by the MFMA kernel")


def padded_k(k: int) -> int:
    return ((k + 63) // 64) * 64


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def new_partials(k: int, dp: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    return (torch.zeros(k, dp, dtype=torch.int64, device=device),
            torch.zeros(k, dtype=torch.int64, device=device))


def partials_to_float(sums: torch.Tensor, counts: torch.Tensor, d: int | None = None,
                      fx_shift: int = FX_SHIFT):
    s = sums.to(torch.float64) / float(1 << fx_shift)
    if d is not None:
        s = s[:, :d]
    return s, counts.to(torch.float64)


class CentroidImage:
    """Device-resident centroids in the layout the assign kernel consumes."""

    def __init__(self, centroids: torch.Tensor, device, fx_shift: int = FX_SHIFT):
        c = centroids.detach().to(device=device, dtype=torch.float32).contiguous()
        self.k, self.d = c.shape
        self.dp = padded_dim(self.d)
        self.k_pad = padded_k(self.k)
        self.fx_shift = fx_shift
        self.device = c.device
        self.cen = c
        self.cbf = torch.zeros(self.k_pad, self.dp, dtype=torch.bfloat16, device=device)
        self.chalf = torch.empty(self.k_pad, dtype=torch.float32, device=device)
        self.shift2 = torch.zeros(self.k, dtype=torch.float32, device=device)
        self.refresh()

    def refresh(self, sums=None, counts=None, stream=None):
        """Reduce-side update: c = sums/counts (clusters with count 0 keep their
        centroid), then rebuild the bf16 image and -||c||²/2."""
        lib = _lib.load()
        rc = lib.hbmr_kmeans_update(_ptr(sums), _ptr(counts), self.fx_shift, self.k, self.d,
                                    self.dp, self.k_pad, _ptr(self.cen), _ptr(self.cbf),
                                    _ptr(self.chalf), _ptr(self.shift2),
                                    _lib.stream_handle(stream))
        _lib.check(rc, "hbmr_kmeans_update")
        self._img16 = {}       # exact mode's 16-bit images and neighbour table: on demand
        self._nbr = None
        if getattr(self, "_nbr_lock", None) is None:
            self._nbr_lock = threading.Lock()

    def set_centroids(self, centroids: torch.Tensor, stream=None):
        self.cen.copy_(centroids.to(self.cen.device, torch.float32))
        self.refresh(stream=stream)

    def image16(self, dtype=torch.float16):
        """Exact mode's 16-bit centroid image for MFMA operands of ``dtype``
        (fp16, the default, or bf16): (c16 [k_pad, dp], chalf [k_pad] =
        -|c~|²/2, |c_j| [k], max |c_j| [1], |c_j - c~_j| [k], max [1]) — norms
        and rounding errors in fp64 rounded up (hbmr_kmeans_image16), built
        once per image on the first caller's stream; other streams wait."""
        with self._nbr_lock:
            cache = self.__dict__.setdefault("_img16", {})
            ent = cache.get(dtype)
            if ent is None:
                dev = self.cen.device
                c16 = torch.empty(self.k_pad, self.dp, dtype=dtype, device=dev)
                ch = torch.empty(self.k_pad, dtype=torch.float32, device=dev)
                cn = torch.empty(self.k, dtype=torch.float32, device=dev)
                ce = torch.empty(self.k, dtype=torch.float32, device=dev)
                mx = torch.empty(2, dtype=torch.float32, device=dev)
                rc = _lib.load().hbmr_kmeans_image16(
                    _ptr(self.cen), self.k, self.d, self.dp, self.k_pad,
                    int(dtype == torch.float16), _ptr(c16), _ptr(ch), _ptr(cn), _ptr(ce),
                    _ptr(mx), _lib.stream_handle(None))
                _lib.check(rc, "hbmr_kmeans_image16")
                c16t = None
                if self.dp in (64, 128):
                    # the v3 fused assign's tiled copy (hbmr_kmeans_image16_tiled)
                    c16t = torch.empty_like(c16)
                    rc = _lib.load().hbmr_kmeans_image16_tiled(
                        _ptr(c16), self.k_pad, self.dp, _ptr(c16t), _lib.stream_handle(None))
                    _lib.check(rc, "hbmr_kmeans_image16_tiled")
                ev = torch.cuda.Event()
                ev.record()
                ent = cache[dtype] = (c16, ch, cn, mx[0:1], ce, mx[1:2], ev, c16t)
        torch.cuda.current_stream().wait_event(ent[6])
        return ent[:6]

    def image16_tiled(self, dtype=torch.float16):
        """The tiled copy of ``image16(dtype)[0]`` (32-row tiles, 16-byte pieces
        piece-major) the v3 fused assign stages lane-linearly, or None (dp > 128)."""
        self.image16(dtype)
        return self._img16[dtype][7]

    def norms(self, dtype=torch.float16):
        """(|c_j| [k], max_j |c_j| [1], |c_j - c~_j| [k], max_j |c_j - c~_j| [1])
        for the 16-bit image of ``dtype`` (exact mode's certification bound)."""
        _, _, cn, cm, ce, cem = self.image16(dtype)
        return cn, cm, ce, cem

    def neighbors(self, L: int | None = None):
        """Each centroid's L nearest centroids (itself first) and their
        distances, fp64 rounded DOWN to fp32 — exact mode's Elkan scan.  Built
        once per image on the first caller's stream; other streams wait on it."""
        with self._nbr_lock:
            if self._nbr is None:
                if L is None:
                    L = int(os.environ.get("HBMR_KMEANS_NBR_L", NBR_L))
                L = max(1, min(L, self.k))
                if self.cen.is_cuda and self.k <= NBR_NATIVE_MAX_K and self.d <= 256:
                    # one kernel (hbmr_kmeans_centroid_nbr): pairwise fp64
                    # distances, bounds rounded outward, per-row bitonic sort
                    # in LDS — instead of ~40 small torch launches whose host
                    # time held the interpreter lock at the iteration seam
                    dev = self.cen.device
                    di = torch.empty(self.k, L, dtype=torch.int32, device=dev)
                    f = torch.empty(self.k, L, dtype=torch.float32, device=dev)
                    pd = torch.empty(self.k, self.k, dtype=torch.float32, device=dev) \
                        if self.k <= PAIR_DIST_MAX_K else None
                    rc = _lib.load().hbmr_kmeans_centroid_nbr(
                        _ptr(self.cen), self.k, self.d, L, _ptr(di), _ptr(f), _ptr(pd),
                        _lib.stream_handle(None))
                    _lib.check(rc, "hbmr_kmeans_centroid_nbr")
                    ev = torch.cuda.Event()
                    ev.record()
                    self._nbr = (di, f, L, ev, pd)
                    di, f, L, ev, _ = self._nbr
                    torch.cuda.current_stream().wait_event(ev)
                    return di, f, L
                # squared distances by the Gram form in fp64 (one DGEMM instead
                # of a pairwise kernel: ~0.8 ms per image at k = 1024), with
                # the form's rounding error bounded explicitly: |D2 - D| <=
                # (d + 4) 2^-53 (|a|^2 + |b|^2) for fp32 inputs, so the lower
                # bounds (Elkan's scan order and stop rule) and upper bounds
                # (the pair rule) stay rigorous
                c = self.cen.double()
                n2 = (c * c).sum(1)
                nsum = n2[:, None] + n2[None, :]
                d2 = torch.addmm(nsum, c, c.T, beta=1.0, alpha=-2.0)
                err = nsum * ((self.d + 4) * 2.0 ** -53 * 1.01)
                lo = (d2 - err).clamp_(min=0.0).sqrt_()
                lo.fill_diagonal_(0.0)
                dv, di = lo.sort(dim=1, stable=True)
                dv, di = dv[:, :L].contiguous(), di[:, :L].to(torch.int32).contiguous()
                f = dv.float()
                f = torch.where(f.double() > dv, torch.nextafter(f, torch.full_like(f, -1.0)), f)
                # the full matrix of upper bounds rounded UP (the pair rule of
                # the certification's step 1); k <= PAIR_DIST_MAX_K
                pd = None
                if self.k <= PAIR_DIST_MAX_K:
                    hi = (d2 + err).clamp_(min=0.0).sqrt_()
                    hi.fill_diagonal_(0.0)
                    pd = hi.float()
                    pd = torch.where(pd.double() < hi, torch.nextafter(
                        pd, torch.full_like(pd, float("inf"))), pd).contiguous()
                ev = torch.cuda.Event()
                ev.record()
                self._nbr = (di, f.contiguous(), L, ev, pd)
        di, f, L, ev, _ = self._nbr
        torch.cuda.current_stream().wait_event(ev)
        return di, f, L

    def pair_dist(self):
        """|c_a - c_b| for every pair, fp64 rounded up to fp32 [k, k] (None past
        PAIR_DIST_MAX_K clusters): the certification's pair rule."""
        self.neighbors()
        return self._nbr[4]

    def max_shift(self) -> float:
        return float(self.shift2.max().sqrt().item()) if self.k else 0.0


def assign(points: torch.Tensor, img: CentroidImage, labels: torch.Tensor | None = None,
           scores: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """labels[i] = argmin_j ||x_i - c_j||² (MFMA bf16 GEMM + fused arg-max)."""
    n, dp = points.shape
    if points.dtype != torch.bfloat16 or dp != img.dp or not points.is_contiguous():
        raise ValueError("points must be contiguous bf16 [n, dp] matching the centroid image")
    if labels is None:
        labels = torch.empty(n, dtype=torch.int32, device=points.device)
    lib = _lib.load()
    rc = lib.hbmr_kmeans_assign_bf16(_ptr(points), n, dp, _ptr(img.cbf), _ptr(img.chalf),
                                     img.k_pad, _ptr(labels), _ptr(scores),
                                     _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_kmeans_assign_bf16")
    return labels


ACCUM_AUTO, ACCUM_LDS, ACCUM_SORTED = 0, 1, 2
_workspaces: dict = {}


def workspace_bytes(n: int, k: int) -> int:
    return int(_lib.load().hbmr_kmeans_accum_workspace_bytes(n, k))


def batch_scratch_sizes(ns: list, k: int) -> tuple[int, int]:
    """(label entries, workspace bytes) a map batch over splits of sizes ``ns`` needs
    (grouped kernels keep every split's labels/permutation side by side)."""
    lib = _lib.load()
    total = int(sum(ns))
    ws = max(int(lib.hbmr_kmeans_batch_workspace_bytes(total, len(ns), k)),
             int(lib.hbmr_kmeans_accum_workspace_bytes(max(ns), k)))
    return total, ws


def accum_workspace(n: int, k: int, device) -> torch.Tensor:
    """Per-(device, stream-free) scratch for the sorted combiner, grown on demand.

    Reused across calls on the same device; callers that run accumulations on
    several streams concurrently must pass their own ``workspace``."""
    lib = _lib.load()
    need = int(lib.hbmr_kmeans_accum_workspace_bytes(n, k))
    key = torch.device(device)
    ws = _workspaces.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(max(need, 1 << 20), dtype=torch.uint8, device=key)
        _workspaces[key] = ws
    return ws


def accumulate(points: torch.Tensor, labels: torch.Tensor, k: int, sums: torch.Tensor,
               counts: torch.Tensor, fx_shift: int = FX_SHIFT, stream=None,
               workspace: torch.Tensor | None = None, mode: int = ACCUM_AUTO) -> None:
    """sums[label] += round(x·2^fx_shift), counts[label] += 1 (int64 fixed point).

    Small k uses LDS-privatised accumulators; large k a counting sort of the
    labels followed by a segmented row sum (no atomics in the hot loop)."""
    n, dp = points.shape
    if sums.shape != (k, dp) or sums.dtype != torch.int64:
        raise ValueError(f"sums must be int64 [{k}, {dp}]")
    if counts.shape != (k,) or counts.dtype != torch.int64:
        raise ValueError(f"counts must be int64 [{k}]")
    if points.dtype not in (torch.bfloat16, torch.float32) or not points.is_contiguous() or \
            dp not in SUPPORTED_DP or labels.numel() < n:
        raise ValueError("points must be contiguous bf16/fp32 [n, dp] with n labels")
    lib = _lib.load()
    if workspace is None and mode != ACCUM_LDS:
        workspace = accum_workspace(n, k, points.device)
    fn, name = ((lib.hbmr_kmeans_accum_f32, "hbmr_kmeans_accum_f32")
                if points.dtype == torch.float32 else
                (lib.hbmr_kmeans_accum_bf16, "hbmr_kmeans_accum_bf16"))
    rc = fn(_ptr(points), n, dp, _ptr(labels), k, _ptr(sums), _ptr(counts), fx_shift,
            _ptr(workspace), 0 if workspace is None else workspace.numel(), mode,
            _lib.stream_handle(stream))
    _lib.check(rc, name)


# --------------------------------------------------------------------------- exact mode
def _f32_up(v: torch.Tensor) -> torch.Tensor:
    """fp64 → fp32 rounded towards +inf (an upper bound stays an upper bound)."""
    f = v.float()
    return torch.where(f.double() < v, torch.nextafter(f, torch.full_like(f, float("inf"))), f)


class ExactSplit:
    """A split held for exact mode (``hbmr.kmeans.exact``): the 16-bit copy the
    MFMA assign reads (``xb``: fp16 by default — 11 significant bits, so the
    certification flags ~8x fewer points than with bf16's 8 — or bf16), the
    fp32 data (rows padded to dp) the certification re-score and the combiner
    read, and per point |x| (fp32 data), |x~|² (16-bit copy) and the rounding
    error |x - x~| (an upper bound), computed in fp64 once when the split is
    made resident (hbmr_kmeans_exact_prep)."""
    __slots__ = ("xb", "x32", "xnorm", "xbn2", "xerr", "d")

    def __init__(self, x32: torch.Tensor, dp: int, dtype=torch.float16):
        n, d = x32.shape
        self.d = d
        dev = x32.device
        if dp == d:
            self.x32 = x32.contiguous()
        else:
            self.x32 = torch.zeros(n, dp, dtype=torch.float32, device=dev)
            self.x32[:, :d] = x32
        if dev.type == "cuda":
            self.xb = torch.empty(n, dp, dtype=dtype, device=dev)
            self.xnorm = torch.empty(n, dtype=torch.float32, device=dev)
            self.xbn2 = torch.empty(n, dtype=torch.float32, device=dev)
            self.xerr = torch.empty(n, dtype=torch.float32, device=dev)
            rc = _lib.load().hbmr_kmeans_exact_prep(
                _ptr(self.x32), n, dp, dp, dp, int(dtype == torch.float16), _ptr(self.xb),
                _ptr(self.xnorm), _ptr(self.xbn2), _ptr(self.xerr), _lib.stream_handle(None))
            _lib.check(rc, "hbmr_kmeans_exact_prep")
            return
        x64 = self.x32.double()
        self.xnorm = x64.norm(dim=1).float()
        lim = 65504.0 if dtype == torch.float16 else float("inf")
        xb = self.x32.clamp(-lim, lim).to(dtype)
        xb64 = xb.double()
        self.xbn2 = xb64.pow(2).sum(1).float()
        self.xerr = _f32_up((x64 - xb64).norm(dim=1))
        self.xb = xb.contiguous()

    @property
    def shape(self):
        return self.xb.shape

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.xb, self.x32, self.xnorm,
                                                          self.xbn2, self.xerr))


def assign_top3(points: torch.Tensor, img: CentroidImage, labels, cand, scores, margin,
                stream=None) -> None:
    """bf16 MFMA assign keeping the three best clusters: labels [n] (best),
    cand [2n] (second | third), scores [n] (best score), margin [2n]
    (best - second | best - third)."""
    n, dp = points.shape
    if points.dtype not in (torch.bfloat16, torch.float16) or dp != img.dp or \
            not points.is_contiguous():
        raise ValueError("points must be contiguous bf16/fp16 [n, dp] matching the image")
    for t, dt, m in ((labels, torch.int32, 1), (cand, torch.int32, 2), (scores, torch.float32, 1),
                     (margin, torch.float32, 2)):
        if t.numel() != m * n or t.dtype != dt or not t.is_contiguous():
            raise ValueError("top-3 outputs: labels/scores [n], cand/margin [2n]")
    f16 = points.dtype == torch.float16
    with torch.cuda.stream(stream) if stream is not None else _nullctx():
        c16, ch = img.image16(points.dtype)[:2]
    fn = "hbmr_kmeans_assign_top3_f16" if f16 else "hbmr_kmeans_assign_top3_bf16"
    rc = getattr(_lib.load(), fn)(
        _ptr(points), n, dp, _ptr(c16), _ptr(ch), img.k_pad, _ptr(labels),
        _ptr(cand), _ptr(scores), _ptr(margin), _lib.stream_handle(stream))
    _lib.check(rc, fn)


REFINE_VERSION = int(os.environ.get("HBMR_REFINE", "3"))
MAX_REFINE_BATCH = 64     # splits per refine v3 batch (the kernels' split table)


def _refine_ws(ns: list, device, scratch: dict | None):
    """Queue workspace of a refine v3 batch, kept in ``scratch`` across calls
    (one stream orders the reuse)."""
    arr = (ctypes.c_long * len(ns))(*ns)
    need = int(_lib.load().hbmr_kmeans_refine_batch_bytes(len(ns), arr))
    if need < 0:
        raise ValueError("refine batch of 1..64 splits expected")
    ws = None if scratch is None else scratch.get("refine_ws")
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=device)
        if scratch is not None:
            scratch["refine_ws"] = ws
    return arr, ws


class _RefineBatch:
    """Refine v3 over a batch of splits: ``q1`` right after each split's top-3
    assign (its candidate scratch may be reused by the next split), ``finish``
    once (step 2 + Elkan scan over the batch's queues)."""

    def __init__(self, splits: list, img: "CentroidImage", stats, scratch, stream):
        self.splits, self.img, self.stats, self.stream = splits, img, stats, stream
        self.dt = splits[0].xb.dtype
        self.ns, self.ws = _refine_ws([sp.shape[0] for sp in splits], splits[0].x32.device,
                                      scratch)
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            self.norms = img.norms(self.dt)
            self.nbr = img.neighbors()
            self.pd = img.pair_dist()
        self.labels = [None] * len(splits)
        self.lib = _lib.load()
        self.st = _lib.stream_handle(stream)

    def q1(self, i, labels_ptr, cand, scores, margin):
        sp, img = self.splits[i], self.img
        cn, cmax, ce, cemax = self.norms
        self.labels[i] = labels_ptr
        rc = self.lib.hbmr_kmeans_refine_batch_q1(
            len(self.splits), self.ns, i, img.d, img.k, img.k_pad, _ptr(sp.xnorm),
            _ptr(sp.xbn2), _ptr(sp.xerr), _ptr(cn), _ptr(cmax), _ptr(ce), _ptr(cemax),
            labels_ptr, _ptr(cand), _ptr(scores), _ptr(margin), _ptr(self.stats),
            _ptr(self.ws), self.ws.numel(), int(i == 0), _ptr(self.pd), self.st)
        _lib.check(rc, "hbmr_kmeans_refine_batch_q1")

    def finish(self):
        B = len(self.splits)
        img = self.img
        _, cmax, _, cemax = self.norms
        ni, nd, L = self.nbr
        xs = (ctypes.c_void_p * B)(*[sp.x32.data_ptr() for sp in self.splits])
        ls = (ctypes.c_void_p * B)(*[(lp.value if isinstance(lp, ctypes.c_void_p) else lp)
                                     for lp in self.labels])
        rc = self.lib.hbmr_kmeans_refine_batch_finish(
            B, self.ns, xs, ls, img.d, self.splits[0].x32.shape[1], _ptr(img.cen), img.k,
            img.k_pad, _ptr(cmax), _ptr(cemax), _ptr(ni), _ptr(nd), L, _ptr(self.stats),
            self.stats.numel(), _ptr(self.ws), self.ws.numel(), self.st)
        _lib.check(rc, "hbmr_kmeans_refine_batch_finish")


def refine_f32(split: ExactSplit, img: CentroidImage, labels, cand, scores, margin,
               stats: torch.Tensor, stream=None, scratch: dict | None = None) -> None:
    """Certify the MFMA labels against the fp32 data; re-score the uncertain
    points in fp64 (refine v3, the queue pipeline; HBMR_REFINE=1/2: the older
    single-kernel forms).  stats (int64 [3]) += (flagged, relabelled, points
    that needed the neighbour scan); a [5] stats also counts the scan's
    neighbour distances and its full scans."""
    n = split.shape[0]
    if stats.dtype != torch.int64 or stats.numel() < 3:
        raise ValueError("stats must be int64 [3]")
    if labels.numel() != n or cand.numel() != 2 * n or margin.numel() != 2 * n:
        raise ValueError("labels [n], cand/margin [2n] from assign_top3 expected")
    if REFINE_VERSION >= 3:
        rb = _RefineBatch([split], img, stats, scratch, stream)
        rb.q1(0, labels.data_ptr(), cand, scores, margin)
        rb.finish()
        return
    with torch.cuda.stream(stream) if stream is not None else _nullctx():
        cn, cmax, ce, cemax = img.norms(split.xb.dtype)
        ni, nd, L = img.neighbors()
    rc = _lib.load().hbmr_kmeans_refine_f32(
        _ptr(split.x32), n, img.d, split.x32.shape[1], _ptr(split.xnorm), _ptr(split.xbn2),
        _ptr(split.xerr), _ptr(img.cen), img.k, img.k_pad, _ptr(cn), _ptr(cmax), _ptr(ce),
        _ptr(cemax), _ptr(ni), _ptr(nd), L,
        _ptr(labels), _ptr(cand), _ptr(scores), _ptr(margin), _ptr(stats), stats.numel(),
        _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_kmeans_refine_f32")


def assign_exact(split: ExactSplit, img: CentroidImage, stats: torch.Tensor,
                 scratch: dict | None = None, stream=None) -> torch.Tensor:
    """Exact labels of the split's fp32 points: top-3 bf16 assign +
    certification / fp64 re-score.  Returns labels [n] (a scratch view)."""
    n = split.shape[0]
    dev = split.xb.device
    scratch = {} if scratch is None else scratch
    key = ("exact", n)
    bufs = scratch.get(key)
    if bufs is None:
        bufs = scratch[key] = (torch.empty(n, dtype=torch.int32, device=dev),
                               torch.empty(2 * n, dtype=torch.int32, device=dev),
                               torch.empty(n, dtype=torch.float32, device=dev),
                               torch.empty(2 * n, dtype=torch.float32, device=dev))
    lab, cand, sc, mg = bufs
    assign_top3(split.xb, img, lab, cand, sc, mg, stream=stream)
    refine_f32(split, img, lab, cand, sc, mg, stats, stream=stream, scratch=scratch)
    return lab


def assign_exact_batch(splits: list, img: CentroidImage, stats: torch.Tensor, out: torch.Tensor,
                       scratch: dict | None = None, stream=None) -> None:
    """Exact labels of a batch of splits, written back to back into ``out``
    (int32 [sum n]): the top-3 assign and the step-1 certification per split
    (the candidate / score / margin scratch shared by every split: one stream
    orders the reuse), then step 2 and the neighbour scan once per up to 64
    splits (refine v3), with the centroid norms / neighbour lists fetched once
    and the labels written in place."""
    if not splits:
        return
    dev = splits[0].xb.device
    total = sum(sp.shape[0] for sp in splits)
    if out.dtype != torch.int32 or out.numel() < total or not out.is_contiguous():
        raise ValueError("out must be contiguous int32 with room for every split's labels")
    if stats.dtype != torch.int64 or stats.numel() < 3:
        raise ValueError("stats must be int64 [3]")
    dt = splits[0].xb.dtype
    for sp in splits:
        if sp.xb.dtype != dt or dt not in (torch.bfloat16, torch.float16) or \
                sp.xb.shape[1] != img.dp or not sp.xb.is_contiguous() or \
                not sp.x32.is_contiguous():
            raise ValueError("exact splits must hold contiguous [n, dp] rows of one 16-bit type")
    nmax = max(sp.shape[0] for sp in splits)
    scratch = {} if scratch is None else scratch
    key = ("exact-batch", nmax)
    bufs = scratch.get(key)
    if bufs is None:
        for kk in [kk for kk in scratch if isinstance(kk, tuple) and kk[0] == "exact-batch"]:
            del scratch[kk]
        bufs = scratch[key] = (torch.empty(2 * nmax, dtype=torch.int32, device=dev),
                               torch.empty(nmax, dtype=torch.float32, device=dev),
                               torch.empty(2 * nmax, dtype=torch.float32, device=dev))
    cand, sc, mg = bufs
    grouped = REFINE_VERSION >= 3 and img.dp <= 128 and GROUPED_EXACT
    with torch.cuda.stream(stream) if stream is not None else _nullctx():
        c16, ch, cn, cmax, ce, cemax = img.image16(dt)
        # the neighbour table is waited for only where the certification
        # needs it (after the first top-3 launch: the reduce builds it on its
        # own stream while that assign runs)
        ni, nd, L = (None, None, 0) if grouped else img.neighbors()
    lib = _lib.load()
    top3 = lib.hbmr_kmeans_assign_top3_f16 if dt == torch.float16 else \
        lib.hbmr_kmeans_assign_top3_bf16
    st = _lib.stream_handle(stream)
    pc, ps, pm, pst = _ptr(cand), _ptr(sc), _ptr(mg), _ptr(stats)
    pcn, pcmax, pce, pcemax, pni, pnd = (_ptr(t) for t in (cn, cmax, ce, cemax, ni, nd))
    base, off = out.data_ptr(), 0
    for g0 in range(0, len(splits), MAX_REFINE_BATCH):
        group = splits[g0:g0 + MAX_REFINE_BATCH]
        if grouped:
            off += _exact_group(group, img, stats, base + 4 * off, c16, ch, (cn, cmax, ce, cemax),
                                dt, scratch, stream, lib, st)
            continue
        rb = _RefineBatch(group, img, stats, scratch, stream) if REFINE_VERSION >= 3 else None
        for i, sp in enumerate(group):
            n = sp.shape[0]
            pl = ctypes.c_void_p(base + 4 * off)
            rc = top3(_ptr(sp.xb), n, img.dp, _ptr(c16), _ptr(ch), img.k_pad, pl, pc, ps, pm, st)
            _lib.check(rc, "hbmr_kmeans_assign_top3")
            if rb is not None:
                rb.q1(i, pl, cand, sc, mg)
            else:
                rc = lib.hbmr_kmeans_refine_f32(
                    _ptr(sp.x32), n, img.d, sp.x32.shape[1], _ptr(sp.xnorm), _ptr(sp.xbn2),
                    _ptr(sp.xerr), _ptr(img.cen), img.k, img.k_pad, pcn, pcmax, pce, pcemax,
                    pni, pnd, L, pl, pc, ps, pm, pst, stats.numel(), st)
                _lib.check(rc, "hbmr_kmeans_refine_f32")
            off += n
        if rb is not None:
            rb.finish()


# the pair rule of the certification keeps a [k, k] centroid distance matrix
PAIR_DIST_MAX_K = int(os.environ.get("HBMR_PAIR_DIST_MAX_K", "8192"))
# the native neighbour table sorts a row of k keys in LDS (k <= 8192)
NBR_NATIVE_MAX_K = int(os.environ.get("HBMR_NBR_NATIVE_MAX_K", "8192"))
# exact batches: one top-3 launch + one step-1 launch per up to 64 splits
# (HBMR_EXACT_GROUPED=0: a launch of each per split)
GROUPED_EXACT = os.environ.get("HBMR_EXACT_GROUPED", "1") != "0"
# step 1 of the certification inside the grouped top-3 kernel's epilogue
# (HBMR_EXACT_FUSED_Q1=0: the separate step-1 scan over materialised arrays)
FUSED_Q1 = os.environ.get("HBMR_EXACT_FUSED_Q1", "1") != "0"


def _exact_group(group, img, stats, labels_ptr, c16, ch, norms, dt, scratch, stream, lib, st):
    """Top-3 assign and certification of up to 64 splits with grouped launches
    (hbmr_kmeans_assign_top3_grouped, hbmr_kmeans_refine_batch_q1g); labels of
    the group written back to back at ``labels_ptr``.  Returns the row count."""
    B = len(group)
    ns = [sp.shape[0] for sp in group]
    N = sum(ns)
    dev = group[0].xb.device
    P = ctypes.c_void_p * B
    xs = P(*[sp.xb.data_ptr() for sp in group])
    nsa = (ctypes.c_long * B)(*ns)
    if FUSED_Q1 and img.dp <= 128:
        # step 1 in the top-3 epilogue: no candidate / score / margin arrays
        rb = _RefineBatch(group, img, stats, scratch, stream)
        if TRACE.on:
            TRACE.instant("kmeans.top3_launch", n=B)
        cn, cmax, ce, cemax = norms
        rc = lib.hbmr_kmeans_assign_top3_q1_grouped(
            B, xs, nsa, img.dp, int(dt == torch.float16), _ptr(c16),
            _ptr(img.image16_tiled(dt)), _ptr(ch), img.k_pad,
            labels_ptr, P(*[sp.xnorm.data_ptr() for sp in group]),
            P(*[sp.xbn2.data_ptr() for sp in group]), P(*[sp.xerr.data_ptr() for sp in group]),
            img.d, img.k, _ptr(cn), _ptr(cmax), _ptr(ce), _ptr(cemax), _ptr(rb.ws),
            rb.ws.numel(), _ptr(rb.pd), st)
        _lib.check(rc, "hbmr_kmeans_assign_top3_q1_grouped")
        o = 0
        for i in range(B):
            rb.labels[i] = labels_ptr + 4 * o
            o += ns[i]
        rb.finish()
        return N
    key = ("exact-group", N)
    bufs = scratch.get(key)
    if bufs is None:
        for kk in [kk for kk in scratch if isinstance(kk, tuple) and kk[0] == "exact-group"]:
            del scratch[kk]
        bufs = scratch[key] = (torch.empty(2 * N, dtype=torch.int32, device=dev),
                               torch.empty(N, dtype=torch.float32, device=dev),
                               torch.empty(2 * N, dtype=torch.float32, device=dev))
    cand, sc, mg = bufs
    rc = lib.hbmr_kmeans_assign_top3_grouped(B, xs, nsa, img.dp, int(dt == torch.float16),
                                             _ptr(c16), _ptr(ch), img.k_pad, labels_ptr,
                                             _ptr(cand), _ptr(sc), _ptr(mg), st)
    _lib.check(rc, "hbmr_kmeans_assign_top3_grouped")
    rb = _RefineBatch(group, img, stats, scratch, stream)
    cn, cmax, ce, cemax = norms
    rc = lib.hbmr_kmeans_refine_batch_q1g(
        B, nsa, img.d, img.k, img.k_pad, P(*[sp.xnorm.data_ptr() for sp in group]),
        P(*[sp.xbn2.data_ptr() for sp in group]), P(*[sp.xerr.data_ptr() for sp in group]),
        _ptr(cn), _ptr(cmax), _ptr(ce), _ptr(cemax), labels_ptr, _ptr(cand), _ptr(sc), _ptr(mg),
        _ptr(rb.ws), rb.ws.numel(), _ptr(rb.pd), st)
    _lib.check(rc, "hbmr_kmeans_refine_batch_q1g")
    o = 0
    for i in range(B):
        rb.labels[i] = labels_ptr + 4 * o
        o += ns[i]
    rb.finish()
    return N


def map_split_exact(split: ExactSplit, img: CentroidImage, sums, counts, scratch: dict,
                    stats: torch.Tensor, stream=None) -> None:
    """One exact-mode GPU map task: top-3 assign, certification + fp64 re-score,
    then the int64 fixed-point combiner over the fp32 rows."""
    n = split.shape[0]
    lab = assign_exact(split, img, stats, scratch, stream=stream)
    need = workspace_bytes(n, img.k)
    if scratch.get("ws") is None or scratch["ws"].numel() < need:
        scratch["ws"] = torch.empty(max(need, 1 << 20), dtype=torch.uint8, device=split.xb.device)
    accumulate(split.x32, lab, img.k, sums, counts, fx_shift=img.fx_shift, stream=stream,
               workspace=scratch["ws"])


def map_batch_gpu(splits: list, img: CentroidImage, sums: torch.Tensor, counts: torch.Tensor,
                  labels: torch.Tensor, workspace: torch.Tensor, stream=None,
                  zero_outputs: bool = True) -> None:
    """A batch of map tasks in one native call: splits[t] (bf16 [n_t, dp]) →
    sums[t] ([B, k, dp] int64), counts[t] ([B, k] int64)."""
    B = len(splits)
    if B == 0:
        return
    for s in splits:
        if s.dtype != torch.bfloat16 or s.shape[1] != img.dp or not s.is_contiguous():
            raise ValueError("splits must be contiguous bf16 [n, dp]")
    if sums.shape != (B, img.k, img.dp) or counts.shape != (B, img.k):
        raise ValueError("batch output shape mismatch")
    need_lab, need_ws = batch_scratch_sizes([s.shape[0] for s in splits], img.k)
    if labels.numel() < need_lab:
        raise ValueError("labels scratch too small")
    lib = _lib.load()
    if workspace.numel() < need_ws:
        raise ValueError("workspace too small")
    ptrs = (ctypes.c_void_p * B)(*[s.data_ptr() for s in splits])
    ns = (ctypes.c_long * B)(*[s.shape[0] for s in splits])
    rc = lib.hbmr_kmeans_map_batch(B, ptrs, ns, img.dp, _ptr(img.cbf), _ptr(img.chalf), img.k_pad,
                                   img.k, _ptr(labels), _ptr(workspace), workspace.numel(),
                                   _ptr(sums), _ptr(counts), img.fx_shift, int(zero_outputs),
                                   _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_kmeans_map_batch")


# --------------------------------------------------------------------------- delta combiner
class Baseline:
    """Reference partition of one split for the delta combiner: labels ``g``
    (int32 [n]) and its exact partials ``S0`` (int64 [k, dp]), ``N0`` (int64
    [k]).  Invariant: S0[c] = Σ_{g(p)=c} fx(x_p), N0[c] = #{p: g(p)=c} — it
    holds for ANY g, so the map output computed against it is bit-identical to
    the direct combiner's; it only pays off when few points changed label.
    ``event`` marks the end of the batch that last updated it (its stream is
    ``stream``): a batch on another stream waits for it first."""
    __slots__ = ("g", "S0", "N0", "event", "stream", "data_ptr", "n")

    def __init__(self, g, S0, N0, data_ptr, n):
        self.g, self.S0, self.N0 = g, S0, N0
        self.event = None
        self.stream = None
        self.data_ptr, self.n = data_ptr, n


def delta_workspace_bytes(total: int, ntasks: int, k: int) -> int:
    return int(_lib.load().hbmr_kmeans_delta_workspace_bytes(total, ntasks, k))


def _delta_args(xs, bases, stream):
    B = len(xs)
    st = torch.cuda.current_stream() if stream is None else stream
    events, blocks = {}, {}
    for b in bases:
        # the reference partition may have been written (g) / allocated (S0, N0)
        # on another stream: order this batch after it, and keep the memory from
        # being reused under this stream's pending reads (once per event and
        # per allocation: the baselines of a batch share a few slabs)
        if b.event is not None and b.stream is not None and b.stream != st:
            events[id(b.event)] = b.event
        for t in (b.g, b.S0, b.N0):
            base = t._base if t._base is not None else t
            blocks[id(base)] = base
    for ev in events.values():
        st.wait_event(ev)
    for t in blocks.values():
        t.record_stream(st)
    ptrs = (ctypes.c_void_p * B)(*[x.data_ptr() for x in xs])
    ns = (ctypes.c_long * B)(*[x.shape[0] for x in xs])
    gs = (ctypes.c_void_p * B)(*[b.g.data_ptr() for b in bases])
    s0 = (ctypes.c_void_p * B)(*[b.S0.data_ptr() for b in bases])
    n0 = (ctypes.c_void_p * B)(*[b.N0.data_ptr() for b in bases])
    return ptrs, ns, gs, s0, n0


def map_batch_delta(splits: list, img: CentroidImage, sums: torch.Tensor, counts: torch.Tensor,
                    labels: torch.Tensor, workspace: torch.Tensor, bases: list,
                    stream=None) -> None:
    """A batch of map tasks against reference partitions (hbmr_kmeans_map_batch_delta):
    grouped MFMA assign, then the delta combiner.  sums/counts [B, k, dp] /
    [B, k] are overwritten; every ``bases[t]`` advances to this batch's labels."""
    B = len(splits)
    if B == 0:
        return
    if B > 64 or len(bases) != B:
        raise ValueError("at most 64 splits per delta batch, one baseline each")
    for s, b in zip(splits, bases):
        if s.dtype != torch.bfloat16 or s.shape[1] != img.dp or not s.is_contiguous():
            raise ValueError("splits must be contiguous bf16 [n, dp]")
        if b.g.numel() != s.shape[0] or tuple(b.S0.shape) != (img.k, img.dp) or \
                b.N0.numel() != img.k:
            raise ValueError("baseline does not match its split")
    if sums.shape != (B, img.k, img.dp) or counts.shape != (B, img.k) or \
            not sums.is_contiguous() or not counts.is_contiguous():
        raise ValueError("batch output shape mismatch")
    total = sum(s.shape[0] for s in splits)
    if labels.numel() < total:
        raise ValueError("labels scratch too small")
    need = delta_workspace_bytes(total, B, img.k)
    if workspace.numel() < need:
        raise ValueError("workspace too small")
    ptrs, ns, gs, s0, n0 = _delta_args(splits, bases, stream)
    rc = _lib.load().hbmr_kmeans_map_batch_delta(
        B, ptrs, ns, img.dp, _ptr(img.cbf), _ptr(img.chalf), img.k_pad, img.k, _ptr(labels),
        _ptr(workspace), workspace.numel(), _ptr(sums), _ptr(counts), img.fx_shift, gs, s0, n0,
        _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_kmeans_map_batch_delta")


def delta_combine(xs: list, labels: torch.Tensor, k: int, sums: torch.Tensor,
                  counts: torch.Tensor, workspace: torch.Tensor, bases: list,
                  fx_shift: int = FX_SHIFT, stream=None) -> None:
    """The delta combiner alone over precomputed labels (concatenated in task
    order): rows are bf16 or fp32 (exact mode) ``[n_t, dp]``."""
    B = len(xs)
    if B == 0:
        return
    dp = xs[0].shape[1]
    f32 = xs[0].dtype == torch.float32
    for x, b in zip(xs, bases):
        if x.dtype != xs[0].dtype or x.shape[1] != dp or not x.is_contiguous() or \
                b.g.numel() != x.shape[0]:
            raise ValueError("delta_combine: rows/baselines mismatch")
    if B > 64 or dp not in SUPPORTED_DP or sums.shape != (B, k, dp) or counts.shape != (B, k):
        raise ValueError("delta_combine: shape mismatch")
    total = sum(x.shape[0] for x in xs)
    need = delta_workspace_bytes(total, B, k)
    if workspace.numel() < need or labels.numel() < total:
        raise ValueError("delta_combine: scratch too small")
    ptrs, ns, gs, s0, n0 = _delta_args(xs, bases, stream)
    rc = _lib.load().hbmr_kmeans_delta_combine(
        B, ptrs, ns, dp, int(f32), k, _ptr(labels), _ptr(workspace), workspace.numel(),
        _ptr(sums), _ptr(counts), fx_shift, gs, s0, n0, _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_kmeans_delta_combine")


def map_split_gpu(points, img: CentroidImage, sums, counts, labels=None, stream=None):
    """One GPU K-Means map task over an HBM-resident split: assign + combine."""
    labels = assign(points, img, labels=labels, stream=stream)
    accumulate(points, labels, img.k, sums, counts, fx_shift=img.fx_shift, stream=stream)
    return labels


def map_split_cpu(points: torch.Tensor, centroids: torch.Tensor, sums: torch.Tensor,
                  counts: torch.Tensor, nthreads: int = 1, labels: torch.Tensor | None = None,
                  fx_shift: int = FX_SHIFT, exact: bool = False, stats: list | None = None):
    """CPU K-Means map task (native C++, fp32 math, int64 fixed-point partials).

    ``sums`` is int64 ``[k, d]`` (or ``[k, dp]``: only the first d columns are
    touched).  Returns the partial cost Σ min_j ||x - c_j||².  ``exact``: near
    ties (fp32 margin within the fp32 error bound) are re-scored in fp64;
    ``stats[0]`` += re-scored points.
    """
    x = points.detach().to(torch.float32).contiguous()
    c = centroids.detach().to(torch.float32).contiguous()
    n, d = x.shape
    k = c.shape[0]
    if counts.shape != (k,) or counts.dtype != torch.int64 or sums.dtype != torch.int64:
        raise ValueError("sums/counts must be int64")
    target = sums
    if sums.shape != (k, d):
        target = torch.zeros(k, d, dtype=torch.int64)
    cost = ctypes.c_double(0.0)
    lib = _lib.load()
    res = ctypes.c_long(0)
    rc = lib.hbmr_kmeans_map_cpu_f32_ex(_ptr(x), n, d, _ptr(c), k, _ptr(labels), _ptr(target),
                                        _ptr(counts), ctypes.byref(cost), fx_shift, int(nthreads),
                                        int(exact), ctypes.byref(res))
    _lib.check(rc, "hbmr_kmeans_map_cpu_f32_ex")
    if stats is not None:
        stats[0] += res.value
    if target is not sums:
        sums[:, :d] += target
    return cost.value
