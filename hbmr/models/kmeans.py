"""K-Means as a MapReduce job family — BASELINE configs 2 and 3.

One Lloyd iteration = one job (as in Shirahata et al.'s K-Means on Hadoop,
where iterations are chained jobs and the centroids travel in the
DistributedCache):

* map (per split)      : assign every point to its nearest centroid and
                         combine in-task to per-cluster (sum, count) partials.
                         GPU slots run the MFMA kernels of
                         native/kernels/kmeans.hip on the HBM-resident split;
                         CPU slots run the native C++ map (native/cpu).
                         Partials are int64 fixed point → exact and
                         placement-independent.
* combine (per tracker): sum the committed attempts' partials on the device.
* reduce (collective)  : one all-reduce of the [k, dp+1] int64 partials over
                         RCCL (xGMI), then every tracker computes the new
                         centroids and keeps them resident for the next
                         iteration — the DistributedCache broadcast becomes a
                         no-op.  Reducer r commits clusters of partition r to
                         the job output directory (if one is set).

Inputs: ``synthetic:<points>:<seed>`` (a Gaussian mixture generated directly
into HBM by a counter-based generator, identical on CPU and GPU) or a path of
SequenceFiles of (LongWritable, FloatVectorWritable).
"""
from __future__ import annotations

import base64
import logging
import math
import os
import threading
import time

import numpy as np
import torch

from ..gpu.splitjob import SplitJob, SplitSpec
from ..mapred import counters as C

log = logging.getLogger("hbmr.kmeans")

K_KEY = "hbmr.kmeans.k"
D_KEY = "hbmr.kmeans.dims"
INPUT_KEY = "hbmr.kmeans.input"
SPLIT_PTS_KEY = "hbmr.split.points"
CIN_KEY = "hbmr.kmeans.centroids.in"
COUT_KEY = "hbmr.kmeans.centroids.out"
INIT_KEY = "hbmr.kmeans.centroids.init"     # base64 fp32 [k, d] (first iteration only)
NCENTERS_KEY = "hbmr.kmeans.synthetic.centers"
RETURN_KEY = "hbmr.kmeans.return.centroids"   # reduce result carries the new centroids
# rank 0's reduce also writes every centroid version here (in the background),
# so a tracker whose GPU worker restarted can re-localise the input centroids of
# the next iteration (the DistributedCache role; the fast path stays in memory)
CDIR_KEY = "hbmr.kmeans.centroids.dir"
# exact mode: 16-bit MFMA assign certified against the fp32 data (top-3 + fp64
# re-score of uncertain points) and fp32 fixed-point sums (ops.kmeans.ExactSplit)
EXACT_KEY = "hbmr.kmeans.exact"
# exact mode's MFMA operand type: "f16" (default: 11 significant bits, ~8x fewer
# points to re-score than bf16) or "bf16"
EXACT_MFMA_KEY = "hbmr.kmeans.exact.mfma"
# GPU combiner: "delta" (default) sums only the points whose label changed
# against the split's reference partition (ops.kmeans.Baseline) — bit-identical
# to "sorted", the counting-sort combiner over every point
COMBINER_KEY = "hbmr.kmeans.combiner"

# --------------------------------------------------------------------------- data
_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """32-bit integer finaliser (values kept in int64, all products < 2^63)."""
    x = x & _M32
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & _M32
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & _M32
    return x ^ (x >> 16)


def _uniform(c: torch.Tensor) -> torch.Tensor:
    return (_mix32(c).to(torch.float64) + 0.5) * (1.0 / 4294967296.0)


def _gauss(c1: torch.Tensor, c2: torch.Tensor) -> torch.Tensor:
    u1 = _uniform(c1)
    u2 = _uniform(c2)
    return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2)


def synthetic_points(seed: int, start: int, n: int, d: int, centers: int, device,
                     chunk: int = 1 << 18) -> torch.Tensor:
    """Gaussian-mixture points [n, d] (float32) for global indices [start, start+n).

    Counter-based: point p, dim j depends only on (seed, p, j), so any split is
    generated independently and identically on CPU or GPU."""
    dev = torch.device(device)
    out = torch.empty(n, d, dtype=torch.float32, device=dev)
    j = torch.arange(d, dtype=torch.int64, device=dev)
    cidx = torch.arange(centers, dtype=torch.int64, device=dev)
    s = (seed * 0x9E3779B1) & _M32
    # centers: 10 × N(0,1) per (center, dim)
    cc = (cidx[:, None] * 131071 + j[None, :] + s * 7) & _M32
    cen = 10.0 * _gauss(cc * 2 + 1, cc * 2 + 2)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        p = torch.arange(start + a, start + b, dtype=torch.int64, device=dev)
        lab = _mix32(p * 3 + s) % centers
        base = ((p[:, None] & 0xFFFFFF) * 1024 + j[None, :] + (s << 7)) & _M32
        noise = _gauss(base * 2 + 11, base * 2 + 12 + (p[:, None] >> 24))
        out[a:b] = (cen[lab] + noise).to(torch.float32)
    return out


def encode_centroids(c: torch.Tensor) -> str:
    a = c.detach().to("cpu", torch.float32).contiguous().numpy()
    return f"{a.shape[0]}x{a.shape[1]}:" + base64.b64encode(a.tobytes()).decode()


def decode_centroids(s: str) -> torch.Tensor:
    shp, b = s.split(":", 1)
    k, d = map(int, shp.split("x"))
    return torch.from_numpy(np.frombuffer(base64.b64decode(b), dtype=np.float32).copy()
                            ).reshape(k, d)


# --------------------------------------------------------------------------- side data
class CentroidStore:
    """Per-process centroid versions, the DistributedCache analogue: key →
    fp32 host centroids and per-device bf16 images (CentroidImage)."""

    def __init__(self):
        self.lock = threading.Lock()
        self.host: dict[str, torch.Tensor] = {}
        self.images: dict[tuple, object] = {}
        self.order: list[str] = []
        self.keep = 4

    def put_host(self, key, cen):
        """New host centroids of ``key``: device images of an earlier version
        of the key (a restarted reduce re-publishing it) are dropped."""
        with self.lock:
            self.host[key] = cen
            for k in [k for k in self.images if k[0] == key]:
                self.images.pop(k)
            self._touch(key)

    def put_image(self, key, device, img):
        """A device image of ``key``; a host copy of an earlier version is
        dropped (re-derived from the images on demand).  Every device's image
        of one key comes from the same all-reduced sums."""
        with self.lock:
            self.host.pop(key, None)
            self.images[(key, str(device))] = img
            self._touch(key)

    def _touch(self, key):
        if key in self.order:
            self.order.remove(key)
        self.order.append(key)
        while len(self.order) > self.keep:
            old = self.order.pop(0)
            self.host.pop(old, None)
            for k in [k for k in self.images if k[0] == old]:
                self.images.pop(k)

    def host_centroids(self, key):
        with self.lock:
            c = self.host.get(key)
            if c is not None:
                return c
            for (k, _dev), img in self.images.items():
                if k == key:
                    ready = getattr(img, "ready", None)
                    if ready is not None:
                        ready.synchronize()     # built on a reduce's own stream
                    c = img.cen.detach().to("cpu")
                    self.host[key] = c
                    return c
        return None

    def image(self, key, device):
        from ..ops import kmeans as km
        with self.lock:
            img = self.images.get((key, str(device)))
        if img is not None:
            return img
        cen = self.host_centroids(key)
        if cen is None:
            raise KeyError(f"centroids {key!r} not resident on this tracker")
        img = km.CentroidImage(cen, device)
        if img.cen.is_cuda:
            # built on the caller's stream: consumers on other streams wait on it
            img.ready = torch.cuda.Event()
            img.ready.record()
        self.put_image(key, device, img)
        return img


STORE = CentroidStore()


def _centroid_file(cdir, key):
    return os.path.join(cdir, key.replace("/", "_").replace(":", "_") + ".npy")


def _save_centroids(cdir, key, cen):
    """Commit centroid version ``key`` to the centroid directory before the
    reduce reports success (the DistributedCache side file of the next
    iteration): a tracker whose GPU worker restarts re-localises it from here,
    so it must exist once the job counts as done — an asynchronous writer could
    die with its worker first.  Runs after the reduce's host sync, when the
    next iteration's maps are already on the device."""
    host = cen.detach().to("cpu", torch.float32).numpy()
    os.makedirs(cdir, exist_ok=True)
    path = _centroid_file(cdir, key)
    tmp = path + ".tmp.npy"
    np.save(tmp, host)
    os.replace(tmp, path)
    old = _SAVED.setdefault(cdir, [])
    old.append(path)
    while len(old) > 3:
        try:
            os.remove(old.pop(0))
        except OSError:
            pass


_SAVED: dict = {}
_PINNED_INFLIGHT: list = []     # (event, pinned host buffer) of in-flight split loads


# --------------------------------------------------------------------------- the job
def _sum_slabs(outs):
    """Sum of per-task (sums, counts) partials.  A batch's tasks are views
    [i] of one [B, k, dp] slab (map_gpu_batch): a batch whose every view is
    present is reduced straight from its slab, without first stacking copies
    of the views; anything else is stacked."""
    groups: dict = {}
    loose = []
    for s, c in outs:
        bs, bc = s._base, c._base
        if bs is not None and bc is not None and bs.dim() == 3 and bc.dim() == 2 and \
                tuple(s.shape) == tuple(bs.shape[1:]) and tuple(c.shape) == tuple(bc.shape[1:]):
            g = groups.setdefault(id(bs), [bs, bc, 0, []])
            g[2] += 1
            g[3].append((s, c))
        else:
            loose.append((s, c))
    parts_s, parts_c = [], []
    for bs, bc, n, members in groups.values():
        if n == bs.shape[0] and len({m[0].data_ptr() for m in members}) == n:
            parts_s.append(bs.sum(0))
            parts_c.append(bc.sum(0))
        else:
            loose.extend(members)
    if loose:
        parts_s.append(torch.stack([s for s, _ in loose]).sum(0))
        parts_c.append(torch.stack([c for _, c in loose]).sum(0))
    sums, counts = parts_s[0], parts_c[0]
    for s, c in zip(parts_s[1:], parts_c[1:]):
        sums = sums + s
        counts = counts + c
    return sums, counts


_EXACT_STATS: dict = {}
_EXACT_LOCK = threading.Lock()

# Reference partitions of the delta combiner, per (split, device, k, dp,
# fx_shift, exact) in this (worker) process; least recently used first.  A
# baseline is a pure function of the split's points and a labelling, so it is
# valid for any job over the same split whatever its centroids.
_BASELINES: "dict" = {}
_BASE_LOCK = threading.Lock()
_BASE_MAX = 4096


def _baseline_plan(ctxs, datas, k, dp, fx, exact, enabled):
    """Split a batch into tasks with a usable baseline (delta path), tasks that
    get one from this batch (direct combiner, then installed) and the rest
    (direct combiner only: a second attempt of a split in the same batch)."""
    have, new, plain = [], [], []
    bases, keys = [], []
    seen = set()
    dev = str(ctxs[0].device)
    with _BASE_LOCK:
        for i, (c, d) in enumerate(zip(ctxs, datas)):
            sp = c.spec.split
            sk = sp.get("key") if enabled and isinstance(sp, dict) else None
            key = None if sk is None else (sk, dev, k, dp, fx, exact)
            keys.append(key)
            if key is None or key in seen:
                plain.append(i)
                bases.append(None)
                continue
            seen.add(key)
            b = _BASELINES.get(key)
            x = d.xb if exact else d
            if b is not None and b.data_ptr == x.data_ptr() and b.n == x.shape[0]:
                have.append(i)
                bases.append(b)
            else:
                new.append(i)
                bases.append(None)
    return have, new, plain, bases, keys


def _baseline_bytes(b) -> int:
    return sum(t.numel() * t.element_size() for t in (b.g, b.S0, b.N0) if t is not None)


def _drop_baselines(split_key, device):
    """Split-cache eviction listener: the split's reference partitions go with
    it (their HBM was charged to the split's cache entry)."""
    dev = f"cuda:{device}" if isinstance(device, int) else str(device)
    with _BASE_LOCK:
        for key in [kk for kk in _BASELINES if kk[0] == split_key and kk[1] == dev]:
            _BASELINES.pop(key)


def _install_baselines(entries, stream, cache=None):
    """entries: (key, Baseline) updated or created by a batch just enqueued on
    ``stream``; their event marks its end.  A NEW baseline's device memory is
    charged to its split's entry in the tracker's split cache (``cache``), so
    it counts against hbmr.gpu.hbm.reserve.gb's capacity and is dropped when
    the split is evicted."""
    ev = torch.cuda.Event()
    ev.record(stream)
    charge = []
    with _BASE_LOCK:
        for key, b in entries:
            b.event, b.stream = ev, stream
            old = _BASELINES.pop(key, None)
            _BASELINES[key] = b
            if old is not b:
                charge.append((key, b))
        while len(_BASELINES) > _BASE_MAX:
            _BASELINES.pop(next(iter(_BASELINES)))
    if cache is not None and charge:
        cache.add_listener(_drop_baselines)
        idx = stream.device.index if stream is not None else 0
        for key, b in charge:
            if not cache.charge(key[0], idx, _baseline_bytes(b)):
                # the split is not cache-resident (streamed through): keep no
                # reference partition HBM the cache cannot account for
                with _BASE_LOCK:
                    if _BASELINES.get(key) is b:
                        _BASELINES.pop(key)


def _exact_stats(cin, device):
    """Device counters (flagged, relabelled) of exact mode for one iteration."""
    key = (cin, str(device))
    with _EXACT_LOCK:
        t = _EXACT_STATS.get(key)
        if t is None:
            t = _EXACT_STATS[key] = torch.zeros(3, dtype=torch.int64, device=device)
        return t


class KMeansSplitJob(SplitJob):
    collective_reduce = True
    needs_reduce = True

    def configure(self, conf):
        self.conf = conf
        self.k = conf.get_int(K_KEY, 64)
        self.d = conf.get_int(D_KEY, 128)
        self.input = conf.get(INPUT_KEY, "synthetic:100000:1")
        self.split_points = conf.get_int(SPLIT_PTS_KEY, 500_000)
        self.cin = conf.get(CIN_KEY)
        self.cout = conf.get(COUT_KEY)
        self.centers = conf.get_int(NCENTERS_KEY, self.k)
        self.fx_shift = conf.get_int("hbmr.kmeans.fx.shift", 24)
        self.cdir = conf.get(CDIR_KEY)
        self.exact = conf.get_boolean(EXACT_KEY, False)
        self.exact_dtype = torch.bfloat16 if (conf.get(EXACT_MFMA_KEY) or "f16").lower() in (
            "bf16", "bfloat16") else torch.float16
        self.combiner = (conf.get(COMBINER_KEY) or "delta").lower()
        if self.combiner not in ("delta", "sorted"):
            raise ValueError(f"{COMBINER_KEY} must be delta or sorted, not {self.combiner!r}")
        init = conf.get(INIT_KEY)
        if init and self.cin and STORE.host_centroids(self.cin) is None:
            STORE.put_host(self.cin, decode_centroids(init))
        if self.cin and self.cdir and STORE.host_centroids(self.cin) is None:
            path = _centroid_file(self.cdir, self.cin)
            if os.path.exists(path):
                STORE.put_host(self.cin, torch.from_numpy(np.load(path)))

    # -- splits -------------------------------------------------------------------
    _split_memo: dict = {}

    def get_splits(self, conf, trackers):
        if self.input.startswith("synthetic:"):
            # iteration jobs re-split the same input: reuse the split list
            mk = (self.input, self.split_points, self.d, self.centers, tuple(trackers),
                  self.exact)
            got = KMeansSplitJob._split_memo.get(mk)
            if got is not None:
                return got
            if len(KMeansSplitJob._split_memo) > 16:
                KMeansSplitJob._split_memo.clear()
            out = KMeansSplitJob._split_memo[mk] = self._synthetic_splits(trackers)
            return out
        return self._file_splits(conf, trackers)

    def _synthetic_splits(self, trackers):
        _, n, seed = self.input.split(":")
        n, seed = int(n), int(seed)
        per = self.split_points
        nsplits = max(1, math.ceil(n / per))
        out = []
        for i in range(nsplits):
            a = i * per
            m = min(per, n - a)
            key = f"kmeans-syn:{seed}:{self.d}:{self.centers}:{a}:{m}" + \
                (":exact" if self.exact else "")
            loc = [trackers[i * len(trackers) // nsplits]] if trackers else []
            out.append(SplitSpec(i, key, "synthetic",
                                 {"seed": seed, "start": a, "n": m}, loc, m * self.d * 2))
        return out

    def _file_splits(self, conf, trackers):
        from ..mapred.formats import FileInputFormat, SequenceFileInputFormat
        from ..mapred.jobconf import JobConf
        jc = JobConf(conf)
        FileInputFormat.setInputPaths(jc, self.input)
        fmt = SequenceFileInputFormat()
        nmaps = max(1, conf.get_int("mapred.map.tasks", 1))
        if conf.get_long("mapred.min.split.size", 0) <= 1 and "://" not in self.input:
            # a local file's block size means nothing here: splits are sized to
            # stay HBM-resident, about input / mapred.map.tasks each (as the
            # synthetic splits are), not one per 32-64 MiB block
            total = sum(f.length for f in fmt.list_status(jc))
            jc.set_long("mapred.min.split.size", max(1, -(-total // nmaps)))
        splits = fmt.getSplits(jc, nmaps)
        out = []
        for i, s in enumerate(splits):
            key = f"kmeans-file:{s.path}:{s.start}:{s.length}" + (":exact" if self.exact else "")
            loc = [trackers[i % len(trackers)]] if trackers else []
            out.append(SplitSpec(i, key, "file", {"path": s.path, "start": s.start,
                                                  "length": s.length}, loc, s.length))
        return out

    def _load_raw(self, spec: SplitSpec, device):
        if spec.kind == "synthetic":
            p = spec.params
            return synthetic_points(p["seed"], p["start"], p["n"], self.d, self.centers, device)
        return self._load_file_split(spec.params, device)

    def _load_fp32(self, spec: SplitSpec, device):
        # bf16 is the storage precision of the points on every slot type
        return self._load_raw(spec, device).to(torch.bfloat16)

    def split_nbytes(self, data) -> int:
        nb = getattr(data, "nbytes", None)
        if callable(nb):
            return int(nb())
        return super().split_nbytes(data)

    def load_split_host(self, spec: SplitSpec):
        """Host half of a file split's load (native decode into pinned memory),
        run by the GPU runtime's loader threads in parallel; None for synthetic
        splits (they are generated on the device)."""
        if spec.kind != "file":
            return None
        from ..io import nativeio
        p = spec.params
        # one pass: size for the most records the byte range can hold (a record
        # is >= 4+4+8+4+4d bytes), decode straight into pinned memory
        n = p["length"] // (20 + 4 * self.d) + 2
        host = torch.empty(n, self.d, dtype=torch.float32,
                           pin_memory=torch.cuda.is_available())
        got = nativeio.read_points_into(p["path"], p["start"], p["length"], host.data_ptr(),
                                        self.d, n)
        return host[:got]

    def load_split_from_host(self, spec: SplitSpec, host, device):
        """Device half: one async H2D on the current stream, bf16 + padding."""
        from ..ops import kmeans as km
        x = host.to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        _PINNED_INFLIGHT.append((ev, host))
        while _PINNED_INFLIGHT and _PINNED_INFLIGHT[0][0].query():
            _PINNED_INFLIGHT.pop(0)
        if self.exact:
            return km.ExactSplit(x, km.padded_dim(self.d), self.exact_dtype)
        xb = x.to(torch.bfloat16)
        dp = km.padded_dim(self.d)
        if dp == self.d:
            return xb.contiguous()
        out = torch.zeros(xb.shape[0], dp, dtype=torch.bfloat16, device=device)
        out[:, :self.d] = xb
        return out

    def _load_file_split(self, p, device):
        """A SequenceFile split → fp32 [n, d] on ``device``: the native reader
        decodes the records straight into pinned host memory, then one
        asynchronous H2D copy on the current (slot) stream."""
        from ..io import nativeio
        n = p["length"] // (20 + 4 * self.d) + 2
        dev = torch.device(device)
        host = torch.empty(n, self.d, dtype=torch.float32, pin_memory=dev.type == "cuda")
        got = nativeio.read_points_into(p["path"], p["start"], p["length"], host.data_ptr(),
                                        self.d, n)
        host = host[:got]
        if dev.type != "cuda":
            return host
        x = host.to(dev, non_blocking=True)
        # the pinned buffer must outlive the copy: keep it until the stream passes
        ev = torch.cuda.Event()
        ev.record()
        _PINNED_INFLIGHT.append((ev, host))
        while _PINNED_INFLIGHT and _PINNED_INFLIGHT[0][0].query():
            _PINNED_INFLIGHT.pop(0)
        return x

    def load_split_sample(self, spec: SplitSpec, device, fraction: float):
        if spec.kind == "synthetic":
            p = dict(spec.params)
            p["n"] = max(1, int(p["n"] * fraction))
            spec = SplitSpec(spec.index, spec.key + f":sample{fraction}", spec.kind, p,
                             spec.locations, spec.length)
            return self.load_split(spec, device)
        return super().load_split_sample(spec, device, fraction)

    def load_split(self, spec: SplitSpec, device):
        from ..ops import kmeans as km
        if self.exact:
            # exact mode keeps the fp32 data: CPU slots compute on it directly,
            # GPU slots hold it beside the bf16 copy
            x = self._load_raw(spec, device)
            if str(device) == "cpu":
                return x.contiguous()
            return km.ExactSplit(x, km.padded_dim(self.d), self.exact_dtype)
        xb = self._load_fp32(spec, device)
        if str(device) == "cpu":
            return xb.to(torch.float32)
        dp = km.padded_dim(self.d)
        if dp == self.d:
            return xb.contiguous()
        out = torch.zeros(xb.shape[0], dp, dtype=torch.bfloat16, device=device)
        out[:, :self.d] = xb
        return out

    # -- map ------------------------------------------------------------------------
    @staticmethod
    def _scratch(ctx, ns, k):
        """Per-(tracker, stream) label + combiner workspace, reused across tasks
        (tasks on one stream are ordered, so reuse is race-free)."""
        from ..ops import kmeans as km
        key = ("kmeans-scratch", str(ctx.device), id(ctx.stream))
        store = ctx.tracker.__dict__.setdefault("_scratch", {})
        ws, labels = store.get(key, (None, None))
        need_lab, need_ws = km.batch_scratch_sizes(ns, k)
        need_ws = max(need_ws, km.delta_workspace_bytes(int(sum(ns)), len(ns), k))
        if ws is None or ws.numel() < need_ws:
            ws = torch.empty(max(need_ws, 1 << 20), dtype=torch.uint8, device=ctx.device)
        if labels is None or labels.numel() < need_lab:
            labels = torch.empty(max(need_lab, 1), dtype=torch.int32, device=ctx.device)
        store[key] = (ws, labels)
        return ws, labels

    def map_gpu(self, ctx, points):
        return self.map_gpu_batch([ctx], [points])[0]

    def map_gpu_batch(self, ctxs, datas):
        st = ctxs[0].stream
        if st is None:
            return self._map_gpu_batch(ctxs, datas)
        with torch.cuda.stream(st):
            return self._map_gpu_batch(ctxs, datas)

    def _map_gpu_batch(self, ctxs, datas):
        """All queued map tasks of this job on one stream, launched by one
        native call per combiner path; each task keeps its own slab.  Splits
        with a reference partition take the delta combiner
        (hbmr_kmeans_map_batch_delta); the others the direct one
        (hbmr_kmeans_map_batch), whose labels become their reference partition."""
        from ..ops import kmeans as km
        ctx = ctxs[0]
        img = STORE.image(self.cin, ctx.device)
        # the image may live on a reduce's stream (pipelined iterations) or on
        # another slot's stream (built from host centroids by its first batch)
        ready = getattr(img, "ready", None)
        if ready is not None:
            torch.cuda.current_stream().wait_event(ready)
        for t in (img.cbf, img.chalf):
            t.record_stream(torch.cuda.current_stream())
        B = len(datas)
        if self.exact:
            return self._map_exact(ctxs, datas, img)
        have, new, plain, bases, keys = _baseline_plan(
            ctxs, datas, self.k, img.dp, img.fx_shift, False, self.combiner == "delta")
        ws, labels = self._scratch(ctx, [d.shape[0] for d in datas], self.k)
        sums = torch.empty(B, self.k, img.dp, dtype=torch.int64, device=ctx.device)
        counts = torch.empty(B, self.k, dtype=torch.int64, device=ctx.device)
        order = have + new + plain
        H = len(have)
        S, N = sums.unbind(0), counts.unbind(0)     # slab views in task order `order`
        out = [None] * B
        for j, i in enumerate(order):
            out[i] = (S[j], N[j])
        installed = []
        if have:
            hb = [bases[i] for i in have]
            km.map_batch_delta([datas[i] for i in have], img, sums[:H], counts[:H], labels, ws,
                               hb, stream=ctx.stream)
            for i, b in zip(have, hb):
                b.S0, b.N0 = out[i]
                installed.append((keys[i], b))
        rest = new + plain
        if rest:
            km.map_batch_gpu([datas[i] for i in rest], img, sums[H:], counts[H:], labels, ws,
                             stream=ctx.stream, zero_outputs=True)
            if new:
                # this batch's labels become the new splits' reference partitions
                # (one allocation for all of them)
                total = sum(datas[i].shape[0] for i in rest)
                gall = labels[:total].clone()
                off = 0
                newset = set(new)
                for i in rest:
                    n = datas[i].shape[0]
                    if keys[i] is not None and i in newset:
                        installed.append((keys[i], km.Baseline(gall[off:off + n], *out[i],
                                                                datas[i].data_ptr(), n)))
                    off += n
        if installed:
            _install_baselines(installed, ctx.stream, getattr(ctx, "split_cache", None))
        for c, d in zip(ctxs, datas):
            c.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, d.shape[0])
        return out

    def _map_exact(self, ctxs, datas, img):
        """Exact mode: per task top-3 assign and certification / fp64 re-score,
        then ONE fp32-row combiner call for the batch (delta against the
        splits' reference partitions where they exist).  The flagged /
        relabelled counts accumulate on the device per (job, device) and are
        reported by the reduce (no host sync here)."""
        from ..ops import kmeans as km
        from ..utils.trace import TRACE
        if TRACE.on:
            TRACE.instant("kmeans.map_exact", n=len(datas))
        ctx = ctxs[0]
        store = ctx.tracker.__dict__.setdefault("_scratch", {})
        scratch = store.setdefault(("kmeans-exact", str(ctx.device), id(ctx.stream)), {})
        stats = _exact_stats(self.cin, ctx.device)
        have, new, plain, bases, keys = _baseline_plan(
            ctxs, datas, self.k, img.dp, img.fx_shift, True, self.combiner == "delta")
        B = len(datas)
        sums = torch.empty(B, self.k, img.dp, dtype=torch.int64, device=ctx.device)
        counts = torch.empty(B, self.k, dtype=torch.int64, device=ctx.device)
        order = have + new + plain
        pos = {i: j for j, i in enumerate(order)}
        H = len(have)
        installed = []
        if have:
            ns = [datas[i].shape[0] for i in have]
            total = sum(ns)
            lab = scratch.get("labcat")
            if lab is None or lab.numel() < total:
                lab = scratch["labcat"] = torch.empty(total, dtype=torch.int32, device=ctx.device)
            need = km.delta_workspace_bytes(total, H, self.k)
            if scratch.get("dws") is None or scratch["dws"].numel() < need:
                scratch["dws"] = torch.empty(need, dtype=torch.uint8, device=ctx.device)
            km.assign_exact_batch([datas[i] for i in have], img, stats, lab, scratch,
                                  stream=ctx.stream)
            hb = [bases[i] for i in have]
            km.delta_combine([datas[i].x32 for i in have], lab, self.k, sums[:H], counts[:H],
                             scratch["dws"], hb, fx_shift=img.fx_shift, stream=ctx.stream)
            for i, b in zip(have, hb):
                b.S0, b.N0 = sums[pos[i]], counts[pos[i]]
                installed.append((keys[i], b))
        for i in new + plain:
            d = datas[i]
            s, c = sums[pos[i]], counts[pos[i]]
            s.zero_()
            c.zero_()
            lab = km.assign_exact(d, img, stats, scratch, stream=ctx.stream)
            need = km.workspace_bytes(d.shape[0], img.k)
            if scratch.get("ws") is None or scratch["ws"].numel() < need:
                scratch["ws"] = torch.empty(max(need, 1 << 20), dtype=torch.uint8,
                                            device=ctx.device)
            km.accumulate(d.x32, lab, img.k, s, c, fx_shift=img.fx_shift, stream=ctx.stream,
                          workspace=scratch["ws"])
            if keys[i] is not None and i in new:
                b = km.Baseline(lab.clone(), s, c, d.xb.data_ptr(), d.shape[0])
                installed.append((keys[i], b))
        if installed:
            _install_baselines(installed, ctx.stream, getattr(ctx, "split_cache", None))
        for c, d in zip(ctxs, datas):
            c.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, d.shape[0])
        return [(sums[pos[i]], counts[pos[i]]) for i in range(B)]

    def map_cpu(self, ctx, points):
        from ..ops import kmeans as km
        cen = STORE.host_centroids(self.cin)
        if cen is None:
            raise KeyError(f"centroids {self.cin!r} not resident")
        sums, counts = km.new_partials(self.k, self.d, "cpu")
        st = [0]
        km.map_split_cpu(points, cen, sums, counts, nthreads=ctx.cpu_threads,
                         fx_shift=self.fx_shift, exact=self.exact, stats=st)
        if self.exact:
            ctx.reporter.incrCounter("KMEANS", "EXACT_FLAGGED_POINTS", st[0])
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, points.shape[0])
        return sums, counts

    def map_sim(self, ctx, points):
        """Simulated GPU slot (hbmr.gpu.simulate): no device, and with
        ``hbmr.gpu.simulate.nodata`` no split either — contributes nothing to
        the partials (the reduce still runs the full-size collective)."""
        if points is None:
            ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, 0)
            return None
        return self.map_cpu(ctx, points)

    # -- combine + reduce -------------------------------------------------------------------
    def combine(self, ctx, outputs):
        from ..ops import kmeans as km
        dev = ctx.device if ctx.device is not None else torch.device("cpu")
        dp = km.padded_dim(self.d) if dev.type == "cuda" else self.d
        outputs = [o for o in outputs if o is not None]   # simulated no-data maps
        if dev.type == "cuda":
            # the slabs were allocated on the slot streams; this (reduce) stream
            # reads them, possibly before those streams are done with the memory
            cur = torch.cuda.current_stream()
            for s, c in outputs:
                if s.is_cuda:
                    s.record_stream(cur)
                    c.record_stream(cur)
        from ..utils.trace import TRACE
        if TRACE.on:
            TRACE.instant("kmeans.combine.recorded", n=len(outputs))
        same = [(s, c) for s, c in outputs if s.device == dev and s.shape[1] == dp]
        other = [(s, c) for s, c in outputs if not (s.device == dev and s.shape[1] == dp)]
        if same:
            sums, counts = _sum_slabs(same)
        else:
            sums = torch.zeros(self.k, dp, dtype=torch.int64, device=dev)
            counts = torch.zeros(self.k, dtype=torch.int64, device=dev)
        for s, c in other:  # e.g. CPU-slot partials on a GPU tracker ([k, d], host)
            sums[:, :s.shape[1]] += s.to(dev, non_blocking=True)
            counts += c.to(dev, non_blocking=True)
        return sums, counts

    def reduce(self, ctx, combined):
        from ..ops import kmeans as km
        from ..utils.trace import TRACE
        sums, counts = combined
        k, dp = sums.shape
        packed = torch.cat([sums.reshape(-1), counts])
        sim = getattr(ctx, "simulated_collective_s", None)
        with TRACE.span("kmeans.allreduce", nbytes=packed.numel() * 8):
            if sim is None:
                ctx.comm.all_reduce(packed)        # exact: int64 over RCCL / gloo
            else:
                # rehearsal without data (hbmr.gpu.simulate.nodata): the device
                # all-reduce is modelled as device time ending at this instant
                ctx.sim_ready = max(time.time(), getattr(ctx, "sim_base", 0.0)) + sim
        sums = packed[:k * dp].view(k, dp)
        counts = packed[k * dp:]
        # exact mode's device counters are read with the shift, after the
        # update is enqueued and the staged maps released (a host read here
        # would wait for every map kernel and leave the device idle until the
        # update and the next job's maps were launched)
        est = _EXACT_STATS.pop((self.cin, str(sums.device)), None) \
            if self.exact and sums.device.type == "cuda" else None
        killed = getattr(ctx, "killed", None)
        if killed is not None and killed():
            raise RuntimeError("reduce killed (collective restart): result not published")
        if sums.device.type == "cuda":
            old = STORE.image(self.cin, sums.device)
            # the previous job's reduce built it on a stream of its own
            # (splitexec._reduce_stream): order the read behind it even where
            # no local map output (which waited on that job's gate) orders it
            ready = getattr(old, "ready", None)
            if ready is not None:
                torch.cuda.current_stream().wait_event(ready)
            img = km.CentroidImage.__new__(km.CentroidImage)
            img.__dict__.update(old.__dict__)
            img.cen = old.cen.clone()
            img.cbf = old.cbf.clone()
            img.chalf = old.chalf.clone()
            img.shift2 = torch.zeros_like(old.shift2)
            img.refresh(sums, counts)
            if self.exact:
                # the 16-bit operand image and the centroid neighbour table
                # (one native kernel each) the next job's first kernels read:
                # built here, behind the update, so the gate's event covers them
                img.image16(self.exact_dtype)
                img.neighbors()
            img.ready = torch.cuda.Event()
            img.ready.record()
            # the host copy of the new centroids (rank 0's saved version, the
            # returned centroids) is enqueued now, right behind the update: on
            # the tracker's shared reduce stream a later read-back would queue
            # behind the next job's combine, which waits for that job's maps —
            # this job then finished a whole iteration late
            host_cen = cen_ev = None
            if ctx.rank == 0 and (self.cdir or self.conf.get_boolean(RETURN_KEY, False)):
                host_cen = torch.empty(tuple(img.cen.shape), dtype=torch.float32,
                                       pin_memory=True)
                host_cen.copy_(img.cen, non_blocking=True)
                cen_ev = torch.cuda.Event()
                cen_ev.record()
            if TRACE.on:
                TRACE.instant("kmeans.refresh_launched")
            STORE.put_image(self.cout, sums.device, img)
            # the next iteration's staged maps may go on the device now, behind
            # the update kernel (hbmr/gpu/gates.py); the host sync comes after
            rel = getattr(ctx, "release_dependents", None)
            if rel is not None:
                rel()
            # the shift, the point count (and exact mode's counters) in one
            # device->host copy (one sync)
            vals = [img.shift2.max().double().sqrt(), counts.sum().double()]
            if est is not None:
                vals += list(est.double().unbind(0))
            got = torch.stack(vals).tolist()
            shift, npts = got[0], got[1]
            if est is not None:
                for name, v in zip(("EXACT_FLAGGED_POINTS", "EXACT_RELABELLED_POINTS",
                                    "EXACT_NEIGHBOUR_SCANS"), got[2:5]):
                    ctx.reporter.incrCounter("KMEANS", name, int(v))
            if TRACE.on:
                TRACE.instant("kmeans.shift_synced")
            new_cen = None
        else:
            host_cen = cen_ev = None
            old = STORE.host_centroids(self.cin)
            if sim is not None:
                # no-data rehearsal: every partial is zero, the centroids stay
                # (the device's update kernel is part of the modelled time)
                new_cen, shift, npts = old, 0.0, 0
            else:
                cnt = counts.to(torch.float64)[:, None]
                s = sums[:, :self.d].to(torch.float64) / float(1 << self.fx_shift)
                new_cen = torch.where(cnt > 0, s / cnt.clamp(min=1),
                                      old.to(torch.float64)).to(torch.float32)
                shift = float((new_cen - old).norm(dim=1).max()) if self.k else 0.0
                npts = int(counts.sum().item())
            STORE.put_host(self.cout, new_cen)
            rel = getattr(ctx, "release_dependents", None)
            if rel is not None:
                rel()
            if sim is not None:
                # the real reduce's host sync on the shift: done when the
                # (simulated) device result is
                delay = ctx.sim_ready - time.time()
                if delay > 0:
                    time.sleep(delay)
        self._write_output(ctx, counts, new_cen)
        if TRACE.on:
            TRACE.instant("kmeans.output_written")
        res = {"shift": shift, "points": int(npts), "centroids_key": self.cout}
        if host_cen is not None:
            cen_ev.synchronize()
        if ctx.rank == 0 and self.cdir:
            cen = new_cen if new_cen is not None else host_cen
            _save_centroids(self.cdir, self.cout, cen[:, :self.d])
        if ctx.rank == 0 and self.conf.get_boolean(RETURN_KEY, False):
            # the new centroids travel back with the result (the client may live
            # in another process than the reduce, e.g. with GPU worker processes)
            cen = new_cen if new_cen is not None else host_cen
            res["centroids"] = encode_centroids(cen[:, :self.d])
        if TRACE.on:
            TRACE.instant("kmeans.reduce_return")
        return res

    def poison_result(self, ctx):
        """Fault injection (hbmr.faultinject.reduce.fail.after.release.attempt):
        publish wrong centroids under this job's output key, as a gang that dies
        mid-update would, before the staged maps are released on them."""
        with STORE.lock:
            host = STORE.host.get(self.cout)
            if host is not None:
                STORE.host[self.cout] = host + 1.0
            for key, img in list(STORE.images.items()):
                if key[0] == self.cout:
                    STORE.images.pop(key)
                    STORE.host[self.cout] = img.cen.detach().to("cpu")[:, :self.d] + 1.0

    def _write_output(self, ctx, counts, new_cen):
        out = self.conf.get("mapred.output.dir")
        if not out:
            return
        import os

        from ..io import sequencefile as seqf
        from ..io.writable import FloatVectorWritable, IntWritable
        cen = new_cen if new_cen is not None else STORE.host_centroids(self.cout)
        W = ctx.world_size
        per = math.ceil(self.k / W)
        lo, hi = ctx.rank * per, min(self.k, (ctx.rank + 1) * per)
        os.makedirs(out, exist_ok=True)
        with seqf.Writer(os.path.join(out, f"part-{ctx.rank:05d}"), IntWritable,
                         FloatVectorWritable) as w:
            for j in range(lo, hi):
                w.append(IntWritable(j), FloatVectorWritable(cen[j].numpy()))


# --------------------------------------------------------------------------- driver
def make_iteration_conf(base, k, d, inp, split_points, cin, cout, init=None,
                        return_centroids=False):
    from ..mapred.jobconf import JobConf
    job = JobConf(base)
    job.set_job_name(f"kmeans {cin}->{cout}")
    job.set("hbmr.splitjob.class", "hbmr.models.kmeans:KMeansSplitJob")
    job.set("hbmr.gpu.mapper.class", "hbmr.models.kmeans:KMeansSplitJob")
    job.set_int(K_KEY, k)
    job.set_int(D_KEY, d)
    job.set(INPUT_KEY, inp)
    job.set_int(SPLIT_PTS_KEY, split_points)
    job.set(CIN_KEY, cin)
    job.set(COUT_KEY, cout)
    job.set("hbmr.job.signature", f"kmeans|{inp}|{k}|{d}|{split_points}")
    if init is not None:
        job.set(INIT_KEY, encode_centroids(init))
    if return_centroids:
        job.set_boolean(RETURN_KEY, True)
    return job


def initial_centroids(inp, k, d, centers=None, exact=False):
    """First k points of the input (deterministic).  The bf16 mode starts from
    their bf16 roundings (the values its image holds); exact mode
    (``hbmr.kmeans.exact``) from the fp32 points themselves."""
    def rnd(x):
        return x if exact else x.to(torch.bfloat16).to(torch.float32)
    if inp.startswith("synthetic:"):
        _, _n, seed = inp.split(":")
        x = synthetic_points(int(seed), 0, k, d, centers or k, "cpu")
        return rnd(x)
    from ..io import sequencefile as seqf
    import os
    path = inp
    if os.path.isdir(path):
        path = os.path.join(path, sorted(f for f in os.listdir(path) if not f.startswith(("_", ".")))[0])
    rows = []
    with seqf.Reader(path) as r:
        while len(rows) < k:
            raw = r.next_raw()
            if raw is None:
                break
            rows.append(np.frombuffer(raw[1][4:], dtype=">f4").astype(np.float32))
    return rnd(torch.from_numpy(np.stack(rows)))


class KMeansDriver:
    """Chains K-Means iteration jobs (what the paper's K-Means driver does with
    separate Hadoop jobs).

    Checkpoint / resume: every iteration's centroids land in ``checkpoint_dir``
    (the reduce writes them asynchronously, the last few are kept) next to a
    ``driver.json`` manifest; :meth:`resume` restarts a run from the newest
    complete centroid file, so a driver that died continues where it stopped."""

    MANIFEST = "driver.json"

    def __init__(self, submit, result_of, conf=None, k=64, d=128, inp="synthetic:100000:1",
                 split_points=500_000, run_id=None, return_centroids=None, checkpoint_dir=None):
        self.submit = submit          # conf -> RunningJob
        self.result_of = result_of    # RunningJob -> reduce result dict
        self.base = conf
        self.k, self.d, self.inp, self.split_points = k, d, inp, split_points
        self.run_id = run_id or f"km{int(time.time() * 1e3) & 0xFFFFFF:x}"
        self.iteration = 0
        self.history = []
        # small models bring their centroids back with every result (cheap);
        # the bench-sized one (k*d = 128K floats) only when asked
        self.return_centroids = (k * d <= 65536) if return_centroids is None else return_centroids
        base_dir = (conf.get("mapred.local.dir") if conf is not None else None) or "/tmp/hbmr-local"
        self.centroid_dir = checkpoint_dir or os.path.join(base_dir, "kmeans-centroids",
                                                           self.run_id)
        self._manifest_written = False
        self.prefetch_delay = 0.005     # s after a job's submission before the next one's
        self._ahead: list = []          # iteration jobs submitted ahead, oldest first

    def _write_manifest(self):
        import json
        os.makedirs(self.centroid_dir, exist_ok=True)
        path = os.path.join(self.centroid_dir, self.MANIFEST)
        with open(path + ".tmp", "w") as f:
            json.dump({"run_id": self.run_id, "k": self.k, "d": self.d, "input": self.inp,
                       "split_points": self.split_points}, f)
        os.replace(path + ".tmp", path)
        self._manifest_written = True

    @classmethod
    def resume(cls, submit, result_of, checkpoint_dir, conf=None, **kw):
        """A driver continuing the run saved in ``checkpoint_dir``: its iteration
        is that of the newest centroid file that loads (a file cut short by a
        crash is skipped for the one before it)."""
        import json
        import re
        with open(os.path.join(checkpoint_dir, cls.MANIFEST)) as f:
            m = json.load(f)
        drv = cls(submit, result_of, conf=conf, k=m["k"], d=m["d"], inp=m["input"],
                  split_points=m["split_points"], run_id=m["run_id"],
                  checkpoint_dir=checkpoint_dir, **kw)
        pat = re.compile(re.escape(_centroid_file("", drv.key(0))[:-len("_0.npy")]) +
                         r"_(\d+)\.npy$")
        found = sorted((int(mm.group(1)), fn) for fn in os.listdir(checkpoint_dir)
                       for mm in [pat.match(fn)] if mm)
        for i, fn in reversed(found):
            try:
                c = torch.from_numpy(np.load(os.path.join(checkpoint_dir, fn)))
            except (OSError, ValueError):
                continue
            if tuple(c.shape) != (drv.k, drv.d):
                continue
            drv.iteration = i
            STORE.put_host(drv.key(i), c.to(torch.float32))
            break
        drv._manifest_written = True
        return drv

    def key(self, i):
        return f"{self.run_id}:{i}"

    def _job_conf(self, i, depends_on=None):
        centers = self.base.get_int(NCENTERS_KEY, self.k) if self.base is not None else None
        exact = self.base.get_boolean(EXACT_KEY, False) if self.base is not None else False
        init = initial_centroids(self.inp, self.k, self.d, centers, exact=exact) if i == 0 \
            else None
        if init is not None:
            STORE.put_host(self.key(0), init)
        job = make_iteration_conf(self.base, self.k, self.d, self.inp, self.split_points,
                                  self.key(i), self.key(i + 1), init=init,
                                  return_centroids=self.return_centroids)
        job.set(CDIR_KEY, self.centroid_dir)
        if depends_on is not None:
            from ..mapred.jobtracker import DEPENDS_KEY
            job.set(DEPENDS_KEY, str(depends_on))
        return job

    def step(self, prefetch=False):
        """One iteration job.  ``prefetch`` (True = 1, or a count): keep that
        many next iterations submitted ahead, each depending on the one before
        (hbmr.job.depends.on).  The JobTracker holds each until its predecessor
        succeeds — and stages its GPU maps behind the predecessor's reduce
        (JobTracker._maybe_stage), so consecutive iterations meet on the device
        without a round trip.  A run that stops early kills them
        (cancel_prefetch)."""
        i = self.iteration
        if not self._manifest_written:
            self._write_manifest()
        t0 = time.time()
        ahead = bool(self._ahead)
        rj = self._ahead.pop(0) if ahead else self.submit(self._job_conf(i))
        depth = int(prefetch)
        # a job submitted ahead is staged and launched already: the next one
        # goes in at once (a wait here, as long as a whole job at 8 GPUs, let
        # the chain drain); a job submitted just now gets its own launch under
        # way first, the next one's submission not in its path
        if depth > 0 and len(self._ahead) < depth and \
                (ahead or not rj.waitForCompletion(self.prefetch_delay)):
            last = self._ahead[-1] if self._ahead else rj
            while len(self._ahead) < depth:
                nxt = self.submit(self._job_conf(i + 1 + len(self._ahead),
                                                 depends_on=last.getID()))
                self._ahead.append(nxt)
                last = nxt
        rj.waitForCompletion()
        if not rj.isSuccessful():
            raise RuntimeError(f"K-Means iteration {i} failed: {rj.getFailureInfo()}")
        res = dict(self.result_of(rj) or {})
        jip = getattr(rj._impl, "jip", None)
        if jip is not None:
            res["timeline"] = jip.timeline()
            res["maps_per_tracker"] = jip.maps_per_tracker()
        res.update(iteration=i, seconds=time.time() - t0, job=str(rj.getID()),
                   counters=rj.getCounters())
        self.history.append(res)
        self.iteration += 1
        return res

    def run(self, max_iter=10, tol=0.0):
        for _ in range(max_iter):
            r = self.step()
            if r.get("shift", 1.0) <= tol:
                break
        return self.centroids()

    def cancel_prefetch(self):
        """Kill the iterations submitted ahead (the run stopped before them)."""
        ahead, self._ahead = self._ahead, []
        for nxt in reversed(ahead):
            nxt.killJob()

    def centroids(self):
        c = STORE.host_centroids(self.key(self.iteration))
        if c is None and self.history and self.history[-1].get("centroids"):
            c = decode_centroids(self.history[-1]["centroids"])
            STORE.put_host(self.key(self.iteration), c)
        return c


def main(argv=None, cluster=None):
    """``hbmr examples kmeans --points N --k K --dims D --iters I``."""
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr kmeans")
    ap.add_argument("--input", default=None, help="SequenceFile dir (default: synthetic)")
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--split-points", type=int, default=500_000)
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args(argv)
    from ..mapred.cluster import LocalCluster
    from ..mapred.jobconf import JobConf
    own = cluster is None
    conf = JobConf()
    if own:
        gpus = [[0]] if torch.cuda.is_available() else None
        cluster = LocalCluster(conf, num_trackers=1, gpus=gpus)
    try:
        drv = KMeansDriver(cluster.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf,
                           k=a.k, d=a.dims, inp=a.input or f"synthetic:{a.points}:{a.seed}",
                           split_points=a.split_points)
        for _ in range(a.iters):
            r = drv.step()
            print(f"iteration {r['iteration']}: shift {r['shift']:.6f} "
                  f"({r['seconds'] * 1e3:.1f} ms)")
        return 0
    finally:
        if own:
            cluster.shutdown()
