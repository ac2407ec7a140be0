"""Mars-style dense matmul as map tasks — BASELINE config 4.

C = A · B with A [M, K] row-split into map tasks and B [K, N] broadcast side
data (the DistributedCache role): each GPU map task multiplies its HBM-resident
row panel of A by the tracker-resident Bᵀ on the MFMA matrix cores
(hbmr.ops.gemm, native/kernels/gemm.hip) and keeps its C panel in HBM; the
collective reduce all-reduces a checksum (and writes the panels if an output
directory is set).  CPU map slots use a float32 torch matmul.

Operands are synthetic: element (i, j) of a matrix is a counter-based hash of
(seed, i, j) mapped to [-1, 1) and rounded to bf16, so any panel is generated
independently and identically on any device.
"""
from __future__ import annotations

import os
import threading

import numpy as np
import torch

from ..gpu.splitjob import SplitJob, SplitSpec
from ..mapred import counters as C
from ..ops import gemm as G

M_KEY, K_KEY, N_KEY = "hbmr.matmul.m", "hbmr.matmul.k", "hbmr.matmul.n"
ROWS_KEY = "hbmr.matmul.split.rows"
SEED_KEY = "hbmr.matmul.seed"
OUTC_KEY = "hbmr.matmul.output.dtype"   # float32 | bfloat16
# GPU GEMM of a map task: "hbmr" (default) = native/kernels/gemm.hip (MFMA,
# hand-written, the checksum fused into its epilogue); "hipblaslt" =
# torch.mm, the vendor library — faster as a bare GEMM (1,366 vs 1,130 TF/s at
# 8192^3 on one box) but slower as the map task (806 vs 899 TF/s for the
# 65536x8192x8192 job: its checksum is a second pass over C,
# profiles/r05_matmul_job_1gpu.json)
GEMM_KEY = "hbmr.matmul.gemm"

_M32 = 0xFFFFFFFF


def _mix(x: torch.Tensor) -> torch.Tensor:
    x = x & _M32
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & _M32
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & _M32
    return x ^ (x >> 16)


def synthetic_matrix(seed: int, row0: int, rows: int, cols: int, device,
                     chunk_rows: int = 4096) -> torch.Tensor:
    """bf16 [rows, cols] with element (i, j) = hash(seed, row0 + i, j) in [-1, 1)."""
    dev = torch.device(device)
    out = torch.empty(rows, cols, dtype=torch.bfloat16, device=dev)
    j = torch.arange(cols, dtype=torch.int64, device=dev)
    s = (seed * 0x9E3779B1) & _M32
    for a in range(0, rows, chunk_rows):
        b = min(rows, a + chunk_rows)
        i = torch.arange(row0 + a, row0 + b, dtype=torch.int64, device=dev)
        h = _mix(_mix(i[:, None] * 0x85EBCA6B + s) ^ (j[None, :] * 0xC2B2AE35))
        out[a:b] = (h.to(torch.float32) * (2.0 / 4294967296.0) - 1.0).to(torch.bfloat16)
    return out


class _SideData:
    """Per-process Bᵀ cache (seed, K, N, device) → bf16 [N, K]."""

    def __init__(self):
        self.lock = threading.Lock()
        self.cache: dict = {}

    def bt(self, seed, k, n, device):
        key = (seed, k, n, str(device))
        with self.lock:
            t = self.cache.get(key)
        if t is None:
            # B[K, N] element (k, n) = hash(seed+1, k, n); store its transpose
            t = synthetic_matrix(seed + 1, 0, k, n, device).t().contiguous()
            with self.lock:
                if len(self.cache) > 4:
                    self.cache.clear()
                self.cache[key] = t
        return t


SIDE = _SideData()


class MatmulSplitJob(SplitJob):
    collective_reduce = True
    needs_reduce = True

    def configure(self, conf):
        self.conf = conf
        self.m = conf.get_long(M_KEY, 8192)
        self.k = conf.get_long(K_KEY, 8192)
        self.n = conf.get_long(N_KEY, 8192)
        self.rows = conf.get_long(ROWS_KEY, 8192)
        self.seed = conf.get_int(SEED_KEY, 1)
        self.out_dtype = torch.bfloat16 if conf.get(OUTC_KEY, "float32") == "bfloat16" \
            else torch.float32
        self.out = conf.get("mapred.output.dir")
        self.gemm = conf.get(GEMM_KEY, "hbmr")
        if self.gemm not in ("hbmr", "hipblaslt"):
            raise ValueError(f"{GEMM_KEY} must be hbmr or hipblaslt, not {self.gemm!r}")

    def get_splits(self, conf, trackers):
        out = []
        nsplit = -(-self.m // self.rows)
        for i in range(nsplit):
            r0 = i * self.rows
            r = min(self.rows, self.m - r0)
            loc = [trackers[i * len(trackers) // nsplit]] if trackers else []
            out.append(SplitSpec(i, f"mm:{self.seed}:{self.k}:{r0}:{r}", "range",
                                 {"row0": r0, "rows": r}, loc, r * self.k * 2))
        return out

    def load_split(self, spec: SplitSpec, device):
        p = spec.params
        return {"row0": p["row0"], "a": synthetic_matrix(self.seed, p["row0"], p["rows"], self.k,
                                                         device)}

    def split_nbytes(self, data):
        return int(data["a"].numel() * 2)

    def _map(self, ctx, data):
        a = data["a"]
        bt = SIDE.bt(self.seed, self.k, self.n, a.device)
        if a.device.type == "cuda" and self.gemm == "hipblaslt":
            # fp32 C straight from the fp32 accumulators (aten::mm.dtype), not
            # a bf16 C widened afterwards
            c = torch.mm(a, bt.t()) if self.out_dtype == torch.bfloat16 else \
                torch.mm(a, bt.t(), out_dtype=torch.float32)
            cs = c.sum(dtype=torch.float64)
        else:
            # the checksum comes out of the GEMM epilogue (no second pass over C)
            c, cs = G.matmul_tn(a, bt, out_dtype=self.out_dtype if a.device.type == "cuda"
                                else torch.float32, with_sum=True)
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, a.shape[0])
        ctx.reporter.incrCounter("hbmr.Matmul", "FLOPS", 2 * a.shape[0] * self.k * self.n)
        return {"row0": data["row0"], "c": c, "checksum": cs}

    def map_gpu(self, ctx, data):
        return self._map(ctx, data)

    def map_cpu(self, ctx, data):
        return self._map(ctx, data)

    def map_gpu_batch(self, ctxs, datas):
        return [self._map(c, d) for c, d in zip(ctxs, datas)]

    def combine(self, ctx, outputs):
        dev = ctx.device if ctx.device is not None else torch.device("cpu")
        cs = torch.zeros(1, dtype=torch.float64, device=dev)
        for o in outputs:
            cs += o["checksum"].to(dev)
        return {"checksum": cs, "parts": [(o["row0"], o["c"]) for o in outputs]}

    def reduce(self, ctx, combined):
        cs = combined["checksum"]
        ctx.comm.all_reduce(cs)
        rows = sum(int(c.shape[0]) for _, c in combined["parts"])
        if self.out:
            os.makedirs(self.out, exist_ok=True)
            for r0, c in combined["parts"]:
                np.save(os.path.join(self.out, f"c-{r0:09d}.npy"), c.float().cpu().numpy())
        return {"checksum": float(cs.item()), "rows": rows}


def matmul_conf(base=None, m=8192, k=8192, n=8192, split_rows=8192, seed=1, output=None,
                out_dtype="float32"):
    from ..mapred.jobconf import JobConf
    job = JobConf(base)
    job.set_job_name(f"matmul {m}x{k}x{n}")
    job.set("hbmr.splitjob.class", "hbmr.models.matmul:MatmulSplitJob")
    job.set_long(M_KEY, m)
    job.set_long(K_KEY, k)
    job.set_long(N_KEY, n)
    job.set_long(ROWS_KEY, split_rows)
    job.set_int(SEED_KEY, seed)
    job.set(OUTC_KEY, out_dtype)
    if output:
        job.set("mapred.output.dir", output)
    return job


def main(argv=None, cluster=None):
    """``hbmr examples matmul --m M --k K --n N --split-rows R``."""
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr matmul")
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--split-rows", type=int, default=2048)
    ap.add_argument("--output", default=None)
    a = ap.parse_args(argv)
    from ..mapred.cluster import LocalCluster
    from ..mapred.jobconf import JobConf
    own = cluster is None
    if own:
        gpus = [[0]] if torch.cuda.is_available() else None
        cluster = LocalCluster(JobConf(), num_trackers=1, gpus=gpus)
    try:
        rj = cluster.submit_job(matmul_conf(m=a.m, k=a.k, n=a.n, split_rows=a.split_rows,
                                            output=a.output))
        rj.waitForCompletion()
        print(rj._impl.jip.result)
        return 0 if rj.isSuccessful() else 1
    finally:
        if own:
            cluster.shutdown()
