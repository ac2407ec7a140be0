"""Delta-combiner micro-benchmark: one batch of B splits (exact mode's fp32
rows), labels alternating between two labellings that differ in ``churn`` of
the points, so every call sees the same number of movers.

usage: python tools/kbench_delta.py [--splits 16] [--n 781250] [--k 1024] [--churn 0.01]
Prints one JSON line (ms per delta_combine call)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hbmr.ops import kmeans as km  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", type=int, default=16)
    ap.add_argument("--n", type=int, default=781250)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dp", type=int, default=128)
    ap.add_argument("--churn", type=float, default=0.01)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    B, n, k, dp = a.splits, a.n, a.k, a.dp
    xs = [torch.randn(n, dp, device=dev, generator=g) * 3 for _ in range(B)]
    l1 = torch.randint(0, k, (B * n,), device=dev, generator=g, dtype=torch.int32)
    move = torch.rand(B * n, device=dev, generator=g) < a.churn
    l2 = torch.where(move, torch.randint(0, k, (B * n,), device=dev, generator=g,
                                         dtype=torch.int32), l1)
    sums = torch.empty(B, k, dp, dtype=torch.int64, device=dev)
    counts = torch.empty(B, k, dtype=torch.int64, device=dev)
    ws = torch.empty(km.delta_workspace_bytes(B * n, B, k), dtype=torch.uint8, device=dev)
    # reference partitions for l1 (exact partials from the direct combiner)
    bases = []
    for t in range(B):
        s0 = torch.zeros(k, dp, dtype=torch.int64, device=dev)
        c0 = torch.zeros(k, dtype=torch.int64, device=dev)
        lab = l1[t * n:(t + 1) * n].clone()
        km.accumulate(xs[t], lab, k, s0, c0)
        bases.append(km.Baseline(lab, s0, c0, xs[t].data_ptr(), n))
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for r in range(a.reps):
        lab = l2 if r % 2 == 0 else l1
        ev[0].record()
        km.delta_combine(xs, lab, k, sums, counts, ws, bases)
        ev[1].record()
        ev[1].synchronize()
        times.append(ev[0].elapsed_time(ev[1]))
        for t, b in enumerate(bases):
            b.S0, b.N0 = sums[t].clone(), counts[t].clone()
    moved = int((l1 != l2).sum())
    print(json.dumps({"splits": B, "n": n, "k": k, "dp": dp, "movers": moved,
                      "ms_min": round(min(times[2:]), 4),
                      "ms_median": round(sorted(times[2:])[len(times[2:]) // 2], 4)}))


if __name__ == "__main__":
    main()
