"""Micro-benchmark of exact K-Means mode's kernels on the bench's data
(synthetic Gaussian mixture, k=1024, d=128, centroids after a few Lloyd
iterations): plain bf16 assign vs top-3 assign, the certification / fp64
re-score (with its flagged / relabelled / neighbour-scan counts), and the
fp32 vs bf16 combiner — where exact mode's extra time per iteration goes.

usage: python tools/kbench_exact.py [--points N] [--split S] [--iters I]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hbmr.models import kmeans as K  # noqa: E402
from hbmr.ops import kmeans as km  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return round(ts[len(ts) // 2], 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=12_500_000)
    ap.add_argument("--split", type=int, default=781_250)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3, help="Lloyd iterations before timing")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--nbr", type=int, default=0, help="neighbour list length (0: default)")
    ap.add_argument("--dtypes", default="f16,bf16", help="MFMA operand types to time")
    a = ap.parse_args()
    dev = torch.device("cuda")
    if a.nbr:
        os.environ["HBMR_KMEANS_NBR_L"] = str(a.nbr)
    n, k, d = a.points, a.k, a.d
    dp = km.padded_dim(d)
    x32 = K.synthetic_points(7, 0, n, d, k, dev)
    img = km.CentroidImage(K.initial_centroids("synthetic:%d:7" % n, k, d), dev)
    xb = torch.zeros(n, dp, dtype=torch.bfloat16, device=dev)
    xb[:, :d] = x32.to(torch.bfloat16)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(a.iters):
        sums, cnt = km.new_partials(k, dp, dev)
        km.assign(xb, img, labels=lab)
        km.accumulate(xb, lab, k, sums, cnt)
        img.refresh(sums, cnt)
    for name in a.dtypes.split(","):
        dt = torch.float16 if name == "f16" else torch.bfloat16
        r = run_dtype(a, n, k, d, dp, x32, img, xb, lab, dt)
        r["mfma_dtype"] = name
        print(json.dumps(r), flush=True)


def run_dtype(a, n, k, d, dp, x32, img, xb, lab, dt):
    dev = x32.device
    splits = [km.ExactSplit(x32[s:s + a.split], dp, dt) for s in range(0, n, a.split)]
    bsplits = [xb[s:s + a.split] for s in range(0, n, a.split)]
    torch.cuda.synchronize()
    stats = torch.zeros(5, dtype=torch.int64, device=dev)
    bufs = {}

    def plain():
        for s in bsplits:
            km.assign(s, img, labels=lab[:s.shape[0]])

    def top3():
        for s in splits:
            m = s.shape[0]
            key = ("b", m)
            if key not in bufs:
                bufs[key] = (torch.empty(m, dtype=torch.int32, device=dev),
                             torch.empty(2 * m, dtype=torch.int32, device=dev),
                             torch.empty(m, dtype=torch.float32, device=dev),
                             torch.empty(2 * m, dtype=torch.float32, device=dev))
            km.assign_top3(s.xb, img, *bufs[key])

    def top3_refine():
        for s in splits:
            m = s.shape[0]
            b = bufs[("b", m)]
            km.assign_top3(s.xb, img, *b)
            km.refine_f32(s, img, *b, stats)

    bscratch = {}
    labcat = torch.empty(n, dtype=torch.int32, device=dev)

    def batch():
        km.assign_exact_batch(splits, img, stats, labcat, bscratch)

    sums, cnt = km.new_partials(k, dp, dev)

    def acc32():
        for s in splits:
            km.accumulate(s.x32, lab[:s.shape[0]], k, sums, cnt)

    def acc16():
        for s in bsplits:
            km.accumulate(s, lab[:s.shape[0]], k, sums, cnt)

    r = {"points": n, "k": k, "d": d, "split": a.split, "lloyd_iters": a.iters,
         "nbr_l": img.neighbors()[2]}
    r["assign_bf16_ms"] = timeit(plain, a.reps)
    r["assign_top3_ms"] = timeit(top3, a.reps)
    stats.zero_()
    r["top3_plus_refine_ms"] = timeit(top3_refine, a.reps)
    runs = a.reps + 1
    f, rl, sc, ev, full = (int(v) // runs for v in stats.tolist())
    r.update(refine_ms=round(r["top3_plus_refine_ms"] - r["assign_top3_ms"], 3),
             flagged_frac=round(f / n, 5), relabelled_frac=round(rl / n, 6),
             neighbour_scan_frac=round(sc / n, 6),
             neighbours_per_scan=round(ev / max(1, sc), 1),
             full_scan_frac=round(full / max(1, sc), 4))
    r["exact_batch_ms"] = timeit(batch, a.reps)
    r["accum_f32_ms"] = timeit(acc32, a.reps)
    r["accum_bf16_ms"] = timeit(acc16, a.reps)
    del splits
    return r


if __name__ == "__main__":
    main()
