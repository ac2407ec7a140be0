"""A/B of the fused exact top-3 assign kernels (v2 vs v3 of
native/kernels/kmeans.hip, selected in-process by hbmr_kmeans_set_exact_kernel)
on the bench's data: 12.5M points x 128-d, k=1024, after a few Lloyd
iterations.  For each kernel: the exact batch time (top-3 assign with step 1
fused + step 2 + neighbour scan), and the labels and certification
statistics, which must equal v2's exactly (the MFMA accumulation order and
the epilogue arithmetic are the same).

usage: python tools/kbench_v3.py [--modes v2,v3] [--points N] [--reps R]
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
    return round(ts[len(ts) // 2], 3), round(ts[0], 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=12_500_000)
    ap.add_argument("--split", type=int, default=781_250)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--modes", default="v2,v3")
    a = ap.parse_args()
    dev = torch.device("cuda")
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
    del xb
    splits = [km.ExactSplit(x32[s:s + a.split], dp, torch.float16) for s in range(0, n, a.split)]
    torch.cuda.synchronize()
    ref = None
    ref_stats = None
    scratch = {}
    lib = km._lib.load()
    for mode in a.modes.split(","):
        lib.hbmr_kmeans_set_exact_kernel(2 if mode == "v2" else 3)
        out = torch.full((n,), -1, dtype=torch.int32, device=dev)
        stats = torch.zeros(5, dtype=torch.int64, device=dev)

        def batch():
            km.assign_exact_batch(splits, img, stats, out, scratch)

        try:
            stats.zero_()
            batch()
            torch.cuda.synchronize()
            st1 = stats.tolist()
            lab_mode = out.clone()
            med, best = timeit(batch, a.reps)
        except Exception as e:  # noqa: BLE001 — report and go on to the next mode
            print(json.dumps({"mode": mode, "error": str(e)[:200]}), flush=True)
            continue
        r = {"mode": mode, "exact_batch_ms": med, "best_ms": best,
             "ms_per_12.5M": round(med * 12_500_000 / n, 3), "stats": st1}
        if ref is None:
            ref, ref_stats = lab_mode, st1
        else:
            r["labels_equal_v2"] = bool(torch.equal(ref, lab_mode))
            r["stats_equal_v2"] = st1 == ref_stats
        print(json.dumps(r), flush=True)
    lib.hbmr_kmeans_set_exact_kernel(-1)


if __name__ == "__main__":
    main()
