"""A/B of the fused exact top-3 assign kernels (v2 vs the v3 modes of
native/kernels/kmeans.hip assign_tile_v3) on the bench's data: 12.5M points x
128-d, k=1024, after a few Lloyd iterations.  For each mode: the exact batch
time (top-3 assign with step 1 fused + step 2 + neighbour scan), and the labels
and certification statistics, which must equal v2's exactly (the MFMA
accumulation order and the epilogue arithmetic are the same).

usage: python tools/kbench_v3.py [--modes v2,0,16,24] [--points N] [--reps R]
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
    ap.add_argument("--modes", default="v2,0,16,18,24,17,20")
    ap.add_argument("--stamps", default="", help="v3 modes with kV3Stamp to time per phase (48)")
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
    for mode in a.modes.split(","):
        os.environ["HBMR_EXACT_V3"] = mode
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
    if a.stamps:
        stamps(a, splits, img, scratch, n)


def stamps(a, splits, img, scratch, n):
    """Per-tile phase cycles of the v3 base kernel (mode 48 = tiled + stamps):
    medians over workgroups < 64, their 4 waves and tiles 4..27."""
    from hbmr.ops import _lib
    dev = splits[0].xb.device
    buf = torch.zeros(64 * 4 * 256, dtype=torch.int32, device=dev)
    _lib.load().hbmr_kmeans_set_stamps(km._ptr(buf))
    for mode in a.stamps.split(","):
        os.environ["HBMR_EXACT_V3"] = mode
        out = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.zeros(5, dtype=torch.int64, device=dev)
        buf.zero_()
        km.assign_exact_batch(splits, img, st, out, scratch)
        torch.cuda.synchronize()
        s = buf.view(64, 4, 32, 8).to(torch.int64).cpu()
        s = (s - s[:, :, :1, :1]) & 0xffffffff          # wrap-safe, per wave
        pair = int(mode) & 64
        names = (["dma_wait", "barrier", "tile_a", "tile_b", "to_next_top"] if pair else
                 ["dma_wait", "barrier", "stage", "mfma_issue", "epilogue", "to_next_top"])
        lo, hi = (2, 14) if pair else (4, 28)
        per = {}
        for i, nm in enumerate(names):
            last = i == len(names) - 1
            nxt = s[:, :, lo + 1:hi + 1, 0] if last else s[:, :, lo:hi, i + 1]
            cur = s[:, :, lo:hi, i]
            per[nm] = int((nxt - cur).median())
        step = s[:, :, lo + 1:hi + 1, 0] - s[:, :, lo:hi, 0]
        per["step_period"] = int(step.median())
        per["tile_period"] = int(step.median()) // (2 if pair else 1)
        per["p10_p90_step"] = [int(v) for v in torch.quantile(
            step.double().flatten(), torch.tensor([0.1, 0.9], dtype=torch.float64))]
        # the wave's share of a phase: medians per phase over every wave and tile
        per["sum_of_medians"] = sum(v for kk, v in per.items() if kk in names)
        print(json.dumps({"stamps_mode": mode, "cycles_per_tile": per}), flush=True)
    _lib.load().hbmr_kmeans_set_stamps(None)


if __name__ == "__main__":
    main()
