"""A/B of the exact top-3 assign kernels on the bench's data (12.5M points x
128-d, k = 1024, after a few Lloyd iterations), interleaved in one process:

* ``fused``: the default v3 kernel with certification step 1 in its epilogue;
* ``v2``:    the grouped v2 top-3 kernel + the separate step-1 scan;
* ``v4``:    the v4 kernel (stationary centroids, streamed points) + step 1.

Per arm: the whole exact batch (assign + certification + fp64 re-score) and
the top-3 kernel alone.  The certified labels of every arm must be equal (they
are the fp64 arg-min); the flagged counts differ (different packing / tracks).

usage: python tools/kbench_v4.py [--arms fused,v2,v4] [--rounds R]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hbmr.models import kmeans as K  # noqa: E402
from hbmr.ops import kmeans as km  # noqa: E402


def elapsed(fn):
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=12_500_000)
    ap.add_argument("--split", type=int, default=781_250)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--arms", default="fused,v2,v4")
    ap.add_argument("--stamps", action="store_true",
                    help="also run the v4 stamped diagnostic build (cycle shares per step phase)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    n, k, d = a.points, a.k, 128
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
    lib = km._lib.load()
    scratch = {}
    arms = a.arms.split(",")
    outs = {m: torch.full((n,), -1, dtype=torch.int32, device=dev) for m in arms}
    stats = {m: torch.zeros(5, dtype=torch.int64, device=dev) for m in arms}
    # raw top-3 kernel (unfused grouped launch) buffers
    B = len(splits)
    ns = [sp.shape[0] for sp in splits]
    P = ctypes.c_void_p * B
    xs = P(*[sp.xb.data_ptr() for sp in splits])
    nsa = (ctypes.c_long * B)(*ns)
    c16, ch = img.image16(torch.float16)[:2]
    lab3 = torch.empty(n, dtype=torch.int32, device=dev)
    cand = torch.empty(2 * n, dtype=torch.int32, device=dev)
    sc = torch.empty(n, device=dev)
    mg = torch.empty(2 * n, device=dev)

    def setup(m):
        km.FUSED_Q1 = m == "fused"
        lib.hbmr_kmeans_set_exact_v4(1 if m == "v4" else 0)

    def batch(m):
        km.assign_exact_batch(splits, img, stats[m], outs[m], scratch)

    def top3(m):
        rc = lib.hbmr_kmeans_assign_top3_grouped(B, xs, nsa, dp, 1, c16.data_ptr(), ch.data_ptr(),
                                                 img.k_pad, lab3.data_ptr(), cand.data_ptr(),
                                                 sc.data_ptr(), mg.data_ptr(), None)
        km._lib.check(rc, "top3")

    times = {m: {"batch": [], "top3": []} for m in arms}
    for m in arms:                       # warm-up + the labels / stats of one call
        setup(m)
        batch(m)
        torch.cuda.synchronize()
        st1 = stats[m].tolist()
        stats[m].zero_()
        times[m]["stats"] = st1
    for _ in range(a.rounds):
        for m in arms:
            setup(m)
            times[m]["batch"].append(elapsed(lambda: batch(m)))
            if m != "fused":
                times[m]["top3"].append(elapsed(lambda: top3(m)))
    if a.stamps:
        buf = torch.zeros(256 * 8 * 4, dtype=torch.int64, device=dev)
        lib.hbmr_kmeans_set_v4_stamps(ctypes.c_void_p(buf.data_ptr()))
        lib.hbmr_kmeans_set_exact_v4(2)
        top3("v4")
        torch.cuda.synchronize()
        lib.hbmr_kmeans_set_v4_stamps(None)
        v = buf.view(-1, 4)
        v = v[v[:, 3] > 0].double()
        names = ["dma_wait", "barrier", "work", "total"]
        med = {nm: float(v[:, i].median()) for i, nm in enumerate(names)}
        steps = -(-((n + 31) // 32) // 256)
        print(json.dumps({"v4_stamps_cycles_per_step": {k: round(x / steps, 1) for k, x in med.items()},
                          "shares": {k: round(med[k] / med["total"], 3) for k in names[:3]},
                          "waves": int(v.shape[0])}), flush=True)
    lib.hbmr_kmeans_set_exact_v4(-1)
    km.FUSED_Q1 = True
    ref = outs[arms[0]]
    for m in arms:
        r = {"arm": m, "stats_one_call": times[m]["stats"]}
        for key in ("batch", "top3"):
            ts = sorted(times[m][key])
            if ts:
                r[key + "_ms_median"] = round(ts[len(ts) // 2], 3)
                r[key + "_ms_min"] = round(ts[0], 3)
        r["labels_equal_" + arms[0]] = bool(torch.equal(ref, outs[m]))
        if m != "fused":
            flops = 2.0 * n * img.k_pad * dp
            r["top3_pflops"] = round(flops / (r["top3_ms_median"] * 1e-3) / 1e15, 3)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
