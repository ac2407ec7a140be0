"""Micro-benchmark of the K-Means kernels (assign / accumulate / update).

usage: python tools/kbench_kmeans.py [--cases n:k:d,...] [--reps R]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

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
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="1000000:64:128,12500000:1024:128,100000000:1024:128")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--split", type=int, default=500000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    out = []
    for case in a.cases.split(","):
        n, k, d = map(int, case.split(":"))
        dp = km.padded_dim(d)
        x = torch.randn(n, dp, device=dev, dtype=torch.bfloat16)
        img = km.CentroidImage(torch.randn(k, d, device=dev), dev)
        lab = torch.empty(n, dtype=torch.int32, device=dev)
        sums, cnt = km.new_partials(k, dp, dev)
        t_as, t_as_min = timeit(lambda: km.assign(x, img, labels=lab), a.reps)
        t_ac, t_ac_min = timeit(lambda: km.accumulate(x, lab, k, sums, cnt), a.reps)
        t_lds, _ = timeit(lambda: km.accumulate(x, lab, k, sums, cnt, mode=km.ACCUM_LDS), a.reps)
        t_srt, _ = timeit(lambda: km.accumulate(x, lab, k, sums, cnt, mode=km.ACCUM_SORTED), a.reps)
        t_up, _ = timeit(lambda: img.refresh(sums, cnt), a.reps)
        flops = 2.0 * n * img.k_pad * dp
        r = dict(n=n, k=k, d=d, assign_ms=t_as, assign_min_ms=t_as_min,
                 assign_tflops=flops / (t_as * 1e-3) / 1e12,
                 assign_x_gbps=n * dp * 2 / (t_as * 1e-3) / 1e9,
                 accum_ms=t_ac, accum_min_ms=t_ac_min,
                 accum_x_gbps=n * dp * 2 / (t_ac * 1e-3) / 1e9, update_ms=t_up,
                 accum_lds_ms=t_lds, accum_sorted_ms=t_srt,
                 points_per_s=n / ((t_as + t_ac) * 1e-3))
        if a.split:
            ns = a.split
            def per_split():
                for s0 in range(0, n, ns):
                    xs = x[s0:s0 + ns]
                    ls = lab[s0:s0 + ns]
                    km.assign(xs, img, labels=ls)
                    km.accumulate(xs, ls, k, sums, cnt)
            t_sp, t_sp_min = timeit(per_split, max(2, a.reps // 2))
            r.update(split=ns, per_split_ms=t_sp, per_split_min_ms=t_sp_min,
                     per_split_points_per_s=n / (t_sp * 1e-3))
            # grouped batches of up to 64 splits (the GPU runtime's launch unit)
            views = [x[s0:s0 + ns] for s0 in range(0, n, ns)]
            batches = [views[i:i + 64] for i in range(0, len(views), 64)]
            scratch = []
            for b in batches:
                nl, nw = km.batch_scratch_sizes([v.shape[0] for v in b], k)
                scratch.append((torch.empty(nl, dtype=torch.int32, device=dev),
                                torch.empty(nw, dtype=torch.uint8, device=dev),
                                torch.empty(len(b), k, dp, dtype=torch.int64, device=dev),
                                torch.empty(len(b), k, dtype=torch.int64, device=dev)))

            def grouped():
                for b, (bl, bw, bs, bc) in zip(batches, scratch):
                    km.map_batch_gpu(b, img, bs, bc, bl, bw)
            t_gr, t_gr_min = timeit(grouped, max(2, a.reps // 2))
            r.update(grouped_ms=t_gr, grouped_min_ms=t_gr_min,
                     grouped_points_per_s=n / (t_gr * 1e-3))
            del scratch
        print(json.dumps(r), flush=True)
        out.append(r)
        del x, lab
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
