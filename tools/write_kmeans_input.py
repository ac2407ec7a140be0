"""Write the bench's synthetic K-Means input as SequenceFiles: the same
counter-based Gaussian mixture bench.py generates in HBM (point p, dim j
depends only on (seed, p, j)), one file per split of ``--split-points``
points, as <LongWritable id, float[d]> records (the native writer).  The data
is generated on a GPU when one is visible, else on the CPU.

    python tools/write_kmeans_input.py --dir /tmp/km100m     # 100M x 128, k=1024 centres
    python bench.py --input /tmp/km100m                      # the same bench over the files
"""
import argparse
import concurrent.futures as cf
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--centers", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--split-points", type=int, default=781_250)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import torch

    from hbmr.io import nativeio
    from hbmr.models.kmeans import synthetic_points
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    os.makedirs(a.dir, exist_ok=True)
    nsplits = -(-a.points // a.split_points)
    t0 = time.perf_counter()
    pool = cf.ThreadPoolExecutor(a.threads)
    pending = []
    for i in range(nsplits):
        s = i * a.split_points
        m = min(a.split_points, a.points - s)
        x = synthetic_points(a.seed, s, m, a.dims, a.centers, dev).to("cpu").numpy()
        pending.append(pool.submit(nativeio.write_points,
                                   os.path.join(a.dir, f"part-{i:05d}"), x, s))
        while len(pending) > 2 * a.threads:
            pending.pop(0).result()
    for f in pending:
        f.result()
    pool.shutdown()
    nbytes = sum(os.path.getsize(os.path.join(a.dir, f)) for f in os.listdir(a.dir))
    print(f"wrote {nsplits} files, {nbytes / 1e9:.2f} GB in {time.perf_counter() - t0:.1f} s",
          flush=True)


if __name__ == "__main__":
    main()
