"""PiEstimator map throughput: fp64 Halton HIP kernel vs the numpy CPU map."""
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hbmr.ops import pi as P  # noqa: E402


def main():
    n = 1 << 30
    P.count_inside_gpu(0, 1 << 20)
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = P.count_inside_gpu(0, n)
    torch.cuda.synchronize()
    g = time.perf_counter() - t
    m = 1 << 22
    t = time.perf_counter()
    cpu = P.count_inside_cpu(0, m)
    c = time.perf_counter() - t
    assert P.count_inside_cpu(12345, 100000) == int(P.count_inside_gpu(12345, 100000).item())
    inside = int(out.item())
    print(json.dumps({"benchmark": "PiEstimator map (Halton bases 2,3; fp64)",
                      "gpu_points": n, "gpu_s": round(g, 4), "gpu_points_per_s": n / g,
                      "cpu_points": m, "cpu_s": round(c, 4), "cpu_points_per_s": m / c,
                      "speedup": (n / g) / (m / c), "pi_estimate": 4 * inside / n,
                      "cpu_inside_check": cpu}))


if __name__ == "__main__":
    main()
