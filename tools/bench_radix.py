"""Micro-benchmark of the device radix sort (native/kernels/sort.hip).

Sorts N random (uint64 key, uint32 value) pairs over 64 key bits (8 passes)
and reports ms per sort and the effective per-pass bandwidth (a pass reads and
writes 12 B per pair and the histogram reads 8 B more).  Checks the result
against a stable numpy argsort on the host.  ``HBMR_RADIX_V1=1`` selects the
round-1 kernels (the switch is read once per process).

    python tools/bench_radix.py --n 100000000 --reps 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--bits", type=int, default=64)
    ap.add_argument("--check", type=int, default=10_000_000, help="check the first sort up to N")
    ap.add_argument("--skew", action="store_true", help="keys with 3 distinct low bytes")
    a = ap.parse_args()
    import numpy as np
    import torch
    from hbmr.ops import sort as S

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    keys = torch.randint(-(1 << 62), 1 << 62, (a.n,), dtype=torch.int64, device=dev, generator=g)
    if a.skew:
        keys = (keys & ~0xFF) | (keys & 0x3) % 3
    vals = torch.arange(a.n, dtype=torch.int32, device=dev)
    if a.check and a.n <= a.check:
        k, v = keys.clone(), vals.clone()
        S.radix_sort_pairs(k, v, 0, a.bits)
        kh = keys.cpu().numpy().view(np.uint64)
        order = np.argsort(kh, kind="stable")
        ok = bool((k.cpu().numpy().view(np.uint64) == kh[order]).all() and
                  (v.cpu().numpy() == order.astype(np.int32)).all())
        if not ok:
            print(json.dumps({"error": "radix sort mismatch"}))
            return 1
    times = []
    for r in range(a.reps + 1):
        k, v = keys.clone(), vals.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        S.radix_sort_pairs(k, v, 0, a.bits)
        torch.cuda.synchronize()
        if r:
            times.append(time.perf_counter() - t0)
    ms = 1e3 * min(times)
    passes = -(-a.bits // 8)
    print(json.dumps({"n": a.n, "bits": a.bits, "kernels": "v1" if os.environ.get("HBMR_RADIX_V1") == "1"
                      else "v2", "skew": a.skew, "ms_per_sort": round(ms, 3),
                      "ms_per_pass": round(ms / passes, 3),
                      "pass_gb_per_s": round(32 * a.n / (ms / passes * 1e-3) / 1e9, 1),
                      "checked": bool(a.check and a.n <= a.check)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
