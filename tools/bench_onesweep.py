"""A/B of the TeraSort reduce's radix sort (native/kernels/sort.hip) on one
group's worth of keys: the pairs sort (uint64 hi + uint32 record id, per-pass
histogram + scan + scatter) over a 40-bit window — the round-5 path — against
the keys-only onesweep sort of packed (32 window bits << 32 | id) keys, and
rocPRIM-free torch.sort as a yardstick.  Checks both against numpy.

    python tools/bench_onesweep.py --n 80000000 --reps 5
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
    ap.add_argument("--n", type=int, default=80_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=4_000_000)
    a = ap.parse_args()
    import numpy as np
    import torch
    from hbmr.ops import sort as S

    dev = torch.device("cuda")
    out = {"n": a.n}
    # correctness on a small case first (the kernels run on what they sort here)
    m = min(a.n, a.check)
    g = torch.Generator(device=dev).manual_seed(3)
    k = torch.randint(-(1 << 62), 1 << 62, (m,), dtype=torch.int64, device=dev, generator=g)
    for lo_b, hi_b in ((32, 64), (0, 64), (3, 29)):
        x = k.clone()
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        S.radix_sort_keys(x, lo_b, hi_b, err=err)
        kh = k.cpu().numpy().view(np.uint64)
        w = hi_b - lo_b
        mask = np.uint64((1 << w) - 1 if w < 64 else 0xFFFFFFFFFFFFFFFF)
        order = np.argsort((kh >> np.uint64(lo_b)) & mask, kind="stable")
        ok = bool((x.cpu().numpy().view(np.uint64) == kh[order]).all()) and int(err.item()) == 0
        out[f"check_{lo_b}_{hi_b}"] = ok
        if not ok:
            print(json.dumps(out), flush=True)
            return 1
    hi = torch.randint(-(1 << 62), 1 << 62, (a.n,), dtype=torch.int64, device=dev, generator=g)
    gid = torch.arange(a.n, dtype=torch.int32, device=dev)
    packed = ((hi >> 24) & 0xFFFFFFFF) << 32 | gid.to(torch.int64)

    def timeit(fn):
        ts = []
        for r in range(a.reps + 1):
            args = fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            args()
            torch.cuda.synchronize()
            if r:
                ts.append(time.perf_counter() - t0)
        return round(1e3 * sorted(ts)[len(ts) // 2], 3)

    def pairs():
        kk, vv = hi.clone(), gid.clone()
        return lambda: S.radix_sort_pairs(kk, vv, 16, 56)

    def onesweep():
        kk = packed.clone()
        return lambda: S.radix_sort_keys(kk, 32, 64)

    def tsort():
        kk = packed.clone()
        return lambda: torch.sort(kk)
    from hbmr.ops import _lib
    lib = _lib.load()
    out["ms_pairs_40bit_5pass"] = timeit(pairs)
    for wv in (4, 8, 16):
        lib.hbmr_radix_set_onesweep_waves(wv)
        x = k.clone()
        S.radix_sort_keys(x, 32, 64)
        kh = k.cpu().numpy().view(np.uint64)
        order = np.argsort(kh >> np.uint64(32), kind="stable")
        out[f"check_waves{wv}"] = bool((x.cpu().numpy().view(np.uint64) == kh[order]).all())
        out[f"ms_onesweep_keys_32bit_4pass_waves{wv}"] = timeit(onesweep)
    lib.hbmr_radix_set_onesweep_waves(-1)
    out["ms_torch_sort_64bit"] = timeit(tsort)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
