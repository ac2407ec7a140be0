"""How much does the TeraSort reduce's 100-byte record gather depend on where
its sources lie?  Gathers 12.5M records (one ~1.2 GB partition group) by a
random permutation from sources spread over 1.25 / 5 / 25 / 100 GB of
HBM-resident splits (10M-row splits), with and without the packed-index
indirection, and reports ms and effective GB/s (record bytes moved both ways).

    python tools/bench_gather_locality.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hbmr.ops import sort as S
    dev = torch.device("cuda")
    rows, n = 10_000_000, 12_500_000
    nsplits = 100
    bases = [torch.empty(rows, 100, dtype=torch.uint8, device=dev) for _ in range(nsplits)]
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    from hbmr.ops import _lib
    lib = _lib.load()
    for u in (1, 2, 4, 8):
        lib.hbmr_gather_set_unroll(u)
        s = torch.randint(0, nsplits, (n,), device=dev, generator=g, dtype=torch.int64)
        r = torch.randint(0, rows, (n,), device=dev, generator=g, dtype=torch.int64)
        gid = ((s << 24) | r).to(torch.int32)
        ts = []
        for rep in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            S.gather_records_gid(bases, gid)
            torch.cuda.synchronize()
            if rep:
                ts.append(time.perf_counter() - t0)
        ms = 1e3 * sorted(ts)[len(ts) // 2]
        out[f"unroll{u}"] = {"ms": round(ms, 3), "GBps": round(2 * n * 100 / ms / 1e6, 1)}
    lib.hbmr_gather_set_unroll(-1)
    # a plain streaming copy of the same bytes, for the ceiling
    src = bases[0][:n]
    dstb = torch.empty_like(src)
    ts = []
    for rep in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dstb.copy_(src)
        torch.cuda.synchronize()
        if rep:
            ts.append(time.perf_counter() - t0)
    ms = 1e3 * sorted(ts)[len(ts) // 2]
    out["copy_same_bytes"] = {"ms": round(ms, 3), "GBps": round(2 * n * 100 / ms / 1e6, 1)}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
