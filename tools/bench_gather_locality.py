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
    for span in (1, 2, 10, 100):     # splits the sources come from (x 1 GB)
        s = torch.randint(0, span, (n,), device=dev, generator=g, dtype=torch.int64)
        r = torch.randint(0, rows, (n,), device=dev, generator=g, dtype=torch.int64)
        gid = ((s << 24) | r).to(torch.int32)
        order = torch.randperm(n, device=dev, generator=g).to(torch.int64)
        for mode in ("gid", "order"):
            ts = []
            for rep in range(6):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if mode == "gid":
                    S.gather_records_gid(bases, gid)
                else:
                    S.gather_records_gid(bases, gid, order=order)
                torch.cuda.synchronize()
                if rep:
                    ts.append(time.perf_counter() - t0)
            ms = 1e3 * sorted(ts)[len(ts) // 2]
            out[f"{span}GB_{mode}"] = {"ms": round(ms, 3), "GBps": round(2 * n * 100 / ms / 1e6, 1)}
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
