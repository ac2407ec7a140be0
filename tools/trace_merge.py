"""Merge a host trace (HBMR_TRACE=*.jsonl) with a rocprofv3 kernel trace of the
same run into one timeline around the K-Means iteration boundaries.

usage: python tools/trace_merge.py RESULTS.db TRACE.jsonl [--iters N] [--names a,b]

Both use CLOCK_MONOTONIC nanoseconds (rocprofv3 timestamps, perf_counter_ns in
the trace's ``mono_ns``); the offset is checked against the first kernel."""
import argparse
import json
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("trace")
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--names", default="gpu.native,gpu.launch,gpu.complete,tt.reduce.start,"
                    "tt.reduce.gathered,tt.reduce.waited,kmeans.combine.recorded,tt.reduce.combined,tt.reduce.gate_open,gpu.wake,gpu.prep,kmeans.map_exact,kmeans.top3_launch,kmeans.refresh_launched,"
                    "kmeans.shift_synced,tt.reduce.done,jt.job_finished,tt.launch_batch,"
                    "jt.assigned,tt.finish,kmeans.reduce_return")
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, start, end from kernels order by start"
                                         ).fetchall()
    want = set(a.names.split(","))
    host = []
    with open(a.trace) as f:
        for line in f:
            r = json.loads(line)
            if r["name"] in want and "mono_ns" in r:
                host.append((r["mono_ns"], r["name"], r["thread"], r.get("args", {})))
    ups = [i for i, r in enumerate(rows) if "kmeans_update_kernel" in r[0]]
    for k in range(max(1, len(ups) - a.iters), len(ups)):
        lo, hi = rows[ups[k - 1]][2], rows[ups[k]][2]
        ev = [(s, "K", re.sub(r"\(.*", "", n.replace("void ", "").replace(
            "(anonymous namespace)::", ""))[:48], (e - s) / 1e3) for n, s, e in rows
              if lo - 200_000 <= s <= hi]
        ev += [(t, "H", f"{n} [{th}] {args if args else ''}"[:90], 0.0) for t, n, th, args in host
               if lo - 200_000 <= t <= hi]
        ev.sort()
        print(f"--- iteration ending at update #{k} (span {(hi - lo) / 1e6:.2f} ms)")
        for t, kind, name, dur in ev:
            if kind == "K" and dur < 1.0 and "kmeans" not in name:
                continue
            print(f"{(t - lo) / 1e3:10.1f} {kind} {dur:8.1f} {name}")


if __name__ == "__main__":
    main()
