"""Summarise a rocprofv3 rocpd SQLite result (``--kernel-trace --stats`` run).

usage: python tools/rocpd_summary.py <results.db> [--top N] [--timeline PATTERN]

Prints per-kernel call count / total / mean / min (µs), sorted by total, as a
markdown table (the form committed under ``profiles/``).  ``--timeline``
additionally lists each dispatch whose name matches PATTERN with its start
offset, so gaps between launches are visible.
"""
import argparse
import re
import sqlite3


def load(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels "
                     "order by start").fetchall()
    return rows


def short(name, width=70):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name if len(name) <= width else name[:width - 3] + "..."


def summary(rows, top):
    agg = {}
    for name, s, e, *_ in rows:
        a = agg.setdefault(short(name), [0, 0.0, float("inf")])
        d = (e - s) / 1e3
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
    tot = sum(v[1] for v in agg.values())
    lines = ["| kernel | calls | total µs | mean µs | min µs | % |", "|---|---|---|---|---|---|"]
    for k, (n, t, mn) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"| `{k}` | {n} | {t:.1f} | {t / n:.1f} | {mn:.1f} | {100 * t / tot:.1f} |")
    return "\n".join(lines)


def iterations(rows, end_pat="kmeans_update_kernel",
               map_pat=r"kmeans_(assign|segsum|scatter|hist|delta|slab)"):
    """Per K-Means iteration (delimited by the reduce's update kernel): span
    between update ends, GPU busy (union of kernel intervals), idle between the
    previous update end and the first assign, last map kernel end -> update end."""
    ends = [i for i, r in enumerate(rows) if end_pat in r[0]]
    rx = re.compile(map_pat)
    out = ["| iteration span ms | GPU busy ms | idle before first assign ms | "
           "last map kernel -> update end ms |", "|---|---|---|---|"]
    for a, b in zip(ends, ends[1:]):
        prev_end = rows[a][2]
        seg = rows[a + 1:b + 1]
        iv = sorted((max(s, prev_end), e) for _n, s, e, *_ in seg if e > prev_end)
        busy, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        first = min((s for n, s, e, *_ in seg if "assign" in n), default=None)
        last_map = max((e for n, s, e, *_ in seg if rx.search(n)), default=None)
        upd = rows[b][2]
        out.append(f"| {(upd - prev_end) / 1e6:.2f} | {busy / 1e6:.2f} | "
                   f"{((first - prev_end) / 1e6) if first else float('nan'):.2f} | "
                   f"{((upd - last_map) / 1e6) if last_map else float('nan'):.2f} |")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", action="store_true",
                    help="per-iteration K-Means table (spans, busy, idle gaps)")
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--timeline")
    ap.add_argument("--from-last", nargs=2, metavar=("PATTERN", "N"),
                    help="summarise only from the N-th last dispatch matching PATTERN on "
                         "(e.g. the timed iterations of a benchmark after its warmup)")
    a = ap.parse_args()
    rows = load(a.db)
    if a.from_last:
        rx, n = re.compile(a.from_last[0]), int(a.from_last[1])
        idx = [i for i, r in enumerate(rows) if rx.search(r[0])]
        if len(idx) >= n:
            rows = rows[idx[-n]:]
        span = (rows[-1][2] - rows[0][1]) / 1e3 if rows else 0.0
        print(f"window: {len(rows)} dispatches over {span:.1f} µs (first to last end)\n")
    print(summary(rows, a.top))
    if a.iterations:
        print()
        print(iterations(rows))
    if a.timeline:
        t0 = None
        rx = re.compile(a.timeline)
        for name, s, e, g, w in rows:
            if rx.search(name):
                t0 = s if t0 is None else t0
                print(f"{(s - t0) / 1e3:12.1f} {(e - s) / 1e3:10.1f}  grid={g} wg={w}  {short(name)}")


if __name__ == "__main__":
    main()
