"""Timeline of the last TeraSort job in a rocprofv3 rocpd result: device span,
busy time, largest idle gaps and per-kernel totals (tools/gpu/r6_tera_prof.sh).

    python tools/tera_timeline.py gpurun_out/r6tprof/run_results.db
"""
import re
import sqlite3
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\(.*$", "", n)[:48]


def main(db):
    rows = sqlite3.connect(db).execute("select name,start,end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if "tera_part_count" in r[0]]
    sorts, prev = [], None
    for i in starts:
        if prev is None or rows[i][1] - rows[prev][2] > 5e6:
            sorts.append(i)
        prev = i
    seg = rows[sorts[-1]:]
    t0 = seg[0][1]
    busy, cs, ce, gaps = 0, None, None, []
    for n, s, e in seg:
        if ce is None:
            cs, ce = s, e
        elif s > ce:
            busy += ce - cs
            gaps.append((ce - t0, s - ce, short(n)))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"sorts {len(sorts)}  span {(ce - t0) / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  "
          f"idle {sum(g[1] for g in gaps) / 1e6:.2f} ms in {len(gaps)} gaps")
    maps_end = max(e for n, s, e in seg if "tera_part_scatter" in n)
    print(f"maps end {(maps_end - t0) / 1e6:.2f} ms")
    for g in sorted(gaps, key=lambda g: -g[1])[:10]:
        print(f"  gap at {g[0] / 1e6:7.2f} ms: {g[1] / 1e3:7.1f} us before {g[2]}")
    agg = {}
    for n, s, e in seg:
        agg[short(n)] = agg.get(short(n), 0) + (e - s)
    for k, v in sorted(agg.items(), key=lambda x: -x[1])[:14]:
        print(f"{v / 1e6:8.2f} ms  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
