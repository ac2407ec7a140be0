"""Kernel table of the last N K-Means iterations in a rocprofv3 kernel-trace
CSV (``--kernel-trace --output-format csv``): iterations are cut at the
kmeans_update kernels; per kernel name the calls and device time per
iteration, and per iteration the span, the GPU busy time (union of kernel
intervals) and the idle gaps.

usage: python tools/iter_table.py run_kernel_trace.csv [N]"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:90]


def main():
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(sys.argv[1]))]
    rows.sort(key=lambda r: r[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ups = [i for i, r in enumerate(rows) if "kmeans_update" in r[0]]
    ups = ups[-(n + 1):]
    t0, t1 = rows[ups[0]][2], rows[ups[-1]][2]
    win = [r for r in rows if t0 <= r[1] < t1]
    iters = len(ups) - 1
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e in win:
        a = agg[short(name)]
        a[0] += 1
        a[1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values())
    print(f"window: {iters} iterations, {(t1 - t0) / 1e6:.2f} ms "
          f"({(t1 - t0) / 1e6 / iters:.2f} ms per iteration)\n")
    print("| kernel | calls / iter | ms / iter | % |")
    print("|---|---|---|---|")
    for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"| `{k}` | {c / iters:.1f} | {ms / iters:.3f} | {100 * ms / tot:.1f} |")
    # busy = union of intervals per iteration
    print("\n| iteration | span ms | GPU busy ms | idle ms |")
    print("|---|---|---|---|")
    for a, b in zip(ups[:-1], ups[1:]):
        s0, s1 = rows[a][2], rows[b][2]
        iv = sorted((max(s, s0), min(e, s1)) for _, s, e in rows if s < s1 and e > s0)
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
        print(f"| | {(s1 - s0) / 1e6:.2f} | {busy / 1e6:.2f} | {(s1 - s0 - busy) / 1e6:.2f} |")


if __name__ == "__main__":
    main()
