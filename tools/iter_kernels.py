"""Per-iteration device time of the K-Means jobs in a rocprofv3 kernel trace:
for each interval between consecutive kmeans_update kernels, the summed
duration of the fused top-3 assign kernels and of all kernels (the same work
every iteration, so a slower iteration means a slower device clock or
contention, not more work).

usage: python tools/iter_kernels.py RESULTS.db"""
import sqlite3
import sys


def main():
    rows = sqlite3.connect(sys.argv[1]).execute(
        "select name, start, end from kernels order by start").fetchall()
    ups = [r for r in rows if "kmeans_update" in r[0]]
    print("iter  span_ms  top3_sum_ms  top3_calls  all_kernels_sum_ms")
    prev = rows[0][1]
    for i, u in enumerate(ups):
        seg = [r for r in rows if prev <= r[1] < u[2]]
        top = [r for r in seg if "top3_q1_grouped" in r[0]]
        print(f"{i:4d} {(u[2] - prev) / 1e6:8.2f} {sum(e - s for _, s, e in top) / 1e6:12.2f} "
              f"{len(top):11d} {sum(e - s for _, s, e in seg) / 1e6:18.2f}")
        prev = u[2]


if __name__ == "__main__":
    main()
