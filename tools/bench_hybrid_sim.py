"""Hybrid vs stock vs optional vs GPU-only map scheduling on a simulated node
(the paper's comparison, Shirahata et al. CloudCom 2010: hybrid 1.93x faster
than stock Hadoop scheduling).  One tracker with one simulated GPU slot
(device time per task fixed) and C CPU slots whose map takes accel x longer;
each policy runs the same split job twice (the first profiles the CPU) and the
second job's makespan is reported.

usage: python tools/bench_hybrid_sim.py [--maps 40] [--gpu-ms 10] [--cpu-slots 4]
       [--accel 3 10 30 100] [--out profiles/hybrid_vs_stock_sim.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from hbmr.mapred.scheduler.costmodel import makespan_estimates  # noqa: E402
from test_scheduler_math import run_policy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--maps", type=int, default=40)
    ap.add_argument("--gpu-ms", type=float, default=10.0)
    ap.add_argument("--cpu-slots", type=int, default=4)
    ap.add_argument("--accel", type=float, nargs="+", default=[3, 10, 30, 100])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for acc in a.accel:
        cpu_ms = a.gpu_ms * acc
        row = {"accel": acc, "gpu_ms": a.gpu_ms, "cpu_ms": cpu_ms, "maps": a.maps,
               "cpu_slots": a.cpu_slots, "gpu_slots": 1,
               "model_ms": {k: (round(v * 1e3, 1) if isinstance(v, float) else v) for k, v in
                            makespan_estimates(a.maps, a.cpu_slots, 1, cpu_ms / 1e3,
                                               a.gpu_ms / 1e3).items()}}
        for name, pol, cpu in [("hybrid", "hybrid", True), ("optional", "optional", True),
                               ("stock", "stock", True), ("gpu_only", "hybrid", False)]:
            t, nc, ng = run_policy(pol, a.maps, a.gpu_ms, cpu_ms, a.cpu_slots, cpu=cpu)
            row[name] = {"makespan_ms": round(t * 1e3, 1), "cpu_maps": nc, "gpu_maps": ng}
        row["stock_over_hybrid"] = round(row["stock"]["makespan_ms"] /
                                         row["hybrid"]["makespan_ms"], 3)
        rows.append(row)
        print(json.dumps(row), flush=True)
    doc = {"what": "second-job makespan per policy on a simulated node (hbmr.gpu.simulate): "
                   "1 GPU slot, C CPU slots, CPU map = accel x GPU map",
           "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
