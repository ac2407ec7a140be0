"""CPU rehearsal of the headline bench's scaling: bench.py --simulate-ms T at
world 1/2/4/8 (simulated GPU slots with T ms of device time per split, no data;
gloo collectives; every rank and its GPU worker process on this host).

The simulated device time per job is 128 splits × T / N, so the remainder of
ms_per_step is the control plane (JobTracker scheduling, heartbeats, bulk
launches, completions), the collective reduce and host contention — on a small
container all 2N processes share its few cores, which a GPU node does not.

    python tools/scale_sim.py --ms 0.24 --reps 3 --out profiles/scale_sim_cpu.json
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=float, default=0.24)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--in-process", action="store_true",
                    help="simulated slots inside each tracker process (no GPU worker processes)")
    a = ap.parse_args()
    rows = []
    for n in [int(x) for x in a.ranks.split(",")]:
        runs = []
        for _ in range(a.reps):
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                                "--simulate-ms", str(a.ms), "--steps", str(a.steps),
                                "--warmup", str(a.warmup)] + (["--in-process"] if a.in_process
                                                              else []), capture_output=True, text=True,
                               timeout=900)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not line:
                raise SystemExit(f"bench failed at n={n}: {r.stderr[-2000:]}")
            runs.append(json.loads(line[-1]))
        ms = [x["ms_per_step"] for x in runs]
        med = sorted(runs, key=lambda x: x["ms_per_step"])[len(runs) // 2]
        device_ms = 128 * a.ms / n
        row = {"n": n, "ms_per_step_median": statistics.median(ms), "ms_per_step_all": ms,
               "simulated_device_ms_per_job": device_ms,
               "overhead_ms_per_job": statistics.median(ms) - device_ms,
               "phases_ms_median_run": med.get("phases_ms"),
               "map_tasks_per_s": med["value"],
               "maps_per_tracker_last_job": med.get("maps_per_tracker_last_job")}
        rows.append(row)
        print(json.dumps(row), flush=True)
    out = {"what": "bench.py --simulate-ms rehearsal of the 1/2/4/8-rank headline job on CPU "
                   "(gloo, simulated GPU slots, no split data)",
           "host": {"cpus": os.cpu_count()}, "simulate_ms_per_split": a.ms,
           "gpu_worker_process": not a.in_process,
           "note": "all ranks, their GPU worker processes and the JobTracker share this host's "
                   "CPUs; on a GPU node they do not, so overhead here is an upper bound",
           "rows": rows, "when": time.strftime("%Y-%m-%d %H:%M:%S")}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
