"""TeraSort benchmark (BASELINE config 5) on the local GPUs.

One job = TeraGen straight into HBM (map input) + per-split radix sort +
range partition + all-to-all-v shuffle + final sort + validation.  The first
job materialises the splits in HBM (split cache); timed jobs re-sort them.

  python tools/bench_terasort.py --rows 100000000 --split-rows 10000000 --steps 3
  torchrun --nproc-per-node N tools/bench_terasort.py ...   (multi-GPU)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--split-rows", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--output", default=None)
    a = ap.parse_args()
    import torch

    from hbmr.gpu.syncjob import sync_conf
    from hbmr.mapred.jobconf import JobConf
    from hbmr.mapred.node import Node
    from hbmr.models import terasort as T

    conf = JobConf()
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 1)
    conf.set_int("hbmr.gpu.queue.depth", 64)
    conf.set_int("mapred.task.timeout", 0)
    node = Node(conf)
    if not node.is_master:
        node.serve_until_shutdown()
        node.shutdown()
        return 0

    def job():
        rj = node.submit_job(T.terasort_conf(conf, rows=a.rows, split_rows=a.split_rows,
                                             output=a.output))
        rj.waitForCompletion()
        if not rj.isSuccessful():
            raise RuntimeError(rj.getFailureInfo())
        return rj

    try:
        for _ in range(a.warmup):
            job()
        node.submit_job(sync_conf(conf)).waitForCompletion()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            rj = job()
        node.submit_job(sync_conf(conf)).waitForCompletion()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        res = rj._impl.jip.result
        ok = all(r["unsorted"] == 0 and r["checksum_ok"] for r in res.values())
        total = sum(r["records"] for r in res.values())
        print(json.dumps({"metric": "TeraSort records sorted per second (whole node)",
                          "value": round(a.rows / dt, 1), "unit": "records/s",
                          "gb_per_s": round(a.rows * 100 / dt / 1e9, 3),
                          "seconds_per_sort": round(dt, 4), "rows": a.rows,
                          "split_rows": a.split_rows, "n_gpus": node.world,
                          "validated": ok and total == a.rows,
                          "timeline": rj._impl.jip.timeline()}))
    finally:
        node.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
