"""TeraSort benchmark (BASELINE config 5) on the local GPUs.

One job = map: key extraction + range partition (counting sort by partition)
of every HBM-resident split; reduce: per partition, collect the pieces of
every map, radix-sort the keys and gather the 100-byte records once (one GPU),
or gather + all-to-all-v over RCCL/xGMI + sort (several GPUs); validation
(order within and across partitions, key checksum) on the device.  The first
job generates the input into HBM with TeraGen (split cache); timed jobs
re-sort it.  The GPU work runs in the per-rank GPU worker process, so the
timing brackets are sync jobs (every worker synchronises its device).

  python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3   # 100 GB
  ... --output /tmp/tera-out   # also time jobs that commit their output (reported alongside)
  ... -D hbmr.terasort.reduce.gid=false  # job properties (here: the v3 permutation reduce)
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
    ap.add_argument("--partitions", type=int, default=0)
    ap.add_argument("-D", dest="defines", action="append", default=[],
                    help="key=value job property, e.g. -D hbmr.terasort.reduce.gid=false")
    a = ap.parse_args()
    from hbmr.gpu.syncjob import sync_conf
    from hbmr.mapred.jobconf import JobConf
    from hbmr.mapred.node import Node
    from hbmr.models import terasort as T

    conf = JobConf()
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 1)
    conf.set_int("hbmr.gpu.queue.depth", 64)
    conf.set_int("mapred.task.timeout", 0)
    for kv in a.defines:
        k, _, v = kv.partition("=")
        conf.set(k, v)
    node = Node(conf)
    if not node.is_master:
        node.serve_until_shutdown()
        node.shutdown()
        return 0

    def job(output=None):
        rj = node.submit_job(T.terasort_conf(conf, rows=a.rows, split_rows=a.split_rows,
                                             output=output, partitions=a.partitions))
        rj.waitForCompletion()
        if not rj.isSuccessful():
            raise RuntimeError(rj.getFailureInfo())
        return rj

    def timed_with_output():
        """TeraSort with its output committed (part files written through the
        attempt work dir, fsync'd, renamed; TeraSort.java:241-247): seconds per
        job, the output directory cleared outside the timed region."""
        import shutil
        total = 0.0
        for i in range(a.steps):
            print(f"bench_terasort: sort with output {i + 1}/{a.steps}", file=sys.stderr,
                  flush=True)
            shutil.rmtree(a.output, ignore_errors=True)
            node.submit_job(sync_conf(conf)).waitForCompletion()
            t0 = time.perf_counter()
            job(a.output)
            node.submit_job(sync_conf(conf)).waitForCompletion()
            total += time.perf_counter() - t0
        def prog(i, nf):
            if i % 8 == 0:
                print(f"bench_terasort: validating part {i}/{nf}", file=sys.stderr, flush=True)
        v = T.teravalidate(a.output, progress=prog)
        return total / a.steps, v

    try:
        for _ in range(a.warmup):
            job()
        node.submit_job(sync_conf(conf)).waitForCompletion()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            rj = job()
        node.submit_job(sync_conf(conf)).waitForCompletion()
        dt = (time.perf_counter() - t0) / a.steps
        res = rj._impl.jip.result
        out_extra = {}
        if a.output:
            dto, v = timed_with_output()
            out_extra = {"seconds_per_sort_with_output": round(dto, 4),
                         "gb_per_s_with_output": round(a.rows * 100 / dto / 1e9, 3),
                         "output_validated": v["records"] == a.rows and v["misordered"] == 0,
                         "output_dir": a.output}
        ok = all(r["unsorted"] == 0 and r["checksum_ok"] for r in res.values())
        total = sum(r["records"] for r in res.values())
        print(json.dumps({"metric": "TeraSort records sorted per second (whole node)",
                          "value": round(a.rows / dt, 1), "unit": "records/s",
                          "gb_per_s": round(a.rows * 100 / dt / 1e9, 3),
                          "seconds_per_sort": round(dt, 4), "rows": a.rows,
                          "split_rows": a.split_rows, "n_gpus": node.world,
                          "validated": ok and total == a.rows,
                          "data_gb": round(a.rows * 100 / 1e9, 2),
                          "partitions": max(r.get("partitions", 0) for r in res.values()),
                          "peak_hbm_gb_per_gpu": round(max(r.get("peak_hbm_bytes", 0)
                                                           for r in res.values()) / 1e9, 2),
                          "defines": a.defines,
                          "hbm_budget_gb": conf.get_float("hbmr.terasort.hbm.budget.gb", 0.0)
                          or None,
                          "spilled_records": rj.getCounters().get(
                              "org.apache.hadoop.mapred.Task$Counter", "MAP_SPILLED_RECORDS"),
                          "timeline": rj._impl.jip.timeline(), **out_extra}))
    finally:
        node.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
