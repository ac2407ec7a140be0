"""Worker for test_rehearsal8: the path the first 8-GPU run takes, on CPU.

Eight rank processes (torchrun), each a Node exactly as bench.py builds it at
8 ranks — the JobTracker in a process of its own (hbmr.jobtracker.process,
default at 8+ ranks), a GPU worker process per rank (hbmr.gpu.worker.process)
started with GPU_MAX_HW_QUEUES from hbmr.gpu.hw.queues (8 with several ranks),
the hybrid scheduler with CPU slots, pre-staged iteration jobs, exact mode —
with simulated GPU slots (hbmr.gpu.simulate: the job's CPU map function and a
simulated device time per split) and gloo collectives.  Rank 0 runs:

* 4 pre-staged exact K-Means iteration jobs (the collective int64 reduce);
* TeraSort with the default multi-rank shuffle (static-shape waves);
* WordCount as a split-level job (the static-shape table shuffle);

and prints one RESULT line with their outputs and every rank's planned
device, its GPU worker's devices and its worker's GPU_MAX_HW_QUEUES."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hbmr.mapred.jobconf import JobConf  # noqa: E402
from hbmr.mapred.node import Node  # noqa: E402
from hbmr.models import kmeans as K  # noqa: E402
from hbmr.models import terasort as T  # noqa: E402
from hbmr.models import wordcount as WC  # noqa: E402
from hbmr.parallel.collectives import COLLECTIVE_GROUP  # noqa: E402

KM = dict(k=16, d=16, inp="synthetic:256000:5", split_points=8000)


def bench_conf(conf: JobConf) -> JobConf:
    """bench.py's configuration of a simulated (--simulate-ms) run."""
    conf.set("hbmr.scheduler.policy", "hybrid")
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 2)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
    conf.set_int("hbmr.gpu.queue.depth", 64)
    conf.set_int("hbmr.heartbeat.interval.ms", 200)
    conf.set_int("mapred.task.timeout", 0)
    conf.set_int("hbmr.locality.wait.ms", 5000)
    conf.set_boolean("hbmr.job.prestage", True)
    conf.set_int("hbmr.job.prestage.depth", 3)
    conf.set_int("hbmr.worker.torch.threads", 1)
    conf.set("hbmr.gpu.simulate", "true")
    conf.set("hbmr.gpu.simulate.task.ms", "0.2")
    conf.set_boolean(K.EXACT_KEY, True)
    return conf


def digest_parts(d):
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.startswith("part-"):
            with open(os.path.join(d, f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def collective_counters(rj):
    g = rj.getCounters().group(COLLECTIVE_GROUP)
    return {c.name: c.getValue() for c in g}


def run_kmeans(submit, result_of, conf, iters=4, prefetch=3):
    drv = K.KMeansDriver(submit, result_of, conf=conf, **KM)
    for i in range(iters):
        drv.step(prefetch=min(prefetch, iters - 1 - i))
    return drv


def main():
    work = os.environ["HBMR_MP_DIR"]
    conf = bench_conf(JobConf())
    node = Node(conf)
    # every rank: its planned device and its GPU worker's view
    tt = node.tt
    end = time.time() + 120
    rt = tt.gpu_runtime
    while rt is not None and not getattr(rt, "worker_info", None) and time.time() < end:
        time.sleep(0.05)
    info = {"rank": node.rank, "local_rank": node.local_rank, "planned": list(tt.gpu_devices),
            "worker": getattr(rt, "worker_info", None), "worker_mode": node.worker_mode}
    node.store.set(f"rehearsal8/{node.rank}", json.dumps(info))
    if not node.is_master:
        node.serve_until_shutdown()
        node.shutdown()
        return
    try:
        res = {"jt_process": bool(getattr(node, "jt_process", False))}
        drv = run_kmeans(node.submit_job, node.job_result, conf)
        res["centroids"] = drv.centroids().tolist()
        J = "org.apache.hadoop.mapred.JobInProgress$Counter"
        res["gpu_maps"] = [h["counters"].get(J, "GPU_MAP_TASKS") for h in drv.history]
        res["maps_per_tracker"] = drv.history[-1].get("maps_per_tracker")
        rj = node.submit_job(T.terasort_conf(conf, rows=400_000, split_rows=25_000,
                                             output=os.path.join(work, "ts")))
        rj.waitForCompletion(300)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res["terasort_digest"] = digest_parts(os.path.join(work, "ts"))
        res["terasort_validate"] = T.teravalidate(os.path.join(work, "ts"))
        res["terasort_counters"] = collective_counters(rj)
        rj = node.submit_job(WC.gpu_job(os.path.join(work, "text.txt"), os.path.join(work, "wc"),
                                        base=conf, maps=8))
        rj.waitForCompletion(300)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res["wordcount_counters"] = collective_counters(rj)
        res["ranks"] = [json.loads(node.store.get(f"rehearsal8/{r}").decode())
                        for r in range(node.world)]
        print("RESULT " + json.dumps(res), flush=True)
    finally:
        node.shutdown()


if __name__ == "__main__":
    main()
