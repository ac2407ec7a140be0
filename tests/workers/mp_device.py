"""Worker for test_gpu_multirank: a 2-rank node sharing one GPU
(HBMR_SHARED_DEVICE=0) whose per-rank GPU workers run the device-tensor data
plane over gloo — the K-Means collective all-reduce, TeraSort's all-to-all-v of
records and GPU WordCount's all-to-all-v of hash tables.  Prints one RESULT
line with the outputs and the collective counters of each job."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hbmr.mapred.jobconf import JobConf  # noqa: E402
from hbmr.mapred.node import Node  # noqa: E402
from hbmr.models import kmeans as K  # noqa: E402
from hbmr.models import terasort as T  # noqa: E402
from hbmr.models import wordcount as WC  # noqa: E402
from hbmr.parallel.collectives import COLLECTIVE_GROUP  # noqa: E402


def digest_dir(d):
    out = {}
    for f in sorted(os.listdir(d)):
        if f.startswith("part-"):
            out[f] = hashlib.sha256(open(os.path.join(d, f), "rb").read()).hexdigest()
    return out


def collective_counters(rj):
    g = rj.getCounters().group(COLLECTIVE_GROUP)
    return {c.name: c.getValue() for c in g}


def run_jobs(submit, result_of, conf, work):
    """The three jobs; shared by this worker and the in-process comparison."""
    res = {}
    drv = K.KMeansDriver(submit, result_of, conf=conf, k=16, d=32,
                         inp="synthetic:400000:5", split_points=50000)
    rjs = []
    for _ in range(3):
        drv.step()
    res["centroids"] = drv.centroids().tolist()
    res["kmeans_job"] = drv.history[-1]["job"]
    rj = submit(T.terasort_conf(conf, rows=400_000, split_rows=50_000,
                                output=os.path.join(work, "ts")))
    rj.waitForCompletion(300)
    assert rj.isSuccessful(), rj.getFailureInfo()
    rjs.append(rj)
    res["terasort"] = digest_dir(os.path.join(work, "ts"))
    res["terasort_counters"] = collective_counters(rj)
    # the same sort with the shuffle in 3 waves (each wave's all-to-all-v
    # issued once its maps are done; with hbmr.job.prestage the reduce starts
    # early and the waves overlap the maps) and sorted runs merged on arrival (K8)
    wc = T.terasort_conf(conf, rows=400_000, split_rows=50_000,
                         output=os.path.join(work, "tsw"))
    wc.set_int("hbmr.terasort.shuffle.waves", 3)
    wc.set_boolean("hbmr.terasort.shuffle.sorted.runs", True)
    rj = submit(wc)
    rj.waitForCompletion(300)
    assert rj.isSuccessful(), rj.getFailureInfo()
    res["terasort_waves"] = digest_dir(os.path.join(work, "tsw"))
    res["terasort_waves_counters"] = collective_counters(rj)
    rj = submit(WC.gpu_job(os.path.join(work, "text.txt"), os.path.join(work, "wc"), base=conf,
                           maps=6))
    rj.waitForCompletion(300)
    assert rj.isSuccessful(), rj.getFailureInfo()
    res["wordcount"] = digest_dir(os.path.join(work, "wc"))
    res["wordcount_counters"] = collective_counters(rj)
    return res


def main():
    work = os.environ["HBMR_MP_DIR"]
    conf = JobConf()
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum",
                 int(os.environ.get("HBMR_MP_CPU_SLOTS", "0")))   # >0: CPU dry run
    node = Node(conf)
    if not node.is_master:
        node.serve_until_shutdown()
        node.shutdown()
        return
    try:
        res = run_jobs(node.submit_job, node.job_result, conf, os.path.join(work, "mp"))
        jip = node.jt.jobs[res.pop("kmeans_job")]
        res["kmeans_counters"] = {c.name: c.getValue()
                                  for c in jip.fold_counters().group(COLLECTIVE_GROUP)}
        res["trackers"] = len(node.jt.trackers)
        res["worker_mode"] = node.worker_mode
        print("RESULT " + json.dumps(res), flush=True)
    finally:
        node.shutdown()


if __name__ == "__main__":
    main()
