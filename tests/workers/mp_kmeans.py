"""Worker for test_multiprocess: K-Means on a multi-process node (gloo, CPU slots)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hbmr.gpu.syncjob import sync_conf  # noqa: E402
from hbmr.mapred.jobconf import JobConf  # noqa: E402
from hbmr.mapred.node import Node  # noqa: E402
from hbmr.models import kmeans as K  # noqa: E402


def _classic_job(node):
    # a classic job across both processes: map outputs of one rank are
    # read by the other rank's reduce (from files: not the in-memory store)
    import collections
    import tempfile
    from hbmr.mapred import JobClient
    from hbmr.models import wordcount
    tmp = tempfile.mkdtemp(prefix="mpwc-")
    os.mkdir(os.path.join(tmp, "in"))
    cnt = collections.Counter()
    for i in range(4):
        lines = [f"w{(i * 5 + j) % 13} w{j % 7}" for j in range(300)]
        with open(os.path.join(tmp, "in", f"f{i}"), "w") as f:
            f.write("\n".join(lines) + "\n")
        for ln in lines:
            cnt.update(ln.split())
    wc = JobConf()
    wc.set_boolean("hbmr.wordcount.native", False)
    wjob = wordcount.make_job(os.path.join(tmp, "in"), os.path.join(tmp, "out"), reduces=4,
                              conf=wc)
    wrj = JobClient.runJob(wjob, cluster=node, verbose=False)
    got = {}
    for fn in os.listdir(os.path.join(tmp, "out")):
        if fn.startswith("part-"):
            for line in open(os.path.join(tmp, "out", fn)):
                k, v = line.rstrip("\n").split("\t")
                got[k] = int(v)
    wjip = node.jt.jobs.get(str(wrj.getID()))
    red_trackers = sorted({t.successful.tracker for t in wjip.reduces}) if wjip else []
    wordcount_ok = wrj.isSuccessful() and got == dict(cnt)
    return wordcount_ok, red_trackers


def main():
    conf = JobConf()
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 2)
    if os.environ.get("HBMR_MP_SIM"):
        # simulated GPU slots in per-rank GPU worker processes (gloo among them)
        conf.set_boolean("hbmr.gpu.simulate", True)
        conf.set_boolean("hbmr.gpu.worker.process", True)
        conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
        conf.set_int("hbmr.worker.torch.threads", 1)
    if os.environ.get("HBMR_MP_CRASH"):
        conf.set("hbmr.faultinject.worker.exit.attempt", os.environ["HBMR_MP_CRASH"])
    node = Node(conf, use_gpu=False)
    if not node.is_master:
        node.serve_until_shutdown()
        node.shutdown()
        return
    try:
        drv = K.KMeansDriver(node.submit_job, node.job_result, conf=conf, k=5, d=8,
                             inp="synthetic:6000:11", split_points=1000)
        for _ in range(3):
            drv.step()
        rj = node.submit_job(sync_conf(conf))
        rj.waitForCompletion()
        assert rj.isSuccessful(), rj.getFailureInfo()
        wordcount_ok, red_trackers = _classic_job(node) if not os.environ.get("HBMR_MP_SIM") \
            else (None, [])
        jip = node.jt.jobs[drv.history[-1]["job"]]
        placed = sorted({t.successful.tracker for t in jip.maps})
        events = [e["event"] for e in node.jt.history.events]
        print("RESULT " + json.dumps({"centroids": drv.centroids().tolist(),
                                      "points": drv.history[-1]["points"],
                                      "trackers": len(node.jt.trackers),
                                      "map_trackers": placed,
                                      "gang_restarts": events.count("GPU_GANG_RESTART"),
                                      "collective_restarts": events.count("COLLECTIVE_RESTART"),
                                      "worker_generation": node.jt.worker_generation,
                                      "wordcount_ok": wordcount_ok,
                                      "wordcount_reduce_trackers": red_trackers}),
              flush=True)
    finally:
        node.shutdown()


if __name__ == "__main__":
    main()
