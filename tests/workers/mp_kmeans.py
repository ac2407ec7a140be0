"""Worker for test_multiprocess: K-Means on a multi-process node (gloo, CPU slots)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hbmr.gpu.syncjob import sync_conf  # noqa: E402
from hbmr.mapred.jobconf import JobConf  # noqa: E402
from hbmr.mapred.node import Node  # noqa: E402
from hbmr.models import kmeans as K  # noqa: E402


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
        jip = node.jt.jobs[drv.history[-1]["job"]]
        placed = sorted({t.successful.tracker for t in jip.maps})
        events = [e["event"] for e in node.jt.history.events]
        print("RESULT " + json.dumps({"centroids": drv.centroids().tolist(),
                                      "points": drv.history[-1]["points"],
                                      "trackers": len(node.jt.trackers),
                                      "map_trackers": placed,
                                      "gang_restarts": events.count("GPU_GANG_RESTART"),
                                      "collective_restarts": events.count("COLLECTIVE_RESTART"),
                                      "worker_generation": node.jt.worker_generation}),
              flush=True)
    finally:
        node.shutdown()


if __name__ == "__main__":
    main()
