"""Worker for test_multiprocess: a 2-rank node whose JobTracker runs in a
process of its own (hbmr.jobtracker.process); pre-staged K-Means iterations
through RemoteJobTracker (long-poll waits, one info call per finished job)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hbmr.mapred.jobconf import JobConf  # noqa: E402
from hbmr.mapred.node import Node  # noqa: E402
from hbmr.models import kmeans as K  # noqa: E402


def main():
    conf = JobConf()
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 2)
    conf.set_boolean("hbmr.jobtracker.process", True)
    node = Node(conf, use_gpu=False)
    if not node.is_master:
        node.serve_until_shutdown()
        node.shutdown()
        return
    try:
        drv = K.KMeansDriver(node.submit_job, node.job_result, conf=conf, k=5, d=8,
                             inp="synthetic:6000:11", split_points=1000)
        for s in range(4):
            drv.step(prefetch=min(2, 3 - s))
        per = {}
        for h in drv.history:
            for t, n in (h.get("maps_per_tracker") or {}).items():
                per[t] = per.get(t, 0) + n
        print("RESULT " + json.dumps({
            "centroids": drv.centroids().tolist(), "points": drv.history[-1]["points"],
            "maps_per_tracker": per, "jt_process": node.jt_process,
            "jt_pid_alive": node.jt.proc.poll() is None,
            "timeline_keys": sorted(drv.history[-1].get("timeline") or {}),
            "jt_cpu_s": node.jt.cpu_seconds()}), flush=True)
    finally:
        node.shutdown()
        # the JobTracker process is gone with the node
        print("JT_EXIT " + str(node.jt.proc.poll()), flush=True)


if __name__ == "__main__":
    main()
