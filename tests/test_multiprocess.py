"""Multi-process node (one process per tracker, gloo + TCP RPC control plane)."""
import json
import os
import subprocess
import sys

import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_process_kmeans_matches_single_process():
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "workers", "mp_kmeans.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(lines[0][7:])
    assert res["points"] == 6000 and res["trackers"] == 2
    assert len(res["map_trackers"]) == 2      # locality spread maps over both processes
    # a classic job whose reduces (in both processes) read the other's map outputs
    assert res["wordcount_ok"] and len(res["wordcount_reduce_trackers"]) == 2
    # same answer as one in-process tracker: fixed-point partials are exact
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                             d=8, inp="synthetic:6000:11", split_points=1000)
        for _ in range(3):
            drv.step()
        ref = drv.centroids()
    assert torch.equal(torch.tensor(res["centroids"], dtype=torch.float32), ref)


def test_jobtracker_in_its_own_process_runs_prestaged_kmeans():
    """hbmr.jobtracker.process: rank 0 starts the JobTracker as a child
    process; both ranks' trackers and the driver reach it over RPC.  The
    pre-staged iterations give the single-process answer."""
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "workers", "mp_jtproc.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(lines[0][7:])
    assert res["jt_process"] and res["jt_pid_alive"] and res["jt_cpu_s"] > 0
    assert res["points"] == 6000 and len(res["maps_per_tracker"]) == 2
    assert sum(res["maps_per_tracker"].values()) == 4 * 6
    assert res["timeline_keys"] == ["finish", "first_map", "first_reduce", "maps_done"]
    ex = [l for l in r.stdout.splitlines() if l.startswith("JT_EXIT ")]
    assert ex and ex[0] != "JT_EXIT None"     # the JobTracker process exited with the node
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                             d=8, inp="synthetic:6000:11", split_points=1000)
        for _ in range(4):
            drv.step()
        ref = drv.centroids()
    assert torch.equal(torch.tensor(res["centroids"], dtype=torch.float32), ref)
