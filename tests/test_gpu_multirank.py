"""Two ranks on the one-GPU box (HBMR_SHARED_DEVICE=0): each rank's GPU worker
drives device 0 and the device-tensor collectives of three jobs go over gloo
(staged through host memory, see TorchComm) — checked bit-exactly against two
TaskTrackers in one process over InProcessComm.  The RCCL branch itself is the
driver's 8-GPU run; its group construction is tested in test_node_groups."""
import json
import os
import subprocess
import sys

import pytest

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "workers"))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _text(path):
    import numpy as np
    rng = np.random.default_rng(7)
    words = [f"w{i}" for i in range(3000)] + ["the", "a", "gpu", "hadoop"]
    idx = rng.zipf(1.3, 400_000) % len(words)
    with open(path, "w") as f:
        for i in range(0, len(idx), 20):
            f.write(" ".join(words[j] for j in idx[i:i + 20]) + "\n")


@pytest.mark.gpu
def test_two_ranks_one_gpu_device_collectives_match_in_process(tmp_path):
    _text(tmp_path / "text.txt")
    for sub in ("mp", "ip"):
        os.makedirs(tmp_path / sub, exist_ok=True)
        os.symlink(tmp_path / "text.txt", tmp_path / sub / "text.txt")
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0",
               HBMR_SHARED_DEVICE="0", HBMR_MP_DIR=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "workers", "mp_device.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    mp = json.loads(lines[0][7:])
    print({k: v for k, v in mp.items() if k.endswith("counters")})
    assert mp["trackers"] == 2 and mp["worker_mode"]
    # the device paths really ran, staged through the host over gloo
    assert mp["kmeans_counters"].get("ALL_REDUCE_CUDA", 0) >= 2
    assert mp["kmeans_counters"].get("ALL_REDUCE_STAGED", 0) >= 2
    # default TeraSort shuffle on 2 ranks: 4 waves of static-shape all-to-alls
    # (records + counts, device-side counts, no host read between waves)
    assert mp["terasort_counters"].get("ALL_TO_ALL_FIXED_CUDA", 0) >= 8
    # WordCount's shuffle: static-shape exchanges of the word tables (slot
    # sizes agreed by a host all-reduce), no size read on the host inside a
    # collective (the one read is the compaction after both are enqueued)
    assert mp["wordcount_counters"].get("ALL_TO_ALL_V_STATIC_CUDA", 0) >= 4
    # no job reads a device tensor on the host inside a collective: the
    # all-to-all(v) row counts travel over the host group
    for job in ("kmeans", "terasort", "terasort_waves", "wordcount"):
        cs = mp[f"{job}_counters"]
        assert cs.get("ALL_TO_ALL_V_HOST_READS", 0) == 0, (job, cs)
        assert cs.get("ALL_TO_ALL_HOST_READS", 0) == 0, (job, cs)
    # waves: 3 all-to-all-v rounds (plus R/splitter agreement), same bytes
    assert mp["terasort_waves_counters"].get("ALL_TO_ALL_V_CUDA", 0) >= 6
    assert mp["terasort_waves"] == mp["terasort"]

    import mp_device
    conf = JobConf()
    with LocalCluster(conf, num_trackers=2, gpus=[[0], [0]], cpu_slots=0) as cl:
        ip = mp_device.run_jobs(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf,
                                str(tmp_path / "ip"))
    assert ip["centroids"] == mp["centroids"]              # exact fixed-point partials
    assert ip["terasort"] == mp["terasort"] and len(mp["terasort"]) == 2
    assert ip["terasort_waves"] == mp["terasort"]
    assert ip["wordcount"] == mp["wordcount"] and len(mp["wordcount"]) == 2
    assert ip["terasort_counters"].get("ALL_TO_ALL_FIXED_CUDA", 0) >= 8   # InProcessComm, device
