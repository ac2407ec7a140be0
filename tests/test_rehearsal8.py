"""VERDICT r5 Next #3: an automated 8-rank regression test of the path the
first 8-GPU run takes — eight rank processes with bench.py's defaults at 8
ranks (JobTracker process, per-rank GPU worker processes with
GPU_MAX_HW_QUEUES=8, hybrid scheduling with CPU slots, pre-staged exact
K-Means iterations) on simulated GPU slots over gloo, against single-process
answers.  The reference's MiniMRCluster runs N trackers in one test
(src/test/org/apache/hadoop/mapred/MiniMRCluster.java); the device each GPU
map gets is checked per rank as JobQueueTaskScheduler.java:354-379 picks it."""
import collections
import json
import os
import subprocess
import sys
import time

import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K
from hbmr.models import terasort as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "workers"))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _text(path, n=120_000):
    import numpy as np
    rng = np.random.default_rng(3)
    words = [f"w{i}" for i in range(2000)] + ["the", "a", "gpu", "hadoop"]
    idx = rng.zipf(1.3, n) % len(words)
    with open(path, "w") as f:
        for i in range(0, len(idx), 16):
            f.write(" ".join(words[j] for j in idx[i:i + 16]) + "\n")


def test_eight_ranks_take_the_8_gpu_path_and_match_one_process(tmp_path):
    import mp_rehearsal8 as R
    _text(tmp_path / "text.txt")
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0",
               HBMR_MP_DIR=str(tmp_path), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="1")
    env.pop("GPU_MAX_HW_QUEUES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "workers", "mp_rehearsal8.py")]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    elapsed = time.time() - t0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(lines[0][7:])
    assert elapsed < 120, elapsed

    # the 8-rank defaults really ran: JobTracker process, GPU worker per rank
    # on its own device (= its local rank), 8 hardware queues per worker
    assert res["jt_process"]
    ranks = sorted(res["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == list(range(8))
    for x in ranks:
        assert x["worker_mode"]
        assert x["planned"] == [x["local_rank"]] == [x["rank"]]
        assert x["worker"]["devices"] == x["planned"]
        assert x["worker"]["gpu_max_hw_queues"] == "8"
    assert len({x["worker"]["pid"] for x in ranks}) == 8
    # K-Means: every job's maps on (simulated) GPU slots of all 8 ranks, and
    # the single-process exact answer bit for bit
    assert all(g == 32 for g in res["gpu_maps"]), res["gpu_maps"]
    assert len(res["maps_per_tracker"]) == 8
    conf = JobConf()
    conf.set_boolean(K.EXACT_KEY, True)
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        drv = R.run_kmeans(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf, prefetch=0)
        ref = drv.centroids()
    assert torch.equal(torch.tensor(res["centroids"], dtype=torch.float32), ref)
    # TeraSort: validated, and byte-identical to one process's sorted output
    v = res["terasort_validate"]
    assert v["records"] == 400_000 and v["misordered"] == 0 and v["files"] == 8
    out1 = tmp_path / "ts1"
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(T.terasort_conf(JobConf(), rows=400_000, split_rows=25_000,
                                           output=str(out1)))
        rj.waitForCompletion(300)
        assert rj.isSuccessful(), rj.getFailureInfo()
    assert res["terasort_digest"] == R.digest_parts(str(out1))
    assert T.teravalidate(str(out1))["checksum"] == v["checksum"]
    # WordCount: the union of the 8 ranks' part files is the word count
    want = collections.Counter((tmp_path / "text.txt").read_text().split())
    got = collections.Counter()
    parts = [f for f in os.listdir(tmp_path / "wc") if f.startswith("part-")]
    assert len(parts) == 8
    for f in parts:
        for ln in (tmp_path / "wc" / f).read_text().splitlines():
            w, n = ln.split("\t")
            assert w not in got
            got[w] = int(n)
    assert got == want
    # no shuffle read sizes on the host inside a collective
    for job in ("terasort", "wordcount"):
        cs = res[f"{job}_counters"]
        assert cs.get("ALL_TO_ALL_V_HOST_READS", 0) == 0, (job, cs)
        assert cs.get("ALL_TO_ALL_HOST_READS", 0) == 0, (job, cs)
