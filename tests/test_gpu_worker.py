"""Crash isolation of device work: GPU maps run in a persistent per-tracker
worker process (hbmr/gpu/worker.py), so a crashed worker is a set of failed
attempts plus a fresh worker — never a dead tracker (the reference: a crashed
Pipes GPU binary is an ordinary task failure, Application.java:274-290,
JvmManager.java:413-485).  Crashes are injected with
``hbmr.faultinject.worker.exit.attempt`` (the worker calls os._exit when it
starts a matching attempt); simulated GPU slots keep these tests on the CPU."""
import json
import os
import subprocess
import sys

import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"


def _conf(crash=None, worker=True):
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_boolean("hbmr.gpu.worker.process", worker)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
    conf.set_int("mapred.task.timeout", 0)
    if crash:
        conf.set("hbmr.faultinject.worker.exit.attempt", crash)
    return conf


def _kmeans(conf, iters=3, tmp=None):
    if tmp is not None:
        conf.set("mapred.local.dir", str(tmp))
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=6,
                             d=16, inp="synthetic:12000:5", split_points=2000)
        for _ in range(iters):
            assert drv.step()["points"] == 12000
        rt = cl.trackers[0].gpu_runtime
        info = {"deaths": getattr(rt, "deaths", 0), "failed": sum(
            h["counters"].get(JIP, "NUM_FAILED_MAPS") for h in drv.history),
            "events": [e["event"] for e in cl.jt.history.events]}
        return drv.centroids(), info


def test_worker_process_matches_in_process_runtime(tmp_path):
    c_w, info = _kmeans(_conf(), tmp=tmp_path / "a")
    c_i, _ = _kmeans(_conf(worker=False), tmp=tmp_path / "b")
    assert info["deaths"] == 0
    assert torch.equal(c_w, c_i)


def test_worker_crash_in_map_is_a_failed_attempt_and_a_new_worker(tmp_path):
    ref, _ = _kmeans(_conf(), tmp=tmp_path / "ref")
    # iteration 2, map 3's first attempt kills the worker mid-job: its in-flight
    # attempts fail, the held outputs of its finished maps are re-executed, the
    # next iteration re-localises its centroids from the centroid directory
    got, info = _kmeans(_conf(crash="_0002_m_000003_0"), tmp=tmp_path / "crash")
    assert info["deaths"] == 1
    assert info["failed"] >= 1
    assert torch.equal(got, ref)        # exact fixed-point partials: identical result


def test_worker_crash_in_collective_reduce_reruns_the_gang(tmp_path):
    ref, _ = _kmeans(_conf(), tmp=tmp_path / "ref")
    got, info = _kmeans(_conf(crash="_0002_r_000000_0"), tmp=tmp_path / "crash")
    assert info["deaths"] == 1
    assert "COLLECTIVE_RESTART" in info["events"]
    assert torch.equal(got, ref)


def test_worker_reduce_that_raises_is_retried_by_the_same_worker(tmp_path):
    """A collective reduce that FAILS (raises, no crash) in worker mode: the
    worker keeps the job, the gang re-runs there (maps again, then the reduce)
    and the worker never dies."""
    ref, _ = _kmeans(_conf(), tmp=tmp_path / "ref")
    conf = _conf()
    conf.set("hbmr.faultinject.reduce.fail.attempt", "_0002_r_000000_0")
    got, info = _kmeans(conf, tmp=tmp_path / "fail")
    assert info["deaths"] == 0
    assert "COLLECTIVE_RESTART" in info["events"]
    assert torch.equal(got, ref)


def test_finished_jobs_are_purged_from_trackers_and_workers(tmp_path):
    """KillJobAction after a job finishes: the tracker and its GPU worker drop
    the job (its device map outputs), so held state does not grow per job."""
    import time
    conf = _conf()
    conf.set("mapred.local.dir", str(tmp_path))
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=4,
                             d=8, inp="synthetic:4000:5", split_points=1000)
        for _ in range(3):
            drv.step()
        tt = cl.trackers[0]
        deadline = time.time() + 10
        while time.time() < deadline and (tt.jobs or tt.gpu_runtime.held or
                                           tt.gpu_runtime.jobs_sent):
            time.sleep(0.05)
        assert not tt.jobs and not tt.gpu_runtime.held and not tt.gpu_runtime.jobs_sent
        assert tt.job_result(drv.history[-1]["job"]) is not None


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("crash", [None, "_0002_m_000004_0"])
def test_two_rank_worker_gang_restart(crash):
    """world 2: rank 1's worker dies mid-job; its peer may be blocked in a
    collective with it, so the JobTracker restarts both workers under a new
    communicator generation and the job still produces the exact answer."""
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0", HBMR_MP_SIM="1")
    if crash:
        env["HBMR_MP_CRASH"] = crash
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "workers", "mp_kmeans.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(lines[0][7:])
    assert res["points"] == 6000 and res["trackers"] == 2
    if crash:
        assert res["gang_restarts"] >= 1 and res["worker_generation"] >= 1
    else:
        assert res["gang_restarts"] == 0
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                             d=8, inp="synthetic:6000:11", split_points=1000)
        for _ in range(3):
            drv.step()
        ref = drv.centroids()
    assert torch.equal(torch.tensor(res["centroids"], dtype=torch.float32), ref)


# ---------------------------------------------------------------- on the MI355X
def _gpu_kmeans(tmp, worker, crash=None):
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.worker.process", worker)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
    conf.set_int("mapred.task.timeout", 0)
    conf.set("mapred.local.dir", str(tmp))
    if crash:
        conf.set("hbmr.faultinject.worker.exit.attempt", crash)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=64,
                             d=128, inp="synthetic:400000:3", split_points=50000)
        for _ in range(3):
            assert drv.step()["points"] == 400000
        rt = cl.trackers[0].gpu_runtime
        return drv.centroids(), getattr(rt, "deaths", 0), drv.history


@pytest.mark.gpu
def test_gpu_worker_process_runs_the_hip_kernels_and_survives_a_crash(tmp_path):
    ref, _, _ = _gpu_kmeans(tmp_path / "inproc", worker=False)
    got, deaths, hist = _gpu_kmeans(tmp_path / "worker", worker=True)
    assert deaths == 0
    assert torch.equal(got, ref)        # same kernels, same exact partials
    # the worker dies (os._exit, like a fatal HIP error) at the start of a map
    # attempt of iteration 2: failed attempts, a new worker, the same answer
    got2, deaths2, hist2 = _gpu_kmeans(tmp_path / "crash", worker=True, crash="_0002_m_000001_0")
    assert deaths2 == 1
    assert sum(h["counters"].get(JIP, "NUM_FAILED_MAPS") for h in hist2) >= 1
    assert torch.equal(got2, ref)


@pytest.mark.gpu
def test_gpu_prestaged_iterations_with_delta_combiner_match_plain_runs(tmp_path):
    """On the MI355X: iterations staged two ahead (maps gated on the device
    behind the previous reduce) with the delta combiner give exactly the
    centroids of plain, one-at-a-time iterations with the sorted combiner."""
    def run(tmp, prestage, combiner, ahead):
        conf = JobConf()
        conf.set_boolean("hbmr.gpu.worker.process", True)
        conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
        conf.set_int("hbmr.gpu.queue.depth", 16)
        conf.set_int("mapred.task.timeout", 0)
        conf.set_boolean("hbmr.job.prestage", prestage)
        conf.set("hbmr.kmeans.combiner", combiner)
        conf.set("mapred.local.dir", str(tmp))
        with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
            drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf,
                                 k=256, d=128, inp="synthetic:600000:3", split_points=50000)
            drv.prefetch_delay = 0.0
            for s in range(6):
                assert drv.step(prefetch=min(ahead, 5 - s))["points"] == 600000
            staged = sum(e["event"] == "JOB_STAGED" for e in cl.jt.history.events)
            return drv.centroids(), staged
    ref, s0 = run(tmp_path / "plain", False, "sorted", 0)
    got, s1 = run(tmp_path / "staged", True, "delta", 2)
    assert s0 == 0 and s1 >= 3
    assert torch.equal(got, ref)
