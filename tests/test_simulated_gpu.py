"""GPU-slot scheduling paths without a GPU (hbmr.gpu.simulate), SleepJob, and
the event tracer.

The reference exercised its GPU scheduler with fake trackers that advertise
GPU devices (src/test/org/apache/hadoop/mapred/TestJobQueueTaskScheduler.java:
183-201); here whole trackers run with simulated GPU slots.
"""
import json

import pytest

import torch

from hbmr.examples.sleepjob import sleep_job_conf, split_sleep_conf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobclient import JobClient
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K
from hbmr.utils.trace import TRACE

JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"


def _sim_conf(**kw):
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 1)
    conf.set_int("mapred.task.timeout", 0)
    for k, v in kw.items():
        conf.set(k, str(v))
    return conf


def _kmeans(cl, conf, iters=3, n=12000, k=6, d=16):
    drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=k, d=d,
                         inp=f"synthetic:{n}:5", split_points=2000)
    for _ in range(iters):
        assert drv.step()["points"] == n
    return drv


def test_simulated_gpu_slots_take_every_map_and_match_cpu_bits():
    conf = _sim_conf()
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = _kmeans(cl, conf)
        cs = drv.history[-1]["counters"]
        assert cs.get(JIP, "GPU_MAP_TASKS") == 6 and cs.get(JIP, "CPU_MAP_TASKS") == 0
        c_gpu = drv.centroids()
    plain = JobConf()
    with LocalCluster(plain, num_trackers=1, cpu_slots=2) as cl:
        c_cpu = _kmeans(cl, plain).centroids()
    # int64 fixed-point partials: identical regardless of where maps ran
    assert torch.equal(c_gpu, c_cpu)


def test_hybrid_policy_keeps_slow_cpu_slots_idle():
    # GPU tasks 1 ms, CPU tasks 40 ms: after the CPU probe, min-makespan gives
    # the CPU slots nothing while the GPU queue can absorb the job
    conf = _sim_conf(**{"hbmr.scheduler.policy": "hybrid", "hbmr.gpu.simulate.task.ms": 1,
                        "hbmr.gpu.queue.depth": 8})
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=2) as cl:
        for _ in range(3):
            rj = cl.submit_job(split_sleep_conf(32, map_ms=40, base=conf))
            rj.waitForCompletion(60)
            assert rj.isSuccessful(), rj.getFailureInfo()
        cs = rj.getCounters()
        assert cs.get(JIP, "GPU_MAP_TASKS") >= 31
        assert cs.get(JIP, "CPU_MAP_TASKS") <= 1
        assert rj._impl.jip.result[0]["maps"] == 32


def test_stock_policy_uses_cpu_slots_too():
    conf = _sim_conf(**{"hbmr.scheduler.policy": "stock", "hbmr.gpu.simulate.task.ms": 5,
                        "hbmr.gpu.queue.depth": 1})
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=2) as cl:
        rj = cl.submit_job(split_sleep_conf(24, map_ms=5, base=conf))
        rj.waitForCompletion(60)
        assert rj.isSuccessful(), rj.getFailureInfo()
        cs = rj.getCounters()
        assert cs.get(JIP, "CPU_MAP_TASKS") > 0 and cs.get(JIP, "GPU_MAP_TASKS") > 0
        assert cs.get(JIP, "CPU_MAP_TASKS") + cs.get(JIP, "GPU_MAP_TASKS") == 24


def test_classic_sleep_job_runs_on_cluster():
    with LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) as cl:
        rj = JobClient.runJob(sleep_job_conf(maps=4, reduces=2, map_ms=5, reduce_ms=5,
                                             reduce_count=3), cluster=cl, verbose=False)
        assert rj.isSuccessful(), rj.getFailureInfo()
        cs = rj.getCounters()
        assert cs.get("org.apache.hadoop.mapred.Task$Counter", "REDUCE_INPUT_GROUPS") == 6


def test_tracer_records_task_flow_and_exports_chrome(tmp_path):
    conf = _sim_conf()
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        TRACE.clear()
        TRACE.enable()
        try:
            rj = cl.submit_job(split_sleep_conf(8, base=conf))
            rj.waitForCompletion(30)
        finally:
            TRACE.disable()
    names = {e[3] for e in TRACE.events}
    assert {"jt.submit", "gpu.launch", "gpu.complete", "tt.finish", "jt.job_finished"} <= names
    out = tmp_path / "trace.json"
    TRACE.to_chrome(str(out))
    doc = json.loads(out.read_text())
    assert any(e.get("cname") == "good" for e in doc["traceEvents"])   # GPU-coloured tasks
    TRACE.to_jsonl(str(tmp_path / "trace.jsonl"))
    assert (tmp_path / "trace.jsonl").read_text().count("\n") == len(TRACE.events)
    TRACE.clear()


def test_split_cache_scan_policy_keeps_a_resident_fraction():
    """Cyclic access to more splits than fit: LRU never hits, scan keeps the
    first ones resident and streams the rest (out-of-core iterations)."""
    from hbmr.gpu.split_cache import SplitCache
    for policy, want_hits in (("lru", 0), ("scan", 3 * 4)):
        c = SplitCache({0: 400}, policy=policy)
        for _ in range(4):
            for i in range(10):
                c.get_or_load(f"s{i}", 0, lambda: object(), lambda _d: 100)
        assert c.hits == want_hits, policy
        assert c.bytes_on(0) <= 400


def test_kmeans_beyond_hbm_streams_splits_with_scan_cache():
    """A data set larger than the (simulated) HBM split cache: every iteration
    is exact and the resident fraction hits."""
    cap = 3 * 2000 * 16 * 4 + 1024       # three of the six fp32 splits
    conf = _sim_conf(**{"hbmr.gpu.split.cache.bytes": cap,
                        "hbmr.gpu.split.cache.policy": "scan"})
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = _kmeans(cl, conf, iters=4)
        cache = cl.trackers[0].split_cache
        c_small = drv.centroids()
        assert 0 < cache.bytes_on(0) <= cap
        assert cache.hits >= 3 * 3 and cache.bypassed >= 3 * 3
    plain = JobConf()
    with LocalCluster(plain, num_trackers=1, cpu_slots=2) as cl:
        c_cpu = _kmeans(cl, plain, iters=4).centroids()
    assert torch.equal(c_small, c_cpu)


def test_split_cache_charges_derived_state_and_notifies_evictions():
    """Device state derived from a split (the delta combiner's reference
    partitions) is charged to its cache entry and dropped with it."""
    from hbmr.gpu.split_cache import SplitCache
    c = SplitCache({0: 100})
    gone = []
    c.add_listener(lambda k, d: gone.append((k, d)))
    c.put("a", 0, "A", 40)
    c.put("b", 0, "B", 40)
    assert c.charge("a", 0, 10) and c.bytes_on(0) == 90
    assert not c.charge("zz", 0, 5)            # not resident: nothing charged
    c.get("a", 0)                               # a is the most recent
    c.charge("a", 0, 20)                        # 110 > 100: b goes, a stays
    assert gone == [("b", 0)] and c.bytes_on(0) == 70
    c.put("c", 0, "C", 50)                      # evicts a (70 + 50 > 100)
    assert ("a", 0) in gone and c.bytes_on(0) == 50
    c.clear(0)
    assert ("c", 0) in gone and c.bytes_on(0) == 0


def _iteration_ms(conf, iters=6):
    import time as _t
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=6,
                             d=16, inp="synthetic:12000:5", split_points=2000)
        drv.step()
        t0 = _t.time()
        for _ in range(iters):
            assert drv.step()["points"] == 12000
        return (_t.time() - t0) * 1e3 / iters, drv.centroids()


def test_report_without_assignment_does_not_stall_on_response_numbers():
    """hbmr.tracker.report.assign=false: a report's actions go back through the
    long-poll, numbered only there — numbering them in the report (whose
    reply carries nothing) left a gap the tracker waited 2 s on."""
    ms, got = _iteration_ms(_sim_conf(**{"hbmr.tracker.report.assign": "false"}))
    ms_ref, want = _iteration_ms(_sim_conf())
    assert torch.equal(got, want)
    assert ms < 1000, ms


@pytest.mark.timeout(60)
def test_lost_report_reply_is_resent():
    """A report reply lost after the JobTracker processed it (the RPC raised):
    the tracker takes the numbered responses back (JobTracker.resend) instead
    of losing their launches / commit approvals and stalling 2 s on the gap."""
    from hbmr.mapred.jobtracker import JobTracker
    real = JobTracker.report
    state = {"n": 0, "lost": 0}

    def flaky(self, status, assign=False):
        r = real(self, status, assign)
        if assign and r.get("actions"):
            state["n"] += 1
        if assign and r.get("actions") and state["n"] % 3 == 1:
            state["lost"] += 1
            raise ConnectionError("reply lost")
        return r

    JobTracker.report = flaky
    try:
        ms, got = _iteration_ms(_sim_conf())
    finally:
        JobTracker.report = real
    _, want = _iteration_ms(_sim_conf())
    assert state["lost"] > 0
    assert torch.equal(got, want)
    assert ms < 1000, ms
