"""Contrib scheduler depth and Vaidya's diagnosis rules.

* FairScheduler preemption (contrib/fairscheduler FairScheduler.java:837):
  a starved pool takes slots back from a pool above its fair share;
* CapacityScheduler user limits (CapacitySchedulerQueue.java:724) and
  memory-based slot matching (CapacityTaskScheduler.java:315-340), plus the
  JobTracker's memory-requirement check at submission;
* Vaidya post-execution rules (contrib/vaidya postexdiagnosis/tests):
  MapSideDiskSpill, BalancedReducePartitioning, Maps/ReducesReExecutionImpact,
  ReadingHDFSFilesAsSideEffect — same impact formulas, on synthetic job
  statistics and on real job history files."""
import os
import time

import pytest

from hbmr.examples.sleepjob import sleep_job_conf, split_sleep_conf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.webui.history import diagnose, load_history, vaidya_rules

JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"
TASK = "org.apache.hadoop.mapred.Task$Counter"


# ----------------------------------------------------------------- fair preemption
def test_fair_scheduler_preempts_for_a_starved_pool():
    conf = JobConf()
    conf.set("mapred.jobtracker.taskScheduler", "hbmr.mapred.scheduler.fair:FairScheduler")
    conf.set_boolean("mapred.fairscheduler.preemption", True)
    conf.set("hbmr.fair.pool.b.minMaps", "2")
    conf.set("hbmr.fair.pool.b.minSharePreemptionTimeout", "0.2")
    conf.set_int("hbmr.heartbeat.interval.ms", 20)
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        a = split_sleep_conf(6, map_ms=2500, base=conf)     # long maps fill both CPU slots
        a.set("mapred.fairscheduler.pool", "a")
        ra = cl.submit_job(a)
        t0 = time.time()
        while ra._impl.jip.running_cpu < 2 and time.time() - t0 < 10:
            time.sleep(0.01)
        b = split_sleep_conf(2, map_ms=50, base=conf)
        b.set("mapred.fairscheduler.pool", "b")
        rb = cl.submit_job(b)
        rb.waitForCompletion(30)
        tb = time.time() - t0
        assert rb.isSuccessful(), rb.getFailureInfo()
        # b finished long before a's 2.5 s maps could have freed a slot
        assert tb < 2.0
        assert cl.jt.scheduler.preempted >= 1
        assert ra._impl.jip.counters.get(JIP, "NUM_PREEMPTED_TASKS") >= 1
        ra.killJob()


# ----------------------------------------------------------------- capacity scheduler
def _cap_conf(**kw):
    conf = JobConf()
    conf.set("mapred.jobtracker.taskScheduler", "hbmr.mapred.scheduler.fair:CapacityScheduler")
    conf.set("mapred.queue.names", "default")
    conf.set_int("hbmr.heartbeat.interval.ms", 20)
    for k, v in kw.items():
        conf.set(k, str(v))
    return conf


def _peak_running(cl, jobs, until):
    peak = [0] * len(jobs)
    t0 = time.time()
    while not until() and time.time() - t0 < 30:
        for i, rj in enumerate(jobs):
            peak[i] = max(peak[i], rj._impl.jip.running_cpu)
        time.sleep(0.003)
    return peak


def test_capacity_user_limit_splits_a_queue_between_users():
    conf = _cap_conf(**{"mapred.capacity-scheduler.queue.default.minimum-user-limit-percent": 50})
    with LocalCluster(conf, num_trackers=1, cpu_slots=4) as cl:
        a = split_sleep_conf(12, map_ms=150, base=conf)
        a.set("user.name", "alice")
        b = split_sleep_conf(12, map_ms=150, base=conf)
        b.set("user.name", "bob")
        ra, rb = cl.submit_job(a), cl.submit_job(b)
        peak = _peak_running(cl, [ra, rb], lambda: rb.isComplete() and ra.isComplete())
        assert ra.isSuccessful() and rb.isSuccessful()
        # each user is held to half of the 4 CPU slots while the other has demand
        assert peak[0] <= 2 and peak[1] <= 2 and peak[1] >= 1


def test_capacity_memory_matching_uses_several_slots_per_task():
    conf = _cap_conf(**{"mapred.cluster.map.memory.mb": 1024})
    with LocalCluster(conf, num_trackers=1, cpu_slots=4) as cl:
        job = split_sleep_conf(8, map_ms=40, base=conf)
        job.set_int("mapred.job.map.memory.mb", 2048)          # 2 slots per task
        rj = cl.submit_job(job)
        peak = _peak_running(cl, [rj], rj.isComplete)
        assert rj.isSuccessful()
        assert peak[0] <= 2            # 4 slots / 2 per task
        tr = next(iter(cl.jt.trackers.values()))
        assert tr.running_cpu == 0     # every slot given back


def test_jobtracker_rejects_jobs_above_the_cluster_memory_limit():
    conf = _cap_conf(**{"mapred.cluster.max.map.memory.mb": 4096})
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        job = split_sleep_conf(2, base=conf)
        job.set_int("mapred.job.map.memory.mb", 8192)
        rj = cl.submit_job(job)
        rj.waitForCompletion(10)
        assert not rj.isSuccessful()
        assert "exceeds the cluster maximum" in rj.getFailureInfo()


# ----------------------------------------------------------------- Vaidya rules
def _att(typ, ok=True, counters=None):
    return {"type": typ, "successful": ok, "state": "SUCCEEDED" if ok else "FAILED",
            "gpu": False, "start": 0.0, "finish": 1.0, "device_time": 0.0, "tracker": "t",
            "speculative": False, "diagnostic": "", "counters": counters or {}}


def test_vaidya_rule_formulas():
    job = {"maps": 4, "reduces": 4, "submit": 0, "finish": 2, "counters": {
        TASK: {"MAP_OUTPUT_BYTES": 1000, "MAP_INPUT_BYTES": 1000},
        JIP: {"TOTAL_LAUNCHED_MAPS": 6, "TOTAL_LAUNCHED_REDUCES": 4},
        "FileSystemCounters": {"HDFS_BYTES_READ": 1500}}}
    maps = [_att("MAP", counters={"FileSystemCounters": {"FILE_BYTES_WRITTEN": 1000}})
            for _ in range(4)]
    reds = [_att("REDUCE", counters={TASK: {"REDUCE_INPUT_RECORDS": r}})
            for r in (970, 10, 10, 10)]
    got = {f["rule"]: f["impact"] for f in vaidya_rules(job, maps + reds)}
    assert got["MapSideDiskSpill"] == pytest.approx(1.0)            # (4000-1000)/1000 ≥ 3
    assert got["BalancedReducePartitioning"] == pytest.approx(0.75)  # 1 of 4 reducers
    assert got["MapsReExecutionImpact"] == pytest.approx(0.5)
    assert got["ReducesReExecutionImpact"] == pytest.approx(0.0)
    assert got["ReadingHDFSFilesAsSideEffect"] == pytest.approx(0.75)  # 1.5 / 2


def test_vaidya_rules_on_real_job_history(tmp_path):
    from hbmr.mapred.lib.basic import HashPartitioner   # noqa: F401
    conf = JobConf()
    conf.set("hbmr.history.dir", str(tmp_path / "hist"))
    conf.set_float("hbmr.faultinject.probability", 0.25)
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        job = sleep_job_conf(maps=8, reduces=4, map_ms=1, reduce_ms=1, base=conf)
        job.set_int("mapred.map.max.attempts", 20)
        job.set_int("mapred.reduce.max.attempts", 20)
        rj = cl.submit_job(job)
        rj.waitForCompletion(60)
        assert rj.isSuccessful(), rj.getFailureInfo()
    files = os.listdir(tmp_path / "hist")
    job_rec, attempts = load_history(str(tmp_path / "hist" / files[0]))
    rules = {f["rule"]: f for f in diagnose(job_rec, attempts)}
    assert "MapsReExecutionImpact" in rules
    launched = job_rec["counters"][JIP]["TOTAL_LAUNCHED_MAPS"]
    assert rules["MapsReExecutionImpact"]["impact"] == pytest.approx(
        min(1.0, (launched - 8) / 8))
    assert all(0.0 <= f["impact"] <= 1.0 for f in rules.values() if "impact" in f)


def test_dependent_job_runs_after_success_and_fails_with_its_dependency():
    """hbmr.job.depends.on (JobControl's depending jobs): held until the job it
    names succeeds; failed if that job is killed."""
    from hbmr.examples.sleepjob import split_sleep_conf
    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.mapred.jobtracker import DEPENDS_KEY
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        a = cl.submit_job(split_sleep_conf(4, map_ms=50.0))
        bc = split_sleep_conf(2, map_ms=1.0)
        bc.set(DEPENDS_KEY, str(a.getID()))
        b = cl.submit_job(bc)
        assert b.status().state == "PREP"
        assert b.waitForCompletion(30) and a.waitForCompletion(30)
        assert b.isSuccessful()
        assert b._impl.jip.release_time >= a._impl.jip.status.finish_time
        c = cl.submit_job(split_sleep_conf(4, map_ms=2000.0))
        dc = split_sleep_conf(2, map_ms=1.0)
        dc.set(DEPENDS_KEY, str(c.getID()))
        d = cl.submit_job(dc)
        c.killJob()
        assert d.waitForCompletion(30)
        assert d.status().state == "FAILED" and "depends on" in d.getFailureInfo()
