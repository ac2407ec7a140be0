"""Fair-scheduler allocation file + job limits (contrib/fairscheduler
PoolManager.java:57-400, FairScheduler.updateRunnability) and the capacity
scheduler's job-initialisation / submission limits
(CapacitySchedulerQueue.java:378-400, 1227-1345) — the reference's
TestFairScheduler / TestCapacityScheduler job-limit cases in miniature."""
import os
import time

import pytest

from hbmr.examples.sleepjob import split_sleep_conf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.mapred.scheduler.pools import (INF, AllocationConfigurationException, Allocations,
                                         PoolManager)

ALLOC = """<?xml version="1.0"?>
<allocations>
  <pool name="research">
    <minMaps>3</minMaps><minReduces>1</minReduces><maxMaps>8</maxMaps>
    <maxRunningJobs>{pool_max}</maxRunningJobs><weight>2.5</weight>
    <minSharePreemptionTimeout>30</minSharePreemptionTimeout>
    <schedulingMode>fifo</schedulingMode>
  </pool>
  <user name="bob"><maxRunningJobs>7</maxRunningJobs></user>
  <userMaxJobsDefault>4</userMaxJobsDefault>
  <fairSharePreemptionTimeout>120</fairSharePreemptionTimeout>
  <defaultPoolSchedulingMode>fair</defaultPoolSchedulingMode>
</allocations>
"""


def _write(path, pool_max):
    path.write_text(ALLOC.format(pool_max=pool_max))


def test_allocation_file_parse_and_lookups(tmp_path):
    f = tmp_path / "fair.xml"
    _write(f, 2)
    conf = JobConf()
    conf.set("mapred.fairscheduler.allocation.file", str(f))
    conf.set("hbmr.fair.pool.other.weight", "3.0")
    pm = PoolManager(conf)
    assert pm.pool_value("research", "minMaps", 0) == 3
    assert pm.pool_value("research", "maxMaps", INF) == 8
    assert pm.pool_value("research", "weight", 1.0) == 2.5
    assert pm.pool_value("research", "mode", "fair") == "fifo"
    assert pm.pool_value("other", "weight", 1.0) == 3.0       # conf-key fallback
    assert pm.pool_value("other", "mode", "fair") == "fair"
    assert pm.pool_max_jobs("research") == 2 and pm.pool_max_jobs("other") == INF
    assert pm.user_max_jobs("bob") == 7 and pm.user_max_jobs("carol") == 4
    assert pm.fair_share_timeout(600.0) == 120.0
    bad = tmp_path / "bad.xml"
    bad.write_text("<pools/>")
    with pytest.raises(AllocationConfigurationException):
        Allocations.parse(bad)


def test_allocation_reload_waits_and_survives_bad_files(tmp_path):
    f = tmp_path / "fair.xml"
    _write(f, 1)
    conf = JobConf()
    conf.set("mapred.fairscheduler.allocation.file", str(f))
    conf.set("mapred.fairscheduler.allocation.reload.interval", "0")
    conf.set("mapred.fairscheduler.allocation.reload.wait", "0.2")
    pm = PoolManager(conf)
    assert pm.pool_max_jobs("research") == 1
    time.sleep(0.02)
    _write(f, 5)
    pm.reload_if_necessary()                   # too fresh: may be half-written
    assert pm.pool_max_jobs("research") == 1
    time.sleep(0.25)
    pm.reload_if_necessary()
    assert pm.pool_max_jobs("research") == 5
    time.sleep(0.02)
    f.write_text("<allocations><pool name='research'><maxRunningJobs>x")
    past = time.time() - 1
    os.utime(f, (past + 0.9, past + 0.9))
    time.sleep(0.15)
    pm.reload_if_necessary()                   # unparsable: keep the old allocations
    assert pm.pool_max_jobs("research") == 5


def _fair_conf(alloc):
    conf = JobConf()
    conf.set("mapred.jobtracker.taskScheduler", "hbmr.mapred.scheduler.fair:FairScheduler")
    conf.set("mapred.fairscheduler.allocation.file", str(alloc))
    conf.set("mapred.fairscheduler.allocation.reload.interval", "0")
    conf.set("mapred.fairscheduler.allocation.reload.wait", "0")
    conf.set_int("hbmr.heartbeat.interval.ms", 20)
    return conf


def _overlap(ra, rb, until, timeout=30):
    """True if both jobs ever had running maps at the same time."""
    t0 = time.time()
    both = False
    while not until() and time.time() - t0 < timeout:
        a, b = ra._impl.jip, rb._impl.jip
        if (a.running_cpu + a.running_gpu) and (b.running_cpu + b.running_gpu):
            both = True
        time.sleep(0.003)
    return both


def test_pool_max_running_jobs_serialises_a_pool_then_reload_lifts_it(tmp_path):
    alloc = tmp_path / "fair.xml"
    _write(alloc, 1)
    conf = _fair_conf(alloc)
    with LocalCluster(conf, num_trackers=1, cpu_slots=4) as cl:
        jobs = []
        for _ in range(2):
            j = split_sleep_conf(6, map_ms=80, base=conf)
            j.set("mapred.fairscheduler.pool", "research")
            jobs.append(cl.submit_job(j))
        ra, rb = jobs
        assert not _overlap(ra, rb, lambda: ra.isComplete() and rb.isComplete())
        assert ra.isSuccessful() and rb.isSuccessful()
        # raise the limit in the file: picked up without a restart
        _write(alloc, 2)
        time.sleep(0.05)
        jobs = []
        for _ in range(2):
            j = split_sleep_conf(6, map_ms=150, base=conf)  # fifo pool: b fills a's tail
            j.set("mapred.fairscheduler.pool", "research")
            jobs.append(cl.submit_job(j))
        ra, rb = jobs
        assert _overlap(ra, rb, lambda: ra.isComplete() and rb.isComplete())
        assert cl.jt.scheduler.pools.reloads >= 2


def test_user_max_jobs_default(tmp_path):
    alloc = tmp_path / "fair.xml"
    alloc.write_text("<allocations><userMaxJobsDefault>1</userMaxJobsDefault></allocations>")
    conf = _fair_conf(alloc)
    with LocalCluster(conf, num_trackers=1, cpu_slots=4) as cl:
        rs = []
        for user in ("alice", "alice", "bob"):
            j = split_sleep_conf(3, map_ms=100, base=conf)
            j.set("user.name", user)
            rs.append(cl.submit_job(j))
        a1, a2, b = rs
        same_user = _overlap(a1, a2, lambda: a1.isComplete() and a2.isComplete())
        assert not same_user
        for r in rs:
            r.waitForCompletion(30)
            assert r.isSuccessful()


def _cap_conf(**kw):
    conf = JobConf()
    conf.set("mapred.jobtracker.taskScheduler", "hbmr.mapred.scheduler.fair:CapacityScheduler")
    conf.set("mapred.queue.names", "default")
    conf.set_int("hbmr.heartbeat.interval.ms", 20)
    for k, v in kw.items():
        conf.set(k, str(v))
    return conf


def test_capacity_initialises_at_most_max_jobs_and_refuses_beyond_accept_limit():
    conf = _cap_conf(**{"mapred.capacity-scheduler.maximum-system-jobs": 1,
                        "mapred.capacity-scheduler.queue.default.init-accept-jobs-factor": 2})
    with LocalCluster(conf, num_trackers=1, cpu_slots=4) as cl:
        ra = cl.submit_job(split_sleep_conf(3, map_ms=100, base=conf))
        rb = cl.submit_job(split_sleep_conf(3, map_ms=100, base=conf))
        rc = cl.submit_job(split_sleep_conf(3, map_ms=10, base=conf))   # 1 × 2 accepted
        rc.waitForCompletion(10)
        assert not rc.isSuccessful() and "jobs to accept" in rc.getFailureInfo()
        assert not _overlap(ra, rb, lambda: ra.isComplete() and rb.isComplete())
        assert ra.isSuccessful() and rb.isSuccessful()


def test_capacity_refuses_a_job_above_the_per_user_task_limit():
    conf = _cap_conf(**{
        "mapred.capacity-scheduler.queue.default.maximum-initialized-active-tasks-per-user": 4})
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(split_sleep_conf(8, base=conf))
        rj.waitForCompletion(10)
        assert not rj.isSuccessful() and "tasks per-user" in rj.getFailureInfo()
        ok = cl.submit_job(split_sleep_conf(2, base=conf))
        ok.waitForCompletion(10)
        assert ok.isSuccessful()
