"""GPU-aware Fair and Capacity schedulers: shares of CPU and GPU slots
(the reference's contrib schedulers were not GPU-aware)."""
import threading
import time

from hbmr.examples.sleepjob import split_sleep_conf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.mapred.scheduler.fair import water_fill


def test_water_fill():
    assert water_fill(10, [100, 100], [1, 1]) == [5.0, 5.0]
    assert water_fill(10, [2, 100], [1, 1]) == [2.0, 8.0]
    s = water_fill(12, [100, 100, 100], [1, 2, 3])
    assert [round(x) for x in s] == [2, 4, 6]
    assert water_fill(10, [100, 100], [1, 1], mins=[8, 0]) == [9.0, 1.0]


def _conf(scheduler, **kw):
    conf = JobConf()
    conf.set("mapred.jobtracker.taskScheduler", scheduler)
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
    conf.set_int("hbmr.gpu.queue.depth", 1)
    conf.set_float("hbmr.gpu.simulate.task.ms", 20)
    conf.set("hbmr.scheduler.policy", "stock")
    for k, v in kw.items():
        conf.set(k, str(v))
    return conf


def _run_two(conf, confs):
    """Submit two jobs together and sample their concurrent GPU occupancy."""
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        jobs = [cl.submit_job(c) for c in confs]
        samples = []
        stop = threading.Event()

        def sample():
            while not stop.is_set():
                samples.append(tuple(rj._impl.jip.running_gpu for rj in jobs))
                time.sleep(0.005)
        t = threading.Thread(target=sample, daemon=True)
        t.start()
        try:
            for rj in jobs:
                rj.waitForCompletion(60)
                assert rj.isSuccessful(), rj.getFailureInfo()
        finally:
            stop.set()
            t.join()
    return [s for s in samples if s[0] and s[1]]


def test_fair_scheduler_shares_gpu_slots_between_pools():
    conf = _conf("hbmr.mapred.scheduler.fair:FairScheduler")
    a = split_sleep_conf(30, base=conf)
    a.set("mapred.fairscheduler.pool", "a")
    b = split_sleep_conf(30, base=conf)
    b.set("mapred.fairscheduler.pool", "b")
    both = _run_two(conf, [a, b])
    # FIFO would run job 1 alone first; fair sharing runs them side by side
    assert len(both) > 3
    assert all(x <= 1 and y <= 1 for x, y in both)


def test_capacity_scheduler_runs_both_queues():
    conf = _conf("hbmr.mapred.scheduler.fair:CapacityScheduler",
                 **{"mapred.queue.names": "prod,dev",
                    "mapred.capacity-scheduler.queue.prod.capacity": 50,
                    "mapred.capacity-scheduler.queue.dev.capacity": 50})
    a = split_sleep_conf(30, base=conf)
    a.set("mapred.job.queue.name", "prod")
    b = split_sleep_conf(30, base=conf)
    b.set("mapred.job.queue.name", "dev")
    both = _run_two(conf, [a, b])
    assert len(both) > 3
