"""Pre-staged iteration jobs (hbmr/gpu/gates.py, JobTracker._maybe_stage): a
job that depends on a running collective split job has its GPU maps launched
early, held on each tracker until the predecessor's reduce there released its
result, and its own collective reduce launched before its maps finished
("expect" mode).  The reference can only start the next K-Means iteration
after a JobControl poll (JobControl.java) and a >= 3 s heartbeat
(MRConstants.java:28).  Simulated GPU slots keep these tests on the CPU."""
import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K

JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"


def _conf(worker, prestage=True, task_ms=3.0, **kw):
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_boolean("hbmr.gpu.worker.process", worker)
    conf.set_float("hbmr.gpu.simulate.task.ms", task_ms)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
    conf.set_int("hbmr.gpu.queue.depth", 16)
    conf.set_int("mapred.task.timeout", 0)
    conf.set_boolean("hbmr.job.prestage", prestage)
    for k, v in kw.items():
        conf.set(k, str(v))
    return conf


def _run(conf, tmp, steps=5, depth=2, trackers=1):
    conf.set("mapred.local.dir", str(tmp))
    gpus = [[i] for i in range(trackers)]
    with LocalCluster(conf, num_trackers=trackers, gpus=gpus, cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                             d=8, inp="synthetic:8000:3", split_points=1000)
        drv.prefetch_delay = 0.0
        for s in range(steps):
            assert drv.step(prefetch=min(depth, steps - 1 - s))["points"] == 8000
        jobs = [cl.jt.jobs[h["job"]] for h in drv.history]
        events = [e for e in cl.jt.history.events]
        return drv.centroids(), jobs, events, drv


@pytest.mark.parametrize("worker", [False, True])
def test_staged_iterations_run_ahead_and_give_the_same_centroids(worker, tmp_path):
    want, _, ev0, _ = _run(_conf(worker, prestage=False), tmp_path / "plain")
    assert not any(e["event"] == "JOB_STAGED" for e in ev0)
    got, jobs, events, _ = _run(_conf(worker), tmp_path / "staged")
    assert torch.equal(got, want)
    assert sum(e["event"] == "JOB_STAGED" for e in events) >= 3
    for prev, nxt in zip(jobs, jobs[1:]):
        # a staged job never completes before the job it depends on
        assert nxt.status.finish_time >= prev.status.finish_time > 0
    # maps of later iterations were launched before their predecessor finished
    ahead = [nxt.t_first_map < prev.status.finish_time for prev, nxt in zip(jobs, jobs[1:])]
    assert sum(ahead) >= 2, ahead
    # and collective reduces started before the last map of their job finished
    assert any(j.t_first_reduce and j.t_maps_done and j.t_first_reduce < j.t_maps_done
               for j in jobs)


def test_staged_iterations_over_two_trackers(tmp_path):
    want, _, _, _ = _run(_conf(False, prestage=False), tmp_path / "plain", trackers=2)
    got, jobs, events, _ = _run(_conf(False), tmp_path / "staged", trackers=2)
    assert torch.equal(got, want)
    assert any(e["event"] == "JOB_STAGED" for e in events)


def test_staged_job_survives_a_worker_crash_in_its_predecessor(tmp_path):
    """Iteration 3's map crashes the GPU worker while iteration 4 is staged on
    it: the held staged attempts die with the worker, everything re-runs and
    the answer is the same."""
    want, _, _, _ = _run(_conf(True, prestage=False), tmp_path / "plain")
    got, jobs, events, _ = _run(
        _conf(True, **{"hbmr.faultinject.worker.exit.attempt": "_0003_m_000002_0"}),
        tmp_path / "crash")
    assert torch.equal(got, want)


def test_killing_a_staged_job_fails_its_dependents(tmp_path):
    conf = _conf(False, task_ms=20.0)
    conf.set("mapred.local.dir", str(tmp_path))
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                             d=8, inp="synthetic:8000:3", split_points=1000)
        drv.prefetch_delay = 0.0
        drv.step(prefetch=2)
        a, b = drv._ahead
        drv.cancel_prefetch()
        assert a.waitForCompletion(20) and b.waitForCompletion(20)
        assert a.status().state == "KILLED"
        assert b.status().state in ("KILLED", "FAILED")
        assert not cl.jt.staged
        # the cluster still runs iterations afterwards
        drv2 = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                              d=8, inp="synthetic:8000:3", split_points=1000)
        assert drv2.step()["points"] == 8000


@pytest.mark.timeout(90)
@pytest.mark.parametrize("worker", [False, True])
def test_staged_maps_do_not_take_the_queue_their_gate_waits_on(worker, tmp_path):
    """A job with more maps than one GPU queue holds (8 maps, 2 slots x depth 1):
    the next iteration's staged maps have their own budget, so they cannot
    fill the queue while the job they wait for still has maps to launch (that
    deadlocked: its reduce, which opens their gate, needed those maps)."""
    want, _, _, _ = _run(_conf(worker, prestage=False), tmp_path / "plain", steps=4)
    conf = _conf(worker, **{"hbmr.gpu.queue.depth": 1})
    got, jobs, events, _ = _run(conf, tmp_path / "staged", steps=4)
    assert torch.equal(got, want)
    assert sum(e["event"] == "JOB_STAGED" for e in events) >= 2


@pytest.mark.timeout(120)
@pytest.mark.parametrize("worker", [False, True])
def test_predecessor_reduce_failing_after_release_restarts_its_staged_job(worker, tmp_path):
    """Iteration 2's reduce opens the gate of staged iteration 3 on poisoned
    centroids and then FAILS: iteration 2 re-runs its gang, iteration 3's maps
    that ran on the poisoned result re-run behind the new gate, and the
    answer equals the unstaged run's."""
    want, _, _, _ = _run(_conf(worker, prestage=False), tmp_path / "plain", steps=4)
    conf = _conf(worker, **{"hbmr.faultinject.reduce.fail.after.release.attempt":
                            "_0002_r_000000_0"})
    got, jobs, events, _ = _run(conf, tmp_path / "late", steps=4)
    names = [e["event"] for e in events]
    assert "COLLECTIVE_RESTART" in names
    assert torch.equal(got, want)


@pytest.mark.timeout(60)
def test_collective_restart_closes_the_gate_on_every_gpu_tracker(tmp_path):
    """A gang restarted with no job staged on it yet still closes its gate on
    every GPU tracker: a failed member may have opened it already, and a job
    staged on the restarted job later must wait for the new reduce instead of
    passing that stale open gate (the close was sent only when a
    staged job already existed)."""
    conf = _conf(False, task_ms=50.0)
    conf.set("mapred.local.dir", str(tmp_path))
    with LocalCluster(conf, num_trackers=2, gpus=[[0], [1]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                             d=8, inp="synthetic:8000:3", split_points=1000)
        rj = drv.submit(drv._job_conf(0))
        jt = cl.jt
        jid = str(rj.getID())
        with jt.lock:
            jip = jt.jobs[jid]
            for t in jt.trackers.values():
                t.extra_actions = [x for x in t.extra_actions if x.get("type") != "close_gate"]
            jt._restart_collective(jip, "test")
            closes = {name: [x for x in t.extra_actions
                             if x.get("type") == "close_gate" and x.get("job_id") == jid]
                      for name, t in jt.trackers.items() if t.status.gpus}
        assert len(closes) == 2 and all(len(v) == 1 for v in closes.values()), closes
        assert rj.waitForCompletion(60)
        assert rj.status().state == "SUCCEEDED"


@pytest.mark.timeout(120)
def test_job_staged_after_a_collective_restart_waits_for_the_new_reduce(tmp_path):
    """Iteration 2's reduce opens its gate on poisoned centroids and fails;
    iteration 3 is submitted (and staged on iteration 2) only AFTER that
    restart.  The restart closed the gate on every GPU tracker, so iteration
    3's maps wait for the re-run reduce instead of passing the stale open gate
    (the gate was closed only when a staged job already existed)."""
    want, _, _, _ = _run(_conf(False, prestage=False, task_ms=20.0), tmp_path / "plain", steps=4)
    conf = _conf(False, task_ms=20.0, **{"hbmr.faultinject.reduce.fail.after.release.attempt":
                                         "_0002_r_000000_0"})
    conf.set("mapred.local.dir", str(tmp_path / "late"))
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=5,
                             d=8, inp="synthetic:8000:3", split_points=1000)
        drv.step()                                 # iteration 1
        jt = cl.jt
        real_submit = drv.submit

        def submit_after_restart(job):
            # iteration 3 (depends on iteration 2): hold its submission until
            # iteration 2's gang has failed and restarted
            if job.get("hbmr.job.depends.on"):
                for _ in range(2000):
                    if any(e["event"] == "COLLECTIVE_RESTART" for e in jt.history.events):
                        break
                    import time as _t
                    _t.sleep(0.005)
            return real_submit(job)

        drv.submit = submit_after_restart
        drv.prefetch_delay = 0.0
        drv.step(prefetch=1)                       # iteration 2, iteration 3 staged late
        drv.step()
        drv.step()
        got = drv.centroids()
        names = [e["event"] for e in jt.history.events]
    assert "COLLECTIVE_RESTART" in names
    restart = names.index("COLLECTIVE_RESTART")
    if "JOB_STAGED" not in names[restart:]:
        # on a loaded host the re-run reduce can finish before iteration 3 is
        # submitted: its dependency is done, so there is nothing to stage
        sub3 = names.index("JOB_SUBMITTED", restart)
        assert "JOB_FINISHED" in names[restart:sub3], names
    assert torch.equal(got, want)
