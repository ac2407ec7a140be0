"""JobTracker restart recovery (RecoveryManager, mapred.jobtracker.restart.recover;
the reference's TestJobTrackerRestart / TestRecoveryManager): unfinished jobs
are re-submitted under their old ids after a restart, trackers re-register."""
import collections
import json
import os
import time

from hbmr.examples.sleepjob import split_sleep_conf
from hbmr.mapred import JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.models import wordcount


def _wait(pred, timeout=20.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.01)
    return False


def _conf(tmp_path, recover=True):
    conf = JobConf()
    conf.set("mapred.system.dir", str(tmp_path / "system"))
    conf.set_boolean("mapred.jobtracker.restart.recover", recover)
    conf.set("hbmr.history.file", str(tmp_path / "history.jsonl"))
    return conf


def test_restart_recovers_running_job(tmp_path):
    conf = _conf(tmp_path)
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        job = split_sleep_conf(24, map_ms=40.0, base=conf)
        rj = cl.submit_job(job)
        jid = str(rj.getID())
        sysdir = tmp_path / "system" / jid
        assert (sysdir / "job.json").exists()
        assert _wait(lambda: any(t.is_complete() for t in rj._impl.jip.maps))
        jt2 = cl.restart_jobtracker()
        assert jt2.restart_count == 1
        assert _wait(lambda: jt2.get_job(jid) is not None)
        rj2 = jt2.get_job(jid)
        rj2.waitForCompletion(60)
        assert rj2.isSuccessful(), rj2.getFailureInfo()
        assert str(rj2.getID()) == jid
        assert not sysdir.exists()          # job files garbage-collected at the end
        # new jobs do not collide with the recovered id
        rj3 = cl.submit_job(split_sleep_conf(2, base=conf))
        rj3.waitForCompletion(30)
        assert rj3.isSuccessful() and str(rj3.getID()) != jid
    info = json.loads((tmp_path / "system" / "jobtracker.json").read_text())
    assert info["restart_count"] == 1 and info["trackers"] == 2


def test_restart_recovers_classic_job_output(tmp_path):
    d = tmp_path / "in"
    d.mkdir()
    cnt = collections.Counter()
    for i in range(6):
        words = [f"w{(i * 7 + j) % 11}" for j in range(300)]
        (d / f"f{i}").write_text(" ".join(words) + "\n")
        cnt.update(words)
    conf = _conf(tmp_path)
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        job = wordcount.make_job(str(d), str(tmp_path / "out"), reduces=2)
        rj = cl.submit_job(job)
        jid = str(rj.getID())
        cl.restart_jobtracker()
        assert _wait(lambda: cl.jt.get_job(jid) is not None)
        rj2 = cl.jt.get_job(jid)
        rj2.waitForCompletion(60)
        assert rj2.isSuccessful(), rj2.getFailureInfo()
    got = {}
    for fn in os.listdir(tmp_path / "out"):
        if fn.startswith("part-"):
            for line in open(tmp_path / "out" / fn):
                k, v = line.rstrip("\n").split("\t")
                got[k] = int(v)
    assert got == dict(cnt)


def test_restart_without_recovery_drops_jobs(tmp_path):
    conf = _conf(tmp_path, recover=False)
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        rj = cl.submit_job(split_sleep_conf(50, map_ms=20.0, base=conf))
        jid = str(rj.getID())
        jt2 = cl.restart_jobtracker()
        time.sleep(0.3)
        assert jt2.get_job(jid) is None
        assert not (tmp_path / "system" / jid).exists()
        # trackers re-registered and the new JT runs jobs
        rj2 = cl.submit_job(split_sleep_conf(3, base=conf))
        rj2.waitForCompletion(30)
        assert rj2.isSuccessful()
