"""Failure handling: task retries under fault injection,
tracker loss (running attempts failed, completed map outputs re-executed),
task timeouts, tracker blacklisting, speculative GPU backups of stragglers."""
import collections
import os
import time

import pytest

from hbmr.examples.sleepjob import sleep_job_conf, split_sleep_conf
from hbmr.io.writable import Text
from hbmr.mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper
from hbmr.mapred.cluster import LocalCluster
from hbmr.models import wordcount

JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"


def _words(tmp_path, files=4):
    d = tmp_path / "in"
    d.mkdir()
    cnt = collections.Counter()
    for i in range(files):
        lines = [" ".join(f"f{(i * 5 + j + t) % 13}" for t in range(j % 6)) for j in range(80)]
        (d / f"p{i}").write_text("\n".join(lines) + "\n")
        for ln in lines:
            cnt.update(ln.split())
    return d, cnt


def _read(out):
    res = {}
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            for line in open(os.path.join(out, fn)):
                k, v = line.rstrip("\n").split("\t")
                res[k] = int(v)
    return res


def test_fault_injection_retries_until_success(tmp_path):
    inp, cnt = _words(tmp_path)
    conf = JobConf()
    conf.set_float("hbmr.faultinject.probability", 0.3)
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        job = wordcount.make_job(str(inp), str(tmp_path / "out"), reduces=2)
        job.set_int("mapred.map.max.attempts", 12)
        job.set_int("mapred.reduce.max.attempts", 12)
        job.set_num_map_tasks(8)
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
    assert _read(tmp_path / "out") == dict(cnt)
    cs = rj.getCounters()
    assert (cs.get(JIP, "NUM_FAILED_MAPS") or 0) + (cs.get(JIP, "NUM_FAILED_REDUCES") or 0) > 0


def test_job_fails_after_max_attempts(tmp_path):
    inp, _ = _words(tmp_path, files=1)
    conf = JobConf()
    conf.set_float("hbmr.faultinject.probability", 1.0)
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        job = wordcount.make_job(str(inp), str(tmp_path / "out"))
        job.set_int("mapred.map.max.attempts", 2)
        with pytest.raises(RuntimeError, match="failed 2 times"):
            JobClient.runJob(job, cluster=cl, verbose=False)


def test_lost_tracker_reexecutes_its_maps(tmp_path):
    conf = JobConf()
    conf.set_int("mapred.tasktracker.expiry.interval", 600)
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        job = sleep_job_conf(maps=12, reduces=2, map_ms=60, reduce_ms=1, reduce_count=2)
        job.set_speculative_execution(False)
        rj = cl.submit_job(job)
        # let some maps finish on both trackers, then lose tracker_1
        deadline = time.time() + 20
        while rj._impl.jip.maps_done < 4 and time.time() < deadline:
            time.sleep(0.01)
        cl.trackers[1].stop()
        assert rj.waitForCompletion(60)
        assert rj.isSuccessful(), rj.getFailureInfo()
        assert "tracker_1" not in cl.jt.trackers
        events = [e["event"] for e in cl.jt.history.events]
        assert "TRACKER_LOST" in events
        # every successful map attempt of the finished job ran on the surviving tracker
        # or completed before the loss and was re-executed
        last = {str(t.tid): t.successful.tracker for t in rj._impl.jip.maps}
        assert set(last.values()) <= {"tracker_0", "tracker_1"}


class HangMapper(Mapper):
    def map(self, key, value, output, reporter):
        time.sleep(3.0)   # no progress reported


def test_task_timeout_fails_hung_attempts(tmp_path):
    inp, _ = _words(tmp_path, files=1)
    conf = JobConf()
    conf.set_int("hbmr.heartbeat.interval.ms", 50)
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        job = JobConf()
        FileInputFormat.setInputPaths(job, str(inp))
        FileOutputFormat.setOutputPath(job, str(tmp_path / "out"))
        job.set_mapper_class(HangMapper)
        job.set_num_reduce_tasks(0)
        job.set_output_key_class(Text)
        job.set_output_value_class(Text)
        job.set_int("mapred.task.timeout", 400)
        job.set_int("mapred.map.max.attempts", 1)
        t0 = time.time()
        rj = cl.submit_job(job)
        rj.waitForCompletion(30)
        assert not rj.isSuccessful()
        assert "failed to report status" in rj.getFailureInfo()
        assert time.time() - t0 < 2.9   # failed by the timeout, not by finishing


def test_faulty_tracker_is_blacklisted(tmp_path):
    inp, cnt = _words(tmp_path, files=6)
    conf = JobConf()
    conf.set_int("mapred.max.tracker.failures", 1)
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        cl.trackers[1].fault_p = 1.0        # every attempt on tracker_1 fails
        job = wordcount.make_job(str(inp), str(tmp_path / "out"), reduces=1)
        job.set_num_map_tasks(24)
        job.set_int("mapred.map.max.attempts", 10)
        job.set_int("mapred.reduce.max.attempts", 10)
        JobClient.runJob(job, cluster=cl, verbose=False)
        assert cl.jt.trackers["tracker_1"].blacklisted
    assert _read(tmp_path / "out") == dict(cnt)


def test_speculative_gpu_backup_of_cpu_straggler():
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 1)
    conf.set_float("hbmr.gpu.simulate.task.ms", 5)
    conf.set_int("hbmr.gpu.queue.depth", 1)
    conf.set_float("hbmr.costmodel.probe.fraction", 0)   # whole-task CPU probe
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=1) as cl:
        job = split_sleep_conf(6, map_ms=1500, base=conf)     # CPU map tasks sleep 1.5 s
        job.set_boolean("mapred.map.tasks.speculative.execution", True)
        t0 = time.time()
        rj = cl.submit_job(job)
        assert rj.waitForCompletion(30) and rj.isSuccessful()
        took = time.time() - t0
        jip = rj._impl.jip
        spec = [a for t in jip.maps for a in t.attempts.values() if a.speculative]
        cpu = [a for t in jip.maps for a in t.attempts.values() if not a.run_on_gpu]
        # the overtaken CPU attempt was the signature's profiling probe: it runs
        # on detached and its real duration lands in the cost model
        deadline = time.time() + 5
        while cl.jt.cost_model.stats(jip.signature, False).n == 0 and time.time() < deadline:
            time.sleep(0.05)
        t_cpu = cl.jt.cost_model.stats(jip.signature, False).mean
    # the CPU straggler got a GPU backup that won; the job did not wait 1.5 s
    assert spec and any(a.run_on_gpu for a in spec)
    assert took < 1.4
    assert len(cpu) == 1 and cpu[0].profile_only
    assert t_cpu >= 1.4


def test_stock_policy_waits_for_cpu_stragglers():
    """GPU-unaware stock scheduling: CPU slots take tasks like any slot, and
    backups only come after Hadoop's 60 s speculative lag."""
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 1)
    conf.set_float("hbmr.gpu.simulate.task.ms", 5)
    conf.set("hbmr.scheduler.policy", "stock")
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=1) as cl:
        job = split_sleep_conf(6, map_ms=600, base=conf)
        t0 = time.time()
        rj = cl.submit_job(job)
        assert rj.waitForCompletion(30) and rj.isSuccessful()
        took = time.time() - t0
        cs = rj.getCounters()
    assert cs.get(JIP, "CPU_MAP_TASKS") >= 1
    assert took >= 0.55


def test_sampled_cpu_probe_profiles_without_straggling():
    """Hybrid scheduling of a split job: the CPU is profiled by a probe that runs
    the map on 1/8 of a split (output dropped) while the GPU slots run every
    real task; the scaled probe time lands in the cost model."""
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 1)
    conf.set_float("hbmr.gpu.simulate.task.ms", 5)
    conf.set_float("hbmr.costmodel.probe.fraction", 0.125)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=2) as cl:
        job = split_sleep_conf(8, map_ms=800, base=conf)
        t0 = time.time()
        rj = cl.submit_job(job)
        assert rj.waitForCompletion(30) and rj.isSuccessful()
        took = time.time() - t0
        cs = rj.getCounters()
        sig = rj._impl.jip.signature
        deadline = time.time() + 5
        while cl.jt.cost_model.stats(sig, False).n == 0 and time.time() < deadline:
            time.sleep(0.02)
        st = cl.jt.cost_model.stats(sig, False)
        # a second job of the same signature starts profiled: no probe, no CPU maps
        rj2 = cl.submit_job(split_sleep_conf(8, map_ms=800, base=conf))
        assert rj2.waitForCompletion(30) and rj2.isSuccessful()
        cs2 = rj2.getCounters()
    assert cs.get(JIP, "PROFILE_TASKS") == 1
    assert (cs.get(JIP, "CPU_MAP_TASKS") or 0) == 0
    assert took < 0.5                      # nobody waited for the 800 ms CPU map
    assert st.n == 1 and 0.7 < st.mean < 1.8   # 100 ms sample scaled by 8 (a loaded host runs it long)
    assert not cs2.get(JIP, "PROFILE_TASKS") and not cs2.get(JIP, "CPU_MAP_TASKS")


def test_debug_script_runs_on_failed_attempts(tmp_path):
    """mapred.map.task.debug.script (TestMiniMRMapRedDebugScript.java): the script
    gets stdout/stderr/syslog/jobconf paths, its output lands in the diagnostics."""
    inp, _ = _words(tmp_path, files=1)
    script = tmp_path / "debug.sh"
    script.write_text("#!/bin/sh\necho \"DEBUG-SCRIPT args=$#\"\nhead -c 200 \"$2\"\n"
                      "grep -c mapred.job.name \"$4\"\n")
    script.chmod(0o755)
    conf = JobConf()
    conf.set_float("hbmr.faultinject.probability", 1.0)
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        job = wordcount.make_job(str(inp), str(tmp_path / "out"))
        job.set_int("mapred.map.max.attempts", 1)
        job.set("mapred.map.task.debug.script", str(script))
        with pytest.raises(RuntimeError):
            JobClient.runJob(job, cluster=cl, verbose=False)
        logs = os.path.join(cl.local_dir, "tt0", "userlogs")
        outs = [open(os.path.join(logs, a, "debugout")).read() for a in os.listdir(logs)
                if os.path.exists(os.path.join(logs, a, "debugout"))]
    assert outs and "DEBUG-SCRIPT args=4" in outs[0]
    assert outs[0].rstrip().endswith("1")
