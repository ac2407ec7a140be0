"""Cluster services: rack awareness (ScriptBasedMapping + rack-local level the
GPU fork dropped), LimitTasksPerJobTaskScheduler, node health
script + GPU health withdrawal (NodeHealthCheckerService)."""
import os
import stat
import threading
import time

from hbmr.examples.sleepjob import split_sleep_conf
from hbmr.mapred import JobClient, JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.formats import FileSplit, TextInputFormat
from hbmr.models import wordcount
from hbmr.net import DEFAULT_RACK, Topology

JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"


def _script(path, body):
    path.write_text("#!/bin/sh\n" + body)
    path.chmod(path.stat().st_mode | stat.S_IEXEC)
    return str(path)


def test_topology_table_script_and_default(tmp_path):
    conf = JobConf()
    conf.set("hbmr.topology.table", "a=/r1, b=r2")
    t = Topology(conf)
    assert t.resolve(["a", "b", "zz"]) == ["/r1", "/r2", DEFAULT_RACK]
    conf = JobConf()
    conf.set("topology.script.file.name",
             _script(tmp_path / "topo.sh", 'for h in "$@"; do echo "/rack-$h"; done\n'))
    conf.set_int("topology.script.number.args", 2)
    t = Topology(conf)
    assert t.resolve(["x", "y", "z"]) == ["/rack-x", "/rack-y", "/rack-z"]
    assert t.rack("y") == "/rack-y"


class HostedTextInputFormat(TextInputFormat):
    """Gives split i the host list of HOSTS[i % 3] (a fake HDFS block map)."""
    HOSTS = [["hostA"], ["hostB"], ["hostC"]]

    def getSplits(self, job, num_splits):  # noqa: N802
        out = []
        for i, s in enumerate(super().getSplits(job, num_splits)):
            out.append(FileSplit(s.getPath(), s.getStart(), s.getLength(),
                                 self.HOSTS[i % 3]))
        return out


def test_data_and_rack_local_counters(tmp_path):
    d = tmp_path / "in"
    d.mkdir()
    for i in range(6):
        (d / f"f{i}").write_text("a b c\n" * 10)
    conf = JobConf()
    conf.set("hbmr.topology.table", "hostA=/r1,hostB=/r1,hostC=/r2")
    with LocalCluster(conf, num_trackers=1, cpu_slots=1, hosts=["hostA"]) as cl:
        job = wordcount.make_job(str(d), str(tmp_path / "out"), reduces=1)
        job.set_input_format(HostedTextInputFormat)
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
    assert rj.isSuccessful()
    cs = rj.getCounters()
    assert cs.get(JIP, "DATA_LOCAL_MAPS") == 2
    assert cs.get(JIP, "RACK_LOCAL_MAPS") == 2
    assert cs.get(JIP, "TOTAL_LAUNCHED_MAPS") == 6


def test_limit_tasks_per_job_scheduler():
    conf = JobConf()
    conf.set("mapred.jobtracker.taskScheduler",
             "hbmr.mapred.scheduler.limit:LimitTasksPerJobTaskScheduler")
    conf.set_int("mapred.jobtracker.scheduler.maxRunningTasksPerJob", 2)
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_int("hbmr.gpu.queue.depth", 4)
    conf.set_float("hbmr.gpu.simulate.task.ms", 10)
    conf.set("hbmr.scheduler.policy", "stock")
    peak = [0]
    with LocalCluster(conf, num_trackers=1, gpus=[[0, 1]], cpu_slots=2,
                      gpu_slots_per_device=2) as cl:
        rj = cl.submit_job(split_sleep_conf(24, base=conf))
        stop = threading.Event()

        def sample():
            while not stop.is_set():
                peak[0] = max(peak[0], rj._impl.jip.running_maps())
                time.sleep(0.002)
        t = threading.Thread(target=sample, daemon=True)
        t.start()
        try:
            rj.waitForCompletion(60)
        finally:
            stop.set()
            t.join()
        assert rj.isSuccessful(), rj.getFailureInfo()
    assert 1 <= peak[0] <= 2


def test_health_script_blocks_then_releases_tracker(tmp_path):
    flag = tmp_path / "sick"
    flag.write_text("1")
    script = _script(tmp_path / "health.sh",
                     f'if [ -f "{flag}" ]; then echo "ERROR disk is gone"; else echo OK; fi\n')
    conf = JobConf()
    conf.set("mapred.healthChecker.script.path", script)
    conf.set_int("mapred.healthChecker.interval", 100)
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(split_sleep_conf(4, base=conf))
        time.sleep(0.5)
        tr = next(iter(cl.jt.trackers.values()))
        assert not tr.status.healthy
        assert "disk is gone" in tr.status.health_report
        jip = rj._impl.jip
        assert jip.running_maps() == 0 and not any(t.is_complete() for t in jip.maps)
        os.unlink(flag)
        rj.waitForCompletion(30)
        assert rj.isSuccessful(), rj.getFailureInfo()
        assert tr.status.healthy


def test_unhealthy_gpu_is_withdrawn():
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set("hbmr.gpu.simulate.bad.devices", "1")
    conf.set("hbmr.scheduler.policy", "stock")
    with LocalCluster(conf, num_trackers=1, gpus=[[0, 1]], cpu_slots=0) as cl:
        rj = cl.submit_job(split_sleep_conf(16, base=conf, cpu_capable=False))
        rj.waitForCompletion(60)
        assert rj.isSuccessful(), rj.getFailureInfo()
        devs = {r.getGPUDeviceId() for r in rj.getTaskReports(True)}
        tr = next(iter(cl.jt.trackers.values()))
        assert [g["device"] for g in tr.status.gpus] == [0]
        assert "gpu1" in tr.status.health_report and tr.status.healthy
    assert devs == {0}
