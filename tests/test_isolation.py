"""IsolationRunner (mapred/IsolationRunner.java, the reference's
TestIsolationRunner): a failing map's kept job.xml + split re-run alone in
this process reproduce the failure; a pattern-kept successful attempt re-runs
to the same map output."""
import glob
import os

import pytest

from hbmr.io.writable import IntWritable, Text
from hbmr.mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.isolation import IsolationRunner, main


class PickyMapper(Mapper):
    def configure(self, job):
        self.bad = job.get("test.bad.word")

    def map(self, key, value, output, reporter):
        for w in str(value).split():
            if w == self.bad:
                raise ValueError(f"poison word {w}")
            output.collect(Text(w), IntWritable(1))


def _job(tmp_path, bad=None):
    inp = tmp_path / "in"
    inp.mkdir(exist_ok=True)
    (inp / "a.txt").write_text("x y z\nx poison\n")
    job = JobConf()
    job.set_mapper_class(PickyMapper)
    job.set_output_key_class(Text)
    job.set_output_value_class(IntWritable)
    job.set_num_reduce_tasks(1)
    if bad:
        job.set("test.bad.word", bad)
    FileInputFormat.setInputPaths(job, str(inp))
    FileOutputFormat.setOutputPath(job, str(tmp_path / ("out-" + str(bad))))
    job.set_int("mapred.map.max.attempts", 1)
    return job


def _kept(local):
    return sorted(glob.glob(os.path.join(str(local), "**", "job.xml"), recursive=True))


def test_isolation_runner_reproduces_failed_map(tmp_path):
    conf = JobConf()
    conf.set("mapred.local.dir", str(tmp_path / "local"))
    with LocalCluster(conf, num_trackers=1, cpu_slots=1, local_dir=str(tmp_path / "local")) as cl:
        job = _job(tmp_path, bad="poison")
        job.set_boolean("keep.failed.task.files", True)
        with pytest.raises(RuntimeError):
            JobClient.runJob(job, cluster=cl, verbose=False)
    kept = _kept(tmp_path / "local")
    assert len(kept) == 1 and "_m_000000_0" in kept[0]
    assert os.path.exists(os.path.join(os.path.dirname(kept[0]), "split.dta"))
    with pytest.raises(ValueError, match="poison word"):
        IsolationRunner().run([kept[0]])


def test_isolation_runner_reruns_kept_attempt(tmp_path, capsys):
    conf = JobConf()
    conf.set("mapred.local.dir", str(tmp_path / "local"))
    with LocalCluster(conf, num_trackers=1, cpu_slots=1, local_dir=str(tmp_path / "local")) as cl:
        job = _job(tmp_path)
        job.set("keep.task.files.pattern", r".*_m_000000_.*")
        JobClient.runJob(job, cluster=cl, verbose=False)
    kept = _kept(tmp_path / "local")
    assert len(kept) == 1
    r = IsolationRunner()
    assert r.run([kept[0]])
    assert r.output and os.path.exists(r.output)
    assert "reporting done" in capsys.readouterr().out
    assert main([]) == 1 and main([str(tmp_path / "nope.xml")]) == 1
