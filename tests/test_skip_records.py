"""Bad-record skipping (the reference's TestBadRecords): after the configured
number of failed attempts, records / key groups whose processing throws are
skipped, counted and logged under the skip output dir."""
import collections
import os

import pytest

from hbmr.io import sequencefile as SF
from hbmr.io.writable import IntWritable, Text
from hbmr.mapred import JobClient, JobConf, Mapper, Reducer
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.skipbadrecords import SkipBadRecords
from hbmr.models import wordcount

TG = "org.apache.hadoop.mapred.Task$Counter"


class PickyMapper(Mapper):
    def map(self, key, value, output, reporter):
        if "BAD" in str(value):
            raise ValueError("bad record")
        for w in str(value).split():
            output.collect(Text(w), IntWritable(1))


class PickyReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        s = 0
        for v in values:
            s += v.get()
        if str(key) == "poison":
            raise ValueError("bad group")
        output.collect(key, IntWritable(s))


def _input(tmp_path):
    d = tmp_path / "in"
    d.mkdir()
    cnt = collections.Counter()
    lines = []
    for i in range(60):
        if i % 20 == 7:
            lines.append(f"BAD line {i}")
        else:
            ws = [f"w{(i + j) % 5}" for j in range(3)] + (["poison"] if i % 30 == 0 else [])
            lines.append(" ".join(ws))
            cnt.update(w for w in ws if w != "poison")
    (d / "f").write_text("\n".join(lines) + "\n")
    return d, cnt


def test_skips_bad_map_records_and_reduce_groups(tmp_path):
    d, cnt = _input(tmp_path)
    out = tmp_path / "out"
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        job = wordcount.make_job(str(d), str(out), reduces=1)
        job.set_mapper_class(PickyMapper)
        job.set_combiner_class(None)
        job.set_reducer_class(PickyReducer)
        job.set_int("mapred.map.max.attempts", 4)
        job.set_int("mapred.reduce.max.attempts", 4)
        SkipBadRecords.setAttemptsToStartSkipping(job, 1)
        SkipBadRecords.setMapperMaxSkipRecords(job, 10)
        SkipBadRecords.setReducerMaxSkipGroups(job, 1)
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
    assert rj.isSuccessful(), rj.getFailureInfo()
    cs = rj.getCounters()
    assert cs.get(TG, "MAP_SKIPPED_RECORDS") == 3
    assert cs.get(TG, "REDUCE_SKIPPED_GROUPS") == 1
    assert cs.get(TG, "REDUCE_SKIPPED_RECORDS") == 2
    got = {}
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            for line in open(out / fn):
                k, v = line.rstrip("\n").split("\t")
                got[k] = int(v)
    assert got == dict(cnt)
    skipdir = out / "_logs" / "skip"
    files = os.listdir(skipdir)
    assert files
    skipped = []
    for fn in files:
        with SF.Reader(skipdir / fn) as r:
            skipped += [str(v) for _, v in r]
    assert sum("BAD" in s for s in skipped) == 3


def test_task_profiling_selected_attempts(tmp_path):
    from hbmr.mapred.profiling import parse_ranges
    sel = parse_ranges("0-1,4,7-")
    assert [n for n in range(10) if sel(n)] == [0, 1, 4, 7, 8, 9]
    d = tmp_path / "in"
    d.mkdir()
    for i in range(4):
        (d / f"f{i}").write_text("a b c\n")
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        job = wordcount.make_job(str(d), str(tmp_path / "out"), reduces=1)
        job.set_boolean("mapred.task.profile", True)
        job.set("mapred.task.profile.maps", "1-2")
        JobClient.runJob(job, cluster=cl, verbose=False)
    profs = sorted(os.listdir(tmp_path / "out" / "_logs" / "profile"))
    assert len(profs) == 3                                # maps 1, 2 and reduce 0
    assert sum("_m_" in p for p in profs) == 2
    assert "function calls" in (tmp_path / "out" / "_logs" / "profile" / profs[0]).read_text()


def test_too_many_bad_records_fail_the_job(tmp_path):
    d, _ = _input(tmp_path)
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=1) as cl:
        job = wordcount.make_job(str(d), str(tmp_path / "out"), reduces=1)
        job.set_mapper_class(PickyMapper)
        job.set_int("mapred.map.max.attempts", 3)
        SkipBadRecords.setAttemptsToStartSkipping(job, 1)
        SkipBadRecords.setMapperMaxSkipRecords(job, 1)
        with pytest.raises(RuntimeError, match="Job failed"):
            JobClient.runJob(job, cluster=cl, verbose=False)
