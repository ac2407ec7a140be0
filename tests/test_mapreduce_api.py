"""The new (mapreduce) API: Job + context objects, on the local runner and the
in-process cluster (the reference's new-API WordCount,
src/examples/org/apache/hadoop/examples/WordCount.java)."""
import collections
import enum
import os

import pytest

from hbmr.io.writable import IntWritable, Text
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.mapreduce import Job, Mapper, Reducer
from hbmr.mapreduce.lib.input import FileInputFormat, NLineInputFormat, TextInputFormat
from hbmr.mapreduce.lib.map import MultithreadedMapper, TokenCounterMapper
from hbmr.mapreduce.lib.output import FileOutputFormat, SequenceFileOutputFormat
from hbmr.mapreduce.lib.reduce import IntSumReducer


class Stats(enum.Enum):
    LINES = 1


class TokenizerMapper(Mapper):
    def setup(self, context):
        self.one = IntWritable(1)
        self.lines = context.getCounter(Stats.LINES)

    def map(self, key, value, context):
        self.lines.increment()
        for w in str(value).split():
            context.write(Text(w), self.one)


class SumReducer(Reducer):
    def setup(self, context):
        self.calls = 0

    def reduce(self, key, values, context):
        self.calls += 1
        context.write(key, IntWritable(sum(v.get() for v in values)))

    def cleanup(self, context):
        context.getCounter("WC", "REDUCE_CALLS").increment(self.calls)


def _input(tmp_path, files=3):
    d = tmp_path / "in"
    d.mkdir()
    cnt = collections.Counter()
    for i in range(files):
        lines = [" ".join(f"t{(i + j * 5 + t) % 11}" for t in range(j % 7)) for j in range(200)]
        (d / f"f{i}.txt").write_text("\n".join(lines) + "\n")
        for ln in lines:
            cnt.update(ln.split())
    return d, cnt


def _read(out):
    res = {}
    for fn in os.listdir(out):
        if fn.startswith("part-r-"):
            for line in open(os.path.join(out, fn)):
                k, v = line.rstrip("\n").split("\t")
                res[k] = int(v)
    return res


@pytest.mark.parametrize("where", ["local", "cluster"])
def test_new_api_wordcount(tmp_path, where):
    inp, cnt = _input(tmp_path)
    conf = JobConf()
    cluster = None
    if where == "cluster":
        cluster = LocalCluster(JobConf(), num_trackers=2, cpu_slots=2)
    else:
        conf.set("mapred.job.tracker", "local")
    try:
        job = Job(conf, "word count", cluster=cluster)
        job.setMapperClass(TokenizerMapper)
        job.setCombinerClass(IntSumReducer)
        job.setReducerClass(SumReducer)
        job.setOutputKeyClass(Text)
        job.setOutputValueClass(IntWritable)
        job.setNumReduceTasks(2)
        FileInputFormat.addInputPath(job, inp)
        FileOutputFormat.setOutputPath(job, tmp_path / "out")
        assert job.waitForCompletion(False)
        assert job.isSuccessful()
        assert _read(tmp_path / "out") == dict(cnt)
        cs = job.getCounters()
        assert cs.get("Stats", "LINES") == 600
        assert cs.get("WC", "REDUCE_CALLS") == len(cnt)
    finally:
        if cluster is not None:
            cluster.shutdown()


def test_new_api_map_only_nline_and_multithreaded(tmp_path):
    inp, cnt = _input(tmp_path, files=1)
    conf = JobConf()
    conf.set("mapred.job.tracker", "local")
    job = Job(conf, "tokens")
    job.setInputFormatClass(NLineInputFormat)
    NLineInputFormat.setNumLinesPerSplit(job, 50)
    job.setMapperClass(MultithreadedMapper)
    MultithreadedMapper.setMapperClass(job, TokenCounterMapper)
    MultithreadedMapper.setNumberOfThreads(job, 4)
    job.setNumReduceTasks(0)
    job.setOutputKeyClass(Text)
    job.setOutputValueClass(IntWritable)
    job.setOutputFormatClass(SequenceFileOutputFormat)
    FileInputFormat.setInputPaths(job, inp)
    FileOutputFormat.setOutputPath(job, tmp_path / "out")
    assert job.waitForCompletion()
    parts = sorted(f for f in os.listdir(tmp_path / "out") if f.startswith("part-m-"))
    assert len(parts) == 4
    from hbmr.io import sequencefile as seqf
    total = collections.Counter()
    for p in parts:
        with seqf.Reader(tmp_path / "out" / p) as r:
            for k, v in r:
                total[str(k)] += v.get()
    assert total == cnt
    _ = TextInputFormat
