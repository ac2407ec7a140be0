"""mapred.lib extras: ChainMapper/ChainReducer, MultipleOutputs,
MultipleTextOutputFormat, CombineFileInputFormat, JobControl, ToolRunner."""
import collections
import os

from hbmr.io.writable import IntWritable, LongWritable, Text
from hbmr.mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from hbmr.mapred.formats import TextOutputFormat
from hbmr.mapred.jobcontrol import SUCCESS, ControlledJob, JobControl
from hbmr.mapred.lib.basic import LongSumReducer, TokenCountMapper
from hbmr.mapred.lib.chain import ChainMapper, ChainReducer
from hbmr.mapred.lib.combine import CombineFileInputFormat
from hbmr.mapred.lib.multiple import MultipleOutputs, MultipleTextOutputFormat
from hbmr.utils.tool import GenericOptionsParser, Tool, ToolRunner


class Upper(Mapper):
    def map(self, key, value, output, reporter):
        output.collect(key, Text(str(value).upper()))


class Split(Mapper):
    def map(self, key, value, output, reporter):
        for w in str(value).split():
            output.collect(Text(w), LongWritable(1))


class Tag(Mapper):
    def configure(self, job):
        self.suffix = job.get("tag.suffix", "")

    def map(self, key, value, output, reporter):
        output.collect(Text(str(key) + self.suffix), value)


def _inp(tmp_path):
    d = tmp_path / "in"
    d.mkdir()
    (d / "a.txt").write_text("x y z\ny y\n")
    (d / "b.txt").write_text("z z x\n")
    return d


def _kv(out):
    res = {}
    for fn in os.listdir(out):
        if not fn.startswith(("_", ".")):
            for line in open(os.path.join(out, fn)):
                k, v = line.rstrip("\n").split("\t")
                res[k] = v
    return res


def test_chain_mapper_and_reducer(tmp_path):
    job = JobConf()
    FileInputFormat.setInputPaths(job, str(_inp(tmp_path)))
    FileOutputFormat.setOutputPath(job, str(tmp_path / "out"))
    ChainMapper.addMapper(job, Upper, mapper_conf={})
    ChainMapper.addMapper(job, Split, out_key=Text, out_val=LongWritable)
    ChainReducer.setReducer(job, LongSumReducer, out_key=Text, out_val=LongWritable)
    ChainReducer.addMapper(job, Tag, mapper_conf={"tag.suffix": "!"})
    JobClient.runJob(job, verbose=False)
    assert _kv(tmp_path / "out") == {"X!": "2", "Y!": "3", "Z!": "3"}


class RoutedOutput(MultipleTextOutputFormat):
    def generateFileNameForKeyValue(self, key, value, name):  # noqa: N802
        return f"{str(key)[0]}-{name}"


class MosReducer(Reducer):
    def configure(self, job):
        self.mos = MultipleOutputs(job)

    def reduce(self, key, values, output, reporter):
        n = sum(v.get() for v in values)
        output.collect(key, LongWritable(n))
        if n > 2:
            self.mos.getCollector("big", reporter).collect(key, IntWritable(n))

    def close(self):
        self.mos.close()


def test_multiple_outputs_and_routed_files(tmp_path):
    job = JobConf()
    FileInputFormat.setInputPaths(job, str(_inp(tmp_path)))
    FileOutputFormat.setOutputPath(job, str(tmp_path / "out"))
    job.set_mapper_class(TokenCountMapper)
    job.set_reducer_class(MosReducer)
    job.set_output_format(RoutedOutput)
    job.set_output_key_class(Text)
    job.set_output_value_class(LongWritable)
    MultipleOutputs.addNamedOutput(job, "big", TextOutputFormat, Text, IntWritable)
    JobClient.runJob(job, verbose=False)
    files = sorted(f for f in os.listdir(tmp_path / "out") if not f.startswith(("_", ".")))
    assert files == ["big-r-00000", "x-part-00000", "y-part-00000", "z-part-00000"]
    assert _kv(tmp_path / "out") == {"x": "2", "y": "3", "z": "3"}
    big = open(tmp_path / "out" / "big-r-00000").read().split()
    assert big == ["y", "3", "z", "3"]


def test_combine_file_input_packs_small_files(tmp_path):
    d = tmp_path / "many"
    d.mkdir()
    cnt = collections.Counter()
    for i in range(12):
        text = f"w{i % 3} common\n" * 5
        (d / f"f{i}").write_text(text)
        cnt.update(text.split())
    job = JobConf()
    job.set_input_format(CombineFileInputFormat)
    job.set_long("mapred.max.split.size", 200)
    FileInputFormat.setInputPaths(job, str(d))
    splits = CombineFileInputFormat().getSplits(job, 1)
    assert 1 < len(splits) < 12 and sum(s.getLength() for s in splits) == sum(
        os.path.getsize(d / f) for f in os.listdir(d))
    FileOutputFormat.setOutputPath(job, str(tmp_path / "out"))
    job.set_mapper_class(TokenCountMapper)
    job.set_reducer_class(LongSumReducer)
    job.set_output_key_class(Text)
    job.set_output_value_class(LongWritable)
    rj = JobClient.runJob(job, verbose=False)
    assert {k: int(v) for k, v in _kv(tmp_path / "out").items()} == dict(cnt)
    assert rj.getCounters().get("org.apache.hadoop.mapred.JobInProgress$Counter",
                                "TOTAL_LAUNCHED_MAPS") in (None, len(splits))


def test_jobcontrol_runs_dependency_chain(tmp_path):
    inp = _inp(tmp_path)

    def wc(src, dst):
        job = JobConf()
        FileInputFormat.setInputPaths(job, str(src))
        FileOutputFormat.setOutputPath(job, str(dst))
        job.set_mapper_class(TokenCountMapper)
        job.set_reducer_class(LongSumReducer)
        job.set_output_key_class(Text)
        job.set_output_value_class(LongWritable)
        return job

    j1 = ControlledJob(wc(inp, tmp_path / "o1"))
    j2 = ControlledJob(wc(tmp_path / "o1", tmp_path / "o2"), depending=[j1])
    jc = JobControl("chain")
    jc.addJobs([j2, j1])
    jc.run()
    assert jc.allFinished() and j1.getState() == SUCCESS and j2.getState() == SUCCESS
    # second job counted the words of "word\tcount" lines
    assert int(_kv(tmp_path / "o2")["x"]) == 1


def test_tool_runner_generic_options(tmp_path):
    seen = {}

    class T(Tool):
        def run(self, args):
            seen["args"] = args
            seen["v"] = self.getConf().get("my.key")
            seen["jt"] = self.getConf().get("mapred.job.tracker")
            return 7

    assert ToolRunner.run(JobConf(), T(), ["-D", "my.key=5", "-jt", "local", "a", "-Dx=y",
                                           "b"]) == 7
    assert seen == {"args": ["a", "b"], "v": "5", "jt": "local"}
    p = GenericOptionsParser(JobConf(), ["-files", "f1,f2", "rest"])
    assert p.getRemainingArgs() == ["rest"]
    assert p.getConfiguration().get("mapred.cache.files").endswith("f2")
