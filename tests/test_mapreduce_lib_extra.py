"""New-API library pieces (mapreduce/lib/{output,partition,fieldsel}):
LazyOutputFormat, FilterOutputFormat, MultipleOutputs, BinaryPartitioner,
KeyFieldBasedPartitioner and FieldSelectionMapper/Reducer, run as local jobs
as the reference's TestMRMultipleOutputs / TestBinaryPartitioner /
TestMRFieldSelection do."""
import os

from hbmr.io.writable import BytesWritable, IntWritable, Text, hash_bytes
from hbmr.mapred.jobconf import JobConf
from hbmr.mapreduce import Job, Mapper, Reducer
from hbmr.mapreduce.lib import fieldsel
from hbmr.mapreduce.lib.input import FileInputFormat, KeyValueTextInputFormat
from hbmr.mapreduce.lib.output import (FileOutputFormat, LazyOutputFormat, MultipleOutputs,
                                       TextOutputFormat)
from hbmr.mapreduce.lib.partition import BinaryPartitioner, KeyFieldBasedPartitioner


def _job(tmp_path, name):
    conf = JobConf()
    conf.set("mapred.job.tracker", "local")
    return Job(conf, name)


def _lines(d, prefix):
    out = []
    for fn in sorted(os.listdir(d)):
        if fn.startswith(prefix):
            out += open(os.path.join(d, fn)).read().splitlines()
    return out


class EvenOnly(Mapper):
    """Emits only from the split that holds even numbers."""

    def map(self, key, value, context):
        n = int(str(value))
        if n % 2 == 0:
            context.write(Text(str(n)), IntWritable(n))


def test_lazy_output_format_skips_empty_parts(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    (inp / "a.txt").write_text("1\n3\n5\n")
    (inp / "b.txt").write_text("2\n4\n")
    job = _job(tmp_path, "lazy")
    job.setMapperClass(EvenOnly)
    job.setNumReduceTasks(0)
    job.setOutputKeyClass(Text)
    job.setOutputValueClass(IntWritable)
    LazyOutputFormat.setOutputFormatClass(job, TextOutputFormat)
    FileInputFormat.addInputPath(job, inp)
    FileOutputFormat.setOutputPath(job, tmp_path / "out")
    assert job.waitForCompletion(False)
    parts = [f for f in os.listdir(tmp_path / "out") if f.startswith("part-")]
    assert len(parts) == 1                       # the odd split wrote no file
    assert sorted(_lines(tmp_path / "out", "part-")) == ["2\t2", "4\t4"]


class Splitter(Mapper):
    def setup(self, context):
        self.mos = MultipleOutputs(context)

    def map(self, key, value, context):
        n = int(str(value))
        if n < 0:
            self.mos.write("neg", Text(str(n)), IntWritable(-n))
        else:
            self.mos.write("pos", Text(str(n)), IntWritable(n), "big/pos" if n > 9 else None)
        context.write(Text("all"), IntWritable(n))

    def cleanup(self, context):
        self.mos.close()


class Sum(Reducer):
    def reduce(self, key, values, context):
        context.write(key, IntWritable(sum(v.get() for v in values)))


def test_new_api_multiple_outputs(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    (inp / "a.txt").write_text("1\n-2\n30\n4\n-5\n")
    job = _job(tmp_path, "mos")
    job.setMapperClass(Splitter)
    job.setReducerClass(Sum)
    job.setOutputKeyClass(Text)
    job.setOutputValueClass(IntWritable)
    MultipleOutputs.addNamedOutput(job, "pos", TextOutputFormat, Text, IntWritable)
    MultipleOutputs.addNamedOutput(job, "neg", TextOutputFormat, Text, IntWritable)
    FileInputFormat.addInputPath(job, inp)
    FileOutputFormat.setOutputPath(job, tmp_path / "out")
    assert job.waitForCompletion(False)
    out = tmp_path / "out"
    assert _lines(out, "part-r-") == ["all\t28"]
    assert sorted(_lines(out, "pos-m-")) == ["1\t1", "4\t4"]
    assert sorted(_lines(out, "neg-m-")) == ["-2\t2", "-5\t5"]
    assert _lines(out / "big", "pos-m-") == ["30\t30"]


def test_binary_partitioner_ranges():
    conf = JobConf()
    p = BinaryPartitioner()
    BinaryPartitioner.setOffsets(conf, 1, -2)
    p.setConf(conf)
    a = BytesWritable(b"\x01abc\x07")
    b = BytesWritable(b"\x09abc\x08")
    assert p.getPartition(a, None, 13) == p.getPartition(b, None, 13)
    assert p.getPartition(a, None, 13) == (hash_bytes(b"abc") & 0x7FFFFFFF) % 13
    BinaryPartitioner.setOffsets(conf, 0, -1)
    p.setConf(conf)
    parts = {p.getPartition(BytesWritable(bytes([i, i * 7 % 256])), None, 8) for i in range(64)}
    assert len(parts) > 1


def test_new_api_key_field_partitioner():
    conf = JobConf()
    conf.set("mapred.text.key.partitioner.options", "-k2,2")
    p = KeyFieldBasedPartitioner()
    p.setConf(conf)
    assert p.getPartition(Text("x\tsame\t1"), None, 7) == p.getPartition(Text("y\tsame\t2"), None, 7)


def test_new_api_field_selection(tmp_path):
    """FieldSelectionMapper/Reducer over a 6-field input, with the key:value
    spec of the reference's TestMRFieldSelection."""
    inp = tmp_path / "in"
    inp.mkdir()
    rows = ["-".join(f"f{c}{r}" for c in range(6)) for r in range(20)]
    (inp / "a.txt").write_text("\n".join(rows) + "\n")
    job = _job(tmp_path, "fieldsel")
    conf = job.getConfiguration()
    conf.set(fieldsel.DATA_FIELD_SEPARATOR, "-")
    conf.set(fieldsel.MAP_OUTPUT_KEY_VALUE_SPEC, "6,5,1-3:0-")
    conf.set(fieldsel.REDUCE_OUTPUT_KEY_VALUE_SPEC, ":4,3,2,1,0,0-")
    job.setMapperClass(fieldsel.FieldSelectionMapper)
    job.setReducerClass(fieldsel.FieldSelectionReducer)
    job.setOutputKeyClass(Text)
    job.setOutputValueClass(Text)
    job.setNumReduceTasks(1)
    FileInputFormat.addInputPath(job, inp)
    FileOutputFormat.setOutputPath(job, tmp_path / "out")
    assert job.waitForCompletion(False)
    got = sorted(_lines(tmp_path / "out", "part-r-"))
    want = []
    for r in rows:
        f = r.split("-")
        key = "-".join(["", f[5], f[1], f[2], f[3]])
        kf = key.split("-") + f                    # reducer record: key + sep + value
        want.append("\t" + "-".join([kf[4], kf[3], kf[2], kf[1], kf[0]] + kf))
    assert got == sorted(want)
    _ = KeyValueTextInputFormat


class Boom(Mapper):
    def map(self, key, value, context):
        raise RuntimeError("boom")


def test_new_api_job_control_runs_a_dag(tmp_path):
    """mapreduce.lib.jobcontrol: b depends on a (reads a's output); c depends
    on a job that fails and becomes DEPENDENT_FAILED."""
    import threading
    from hbmr.mapreduce.lib.jobcontrol import ControlledJob, JobControl, State
    from hbmr.mapreduce.lib.input import KeyValueTextInputFormat

    inp = tmp_path / "in"
    inp.mkdir()
    (inp / "a.txt").write_text("3\n1\n2\n")

    def mk(name, mapper, src, dst):
        j = _job(tmp_path, name)
        j.setMapperClass(mapper)
        j.setNumReduceTasks(0)
        j.setOutputKeyClass(Text)
        j.setOutputValueClass(IntWritable)
        FileInputFormat.addInputPath(j, src)
        FileOutputFormat.setOutputPath(j, dst)
        return j
    a = ControlledJob(mk("a", EvenOnly, inp, tmp_path / "oa"))
    b = ControlledJob(mk("b", Mapper, tmp_path / "oa", tmp_path / "ob"), [a])
    bad = ControlledJob(mk("bad", Boom, inp, tmp_path / "obad"))
    bad.getJob().getConfiguration().set_int("mapred.map.max.attempts", 1)
    c = ControlledJob(mk("c", Mapper, inp, tmp_path / "oc"), [bad])
    jc = JobControl("g")
    jc.addJobCollection([a, b, bad, c])
    assert [j.getJobID() for j in (a, b, bad, c)] == ["g1", "g2", "g3", "g4"]
    t = threading.Thread(target=jc.run)
    t.start()
    t.join(60)
    assert jc.allFinished()
    assert a.getJobState() == b.getJobState() == State.SUCCESS
    assert bad.getJobState() == State.FAILED and c.getJobState() == State.DEPENDENT_FAILED
    assert set(jc.getSuccessfulJobList()) == {a, b} and set(jc.getFailedJobList()) == {bad, c}
    assert sorted(_lines(tmp_path / "ob", "part-")) == ["0\t2\t2"]
    _ = KeyValueTextInputFormat
