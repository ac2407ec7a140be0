"""End-to-end jobs on the LocalJobRunner (BASELINE config 1: WordCount)."""
import collections
import os

import pytest

from hbmr.io import sequencefile as seqf
from hbmr.io.writable import IntWritable, LongWritable, Text
from hbmr.mapred import (FileInputFormat, FileOutputFormat, JobClient, JobConf, NLineInputFormat,
                         SequenceFileInputFormat, SequenceFileOutputFormat)
from hbmr.mapred import counters as C
from hbmr.mapred.lib import IdentityMapper, IdentityReducer, InverseMapper
from hbmr.models import wordcount

WORDS = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta", "theta"]


def _write_text(path, nlines, seed=0):
    import random
    rng = random.Random(seed)
    cnt = collections.Counter()
    with open(path, "w") as f:
        for _ in range(nlines):
            ws = [rng.choice(WORDS) for _ in range(rng.randint(0, 12))]
            cnt.update(ws)
            f.write(" ".join(ws) + "\n")
    return cnt


def _read_output(outdir):
    res = {}
    for fn in sorted(os.listdir(outdir)):
        if fn.startswith("part-"):
            for line in open(os.path.join(outdir, fn)):
                k, v = line.rstrip("\n").split("\t")
                assert k not in res
                res[k] = int(v)
    return res


@pytest.mark.parametrize("reduces,sort_mb", [(1, 100), (3, 100), (2, 0)])
def test_wordcount(tmp_path, reduces, sort_mb):
    inp = tmp_path / "in"
    inp.mkdir()
    expect = collections.Counter()
    for i in range(3):
        expect += _write_text(inp / f"part{i}.txt", 400, seed=i)
    (inp / "_hidden").write_text("alpha alpha alpha\n")  # must be ignored
    out = tmp_path / "out"
    job = wordcount.make_job(str(inp), str(out), reduces=reduces)
    job.set_num_map_tasks(5)
    job.set_int("io.sort.mb", sort_mb)  # 0 => spill on every record, exercises merge
    rj = JobClient.runJob(job, verbose=False)
    assert rj.isSuccessful()
    assert _read_output(out) == dict(expect)
    assert os.path.exists(out / "_SUCCESS")
    assert not os.path.exists(out / "_temporary")
    cs = rj.getCounters()
    assert cs.get(C.TASK_GROUP, C.REDUCE_OUTPUT_RECORDS) == len(expect)
    assert cs.get(C.TASK_GROUP, C.MAP_INPUT_RECORDS) == 1200
    assert cs.get(C.TASK_GROUP, C.COMBINE_INPUT_RECORDS) > 0
    assert len([f for f in os.listdir(out) if f.startswith("part-")]) == reduces
    # hash partitioning is Hadoop's: each word lands in (hash & MAX) % R
    if reduces > 1:
        for fn in os.listdir(out):
            if fn.startswith("part-"):
                r = int(fn[5:])
                for line in open(out / fn):
                    w = line.split("\t")[0]
                    assert (Text(w).hash_code() & 0x7FFFFFFF) % reduces == r


def test_output_exists_fails(tmp_path):
    inp = tmp_path / "in.txt"
    inp.write_text("a b\n")
    out = tmp_path / "out"
    out.mkdir()
    (out / "x").write_text("1")
    job = wordcount.make_job(str(inp), str(out))
    with pytest.raises(RuntimeError):
        JobClient.runJob(job, verbose=False)


def test_nline_input_one_line_per_map(tmp_path):
    inp = tmp_path / "lines.txt"
    inp.write_text("".join(f"line {i}\n" for i in range(7)))
    job = JobConf()
    job.set_input_format(NLineInputFormat)
    job.set_int("mapred.line.input.format.linespermap", 1)
    FileInputFormat.setInputPaths(job, str(inp))
    splits = NLineInputFormat().getSplits(job, 1)
    assert len(splits) == 7
    from hbmr.mapred.formats import LineRecordReader
    seen = []
    for sp in splits:
        rr = LineRecordReader(job, sp)
        recs = [str(v) for _, v in rr]
        assert len(recs) == 1
        seen += recs
    assert seen == [f"line {i}" for i in range(7)]


def test_text_splits_read_every_line_once(tmp_path):
    inp = tmp_path / "t.txt"
    lines = [("x" * (i % 50)) + str(i) for i in range(2000)]
    inp.write_text("\n".join(lines) + "\n")
    job = JobConf()
    FileInputFormat.setInputPaths(job, str(inp))
    job.set_long("mapred.min.split.size", 1)
    from hbmr.mapred.formats import TextInputFormat
    fmt = TextInputFormat()
    for n in (1, 2, 7, 31):
        got = []
        for sp in fmt.getSplits(job, n):
            rr = fmt.getRecordReader(sp, job, None)
            got += [str(v) for _, v in rr]
        assert got == lines


def test_sequencefile_job_and_inverse(tmp_path):
    src = tmp_path / "in.seq"
    with seqf.Writer(src, Text, LongWritable) as w:
        for i in range(100):
            w.append(Text(f"k{i % 10}"), LongWritable(i))
    out = tmp_path / "out"
    job = JobConf()
    job.set_input_format(SequenceFileInputFormat)
    job.set_output_format(SequenceFileOutputFormat)
    job.set_mapper_class(InverseMapper)
    job.set_reducer_class(IdentityReducer)
    job.set_map_output_key_class(LongWritable)
    job.set_map_output_value_class(Text)
    job.set_output_key_class(LongWritable)
    job.set_output_value_class(Text)
    job.set_num_reduce_tasks(2)
    FileInputFormat.setInputPaths(job, str(src))
    FileOutputFormat.setOutputPath(job, str(out))
    JobClient.runJob(job, verbose=False)
    recs = []
    for r in SequenceFileOutputFormat.get_readers(str(out)):
        part = [(k.get(), str(v)) for k, v in r]
        assert [k for k, _ in part] == sorted(k for k, _ in part)  # sorted within a reducer
        recs += part
    assert sorted(recs) == sorted((i, f"k{i % 10}") for i in range(100))


def test_map_only_job(tmp_path):
    inp = tmp_path / "in.txt"
    inp.write_text("a\nb\nc\n")
    out = tmp_path / "out"
    job = JobConf()
    job.set_mapper_class(IdentityMapper)
    job.set_num_reduce_tasks(0)
    FileInputFormat.setInputPaths(job, str(inp))
    FileOutputFormat.setOutputPath(job, str(out))
    JobClient.runJob(job, verbose=False)
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    text = [line for p in parts for line in open(out / p).read().splitlines()]
    assert [line.split("\t")[1] for line in text] == ["a", "b", "c"]


def test_type_mismatch_fails(tmp_path):
    inp = tmp_path / "in.txt"
    inp.write_text("a\n")
    job = JobConf()
    job.set_mapper_class(IdentityMapper)
    job.set_map_output_key_class(Text)   # identity emits LongWritable keys
    FileInputFormat.setInputPaths(job, str(inp))
    FileOutputFormat.setOutputPath(job, str(tmp_path / "o"))
    rj = JobClient(job).submitJob(job)
    rj.waitForCompletion()
    assert not rj.isSuccessful()
    assert "Type mismatch" in rj.getFailureInfo()
    _ = IntWritable


@pytest.mark.parametrize("split_mb", [0.0005, 0.003, 64])
def test_native_wordcount_runner_matches_python_mapper(tmp_path, split_mb):
    """NativeWordCountRunner (C++ tokenizer + table over whole-line blocks of
    the split) gives the per-record mapper's counts for any split boundaries
    (lines crossing splits, CRLF, tabs/form feeds, a last line without a newline)."""
    import collections
    from hbmr.models import wordcount as W
    d = tmp_path / "in"
    d.mkdir()
    rng = __import__("random").Random(5)
    words = [f"w{i}" for i in range(300)] + ["é", "naïve", "x" * 40]
    lines = []
    for i in range(3000):
        sep = rng.choice([" ", "  ", "\t", " \x0c "])
        lines.append(sep.join(rng.choice(words) for _ in range(rng.randrange(0, 9))))
    text = "\r\n".join(lines[:1500]) + "\n" + "\n".join(lines[1500:])    # no final newline
    (d / "a.txt").write_text(text)
    want = collections.Counter(text.encode().split())
    res = {}
    for native in (True, False):
        conf = JobConf()
        conf.set("mapred.job.tracker", "local")
        conf.set_boolean("hbmr.wordcount.native", native)
        conf.set_long("mapred.min.split.size", 1)
        conf.set_long("mapred.max.split.size", int(split_mb * (1 << 20)))
        out = tmp_path / f"out{native}"
        job = W.make_job(str(d), str(out), reduces=2, conf=conf)
        job.set_num_map_tasks(max(1, int(len(text) / max(1, split_mb * (1 << 20)))))
        rj = JobClient.runJob(job, verbose=False)
        got = {}
        for fn in os.listdir(out):
            if fn.startswith("part-"):
                for line in open(out / fn, "rb"):
                    k, v = line.rstrip(b"\n").rsplit(b"\t", 1)
                    got[k] = int(v)
        res[native] = got
        recs = rj.getCounters().get("org.apache.hadoop.mapred.Task$Counter", "MAP_INPUT_RECORDS")
        assert recs == 3000 - 0, (native, recs)
    assert res[True] == res[False] == dict(want)
