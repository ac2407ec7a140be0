"""io.serializations: non-Writable map-output types through the whole
map → sort/spill → combine → shuffle → reduce path (the reference's
io/serializer tests + TestJavaSerialization.java)."""
from __future__ import annotations

import os

import pytest

from hbmr.io import serializer as S
from hbmr.io.writable import IntWritable, Text
from hbmr.mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from hbmr.mapred.api import Mapper, Reducer
from hbmr.mapred.cluster import LocalCluster


class LenMapper(Mapper):
    """(word length: int, (word, 1): tuple) — plain Python types."""

    def map(self, key, value, output, reporter):
        for w in str(value).split():
            output.collect(len(w), (w, 1))


class CountReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        words, n = set(), 0
        for w, c in values:
            words.add(w)
            n += c
        output.collect(key, (",".join(sorted(words)), n))


class CountCombiner(Reducer):
    def reduce(self, key, values, output, reporter):
        acc = {}
        for w, c in values:
            acc[w] = acc.get(w, 0) + c
        for w, c in acc.items():
            output.collect(key, (w, c))


def test_factory_picks_serialization():
    f = S.SerializationFactory(JobConf())
    assert isinstance(f.get_serialization(Text), S.WritableSerialization)
    assert isinstance(f.get_serialization(int), S.MsgpackSerialization)
    with pytest.raises(TypeError):
        f.get_serialization(object)
    ad = S.adapter_for(tuple)
    raw = S.to_bytes(("a", 3), ad)
    assert ad.deserialize(raw) == ("a", 3)
    assert isinstance(("x",), ad) and not isinstance([1], ad)
    assert S.adapter_for(IntWritable) is IntWritable
    keys = [5, -2, 100, 0]
    ki = S.adapter_for(int)
    assert sorted(keys) == sorted(keys, key=lambda k: ki.raw_sort_key(S.to_bytes(k, ki)))
    js = S.JsonSerialization()
    assert js.deserialize(js.serialize({"a": [1, 2]}), dict) == {"a": [1, 2]}


@pytest.mark.parametrize("mode", ["local", "cluster-process"])
def test_plain_python_types_through_a_job(tmp_path, mode):
    inp = tmp_path / "in"
    inp.mkdir()
    words = "a bb cc ddd a bb eeee ffff gggg a".split()
    (inp / "f").write_text(" ".join(words) + "\n" + " ".join(words[::-1]) + "\n")
    job = JobConf()
    FileInputFormat.setInputPaths(job, str(inp))
    FileOutputFormat.setOutputPath(job, str(tmp_path / "out"))
    job.set_mapper_class(LenMapper)
    job.set_combiner_class(CountCombiner)
    job.set_reducer_class(CountReducer)
    job.set_map_output_key_class(int)
    job.set_map_output_value_class(tuple)
    job.set_output_key_class(int)
    job.set_output_value_class(tuple)
    job.set_num_reduce_tasks(2)
    job.set_int("io.sort.mb", 1)
    if mode == "local":
        JobClient.runJob(job, verbose=False)
    else:
        job.set("mapred.task.isolation", "process")
        with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
            JobClient.runJob(job, cluster=cl, verbose=False)
    got = {}
    for p in sorted(os.listdir(tmp_path / "out")):
        if p.startswith("part-"):
            for ln in open(tmp_path / "out" / p):
                k, v = ln.rstrip("\n").split("\t")
                got[int(k)] = v
    exp = {}
    for w in words * 2:
        exp.setdefault(len(w), {}).setdefault(w, 0)
        exp[len(w)][w] += 1
    assert got == {k: str((",".join(sorted(v)), sum(v.values()))) for k, v in exp.items()}
