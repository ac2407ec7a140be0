"""Join two (or more) keyed text datasets (the role of src/examples/org/apache/
hadoop/examples/Join.java and contrib/data_join): a reduce-side join.

Each input line is ``key<TAB>value``; MultipleInputs tags every record with its
source index, the reducer groups by key and emits the cross product of the
sources' values (inner join) or pads missing sides (outer)."""
from __future__ import annotations

import argparse
import itertools

from ..io.writable import Text
from ..mapred import FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from ..mapred.formats import KeyValueTextInputFormat
from ..mapred.lib.multiple import MultipleInputs


def _tagging_mapper(tag):
    class _Tag(Mapper):
        def map(self, key, value, output, reporter):
            output.collect(key, Text(f"{tag}\x01{value}"))
    _Tag.__name__ = _Tag.__qualname__ = f"TagMapper{tag}"
    globals()[_Tag.__name__] = _Tag
    return _Tag


class JoinReducer(Reducer):
    def configure(self, job):
        self.n = job.get_int("join.sources", 2)
        self.outer = job.get("join.type", "inner") == "outer"

    def reduce(self, key, values, output, reporter):
        sides = [[] for _ in range(self.n)]
        for v in values:
            tag, _, val = str(v).partition("\x01")
            sides[int(tag)].append(val)
        if self.outer:
            sides = [s or [""] for s in sides]
        for combo in itertools.product(*sides):
            output.collect(key, Text("\t".join(combo)))


def make_job(inputs, out, join_type="inner", reduces=1, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name(f"join ({join_type})")
    for i, p in enumerate(inputs):
        MultipleInputs.addInputPath(job, p, KeyValueTextInputFormat, _tagging_mapper(i))
    job.set_int("join.sources", len(inputs))
    job.set("join.type", join_type)
    job.set_reducer_class(JoinReducer)
    job.set_output_key_class(Text)
    job.set_output_value_class(Text)
    job.set_num_reduce_tasks(reduces)
    FileOutputFormat.setOutputPath(job, out)
    return job


for _i in range(8):   # importable tag mappers for up to 8 sources
    _tagging_mapper(_i)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr join")
    ap.add_argument("-joinOp", default="inner", choices=["inner", "outer"])
    ap.add_argument("-r", type=int, default=1)
    ap.add_argument("paths", nargs="+", help="input1 input2 [...] output")
    a = ap.parse_args(argv)
    rj = JobClient.runJob(make_job(a.paths[:-1], a.paths[-1], a.joinOp, a.r), cluster=cluster)
    return 0 if rj.isSuccessful() else 1
