"""Join over sorted, equally partitioned datasets (src/examples/org/apache/hadoop/
examples/Join.java).

``make_job`` is the reference's map-side join: CompositeInputFormat with
``mapred.join.expr = <op>(tbl(<inFormat>,"in1"),tbl(<inFormat>,"in2"),...)``
(Join.java:144-145), IdentityMapper / IdentityReducer, keys of the sources
joined inside the map task and emitted as (key, TupleWritable).  The inputs
must be sorted by key and partitioned identically (e.g. outputs of jobs with
the same partitioner and reduce count).

``make_reduce_side_job`` is the general join for inputs that are not (the
contrib/data_join approach): MultipleInputs tags every record with its source,
the reducer groups by key and emits the cross product of the sources' values
(inner) or pads missing sides (outer)."""
from __future__ import annotations

import argparse
import itertools

from ..io.writable import BytesWritable, Text
from ..mapred import FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from ..mapred.formats import KeyValueTextInputFormat, SequenceFileInputFormat, \
    SequenceFileOutputFormat
from ..mapred.join import CompositeInputFormat, TupleWritable
from ..mapred.lib.multiple import MultipleInputs
from ..utils.reflection import load_class


def make_job(inputs, out, join_type="inner", reduces=0, conf=None,
             in_format=SequenceFileInputFormat, out_format=SequenceFileOutputFormat,
             out_key=BytesWritable, out_value=TupleWritable) -> JobConf:
    """Map-side join job (Join.java:run)."""
    job = JobConf(conf)
    job.set_job_name("join")
    job.set_mapper_class("hbmr.mapred.lib.basic:IdentityMapper")
    job.set_reducer_class("hbmr.mapred.lib.basic:IdentityReducer")
    job.set_num_reduce_tasks(reduces)
    job.set_input_format(CompositeInputFormat)
    job.set("mapred.join.expr", CompositeInputFormat.compose(join_type, in_format, *inputs))
    job.set_output_format(out_format)
    job.set_output_key_class(out_key)
    job.set_output_value_class(out_value)
    FileOutputFormat.setOutputPath(job, out)
    return job


# ---------------------------------------------------------------- reduce-side join
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


def make_reduce_side_job(inputs, out, join_type="inner", reduces=1, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name(f"reduce-side join ({join_type})")
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
    """``hbmr examples join [-m maps] [-r reduces] [-inFormat C] [-outFormat C]
    [-outKey C] [-outValue C] [-joinOp inner|outer|override] in1 in2 ... out``"""
    ap = argparse.ArgumentParser(prog="hbmr examples join")
    ap.add_argument("-m", type=int, default=None)
    ap.add_argument("-r", type=int, default=0)
    ap.add_argument("-inFormat", default=None)
    ap.add_argument("-outFormat", default=None)
    ap.add_argument("-outKey", default=None)
    ap.add_argument("-outValue", default=None)
    ap.add_argument("-joinOp", default="inner")
    ap.add_argument("paths", nargs="+", help="input1 input2 [...] output")
    a = ap.parse_args(argv)
    if len(a.paths) < 3:
        ap.error("at least two inputs and an output")
    kw = {}
    for opt, key in (("inFormat", "in_format"), ("outFormat", "out_format"),
                     ("outKey", "out_key"), ("outValue", "out_value")):
        if getattr(a, opt):
            kw[key] = load_class(getattr(a, opt))
    job = make_job(a.paths[:-1], a.paths[-1], a.joinOp, a.r, **kw)
    if a.m:
        job.set_num_map_tasks(a.m)
    rj = JobClient.runJob(job, cluster=cluster)
    return 0 if rj.isSuccessful() else 1
