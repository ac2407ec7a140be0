"""Sort: identity map/reduce over SequenceFiles, optionally totally ordered
(src/examples/org/apache/hadoop/examples/Sort.java: -inFormat/-outFormat,
-outKey/-outValue, -r reduces, -totalOrder pcnt numSamples maxSplits →
InputSampler.RandomSampler + TotalOrderPartitioner)."""
from __future__ import annotations

import argparse
import os

from ..io import sequencefile as seqf
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.formats import SequenceFileInputFormat, SequenceFileOutputFormat
from ..mapred.lib.basic import IdentityMapper, IdentityReducer, InputSampler, TotalOrderPartitioner
from ..utils.reflection import load_class


def make_job(inp, out, reduces=1, total_order=None, conf=None, in_format=None,
             out_format=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name("sorter")
    FileInputFormat.setInputPaths(job, *([inp] if isinstance(inp, str) else inp))
    FileOutputFormat.setOutputPath(job, out)
    job.set_input_format(in_format or SequenceFileInputFormat)
    job.set_output_format(out_format or SequenceFileOutputFormat)
    job.set_mapper_class(IdentityMapper)
    job.set_reducer_class(IdentityReducer)
    job.set_num_reduce_tasks(reduces)
    # key/value classes of the (first) input file
    first = _first_file(inp)
    if first and (in_format is None or in_format is SequenceFileInputFormat):
        with seqf.Reader(first) as r:
            job.set_output_key_class(r.key_class)
            job.set_output_value_class(r.value_class)
    if total_order is not None and reduces > 1:
        pcnt, num_samples, max_splits = total_order
        sampler = InputSampler(pcnt, num_samples, max_splits)
        fmt = (in_format or SequenceFileInputFormat)()
        path = os.path.join(os.path.dirname(os.path.abspath(out)),
                            f"_sortPartitioning-{os.path.basename(out)}")
        sampler.write_partition_file(fmt, job, path)
        job.set_partitioner_class(TotalOrderPartitioner)
    return job


def _first_file(inp):
    p = inp if isinstance(inp, str) else inp[0]
    if os.path.isdir(p):
        fs = sorted(f for f in os.listdir(p) if not f.startswith(("_", ".")))
        return os.path.join(p, fs[0]) if fs else None
    return p if os.path.exists(p) else None


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr sort")
    ap.add_argument("indir")
    ap.add_argument("outdir")
    ap.add_argument("-r", type=int, default=1)
    ap.add_argument("-inFormat")
    ap.add_argument("-outFormat")
    ap.add_argument("-totalOrder", nargs=3, metavar=("pcnt", "numSamples", "maxSplits"))
    a = ap.parse_args(argv)
    to = None
    if a.totalOrder:
        to = (float(a.totalOrder[0]), int(a.totalOrder[1]), int(a.totalOrder[2]))
    job = make_job(a.indir, a.outdir, a.r, to,
                   in_format=load_class(a.inFormat) if a.inFormat else None,
                   out_format=load_class(a.outFormat) if a.outFormat else None)
    rj = JobClient.runJob(job, cluster=cluster)
    return 0 if rj.isSuccessful() else 1
