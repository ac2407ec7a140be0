"""Grep: count regex matches, then sort by count descending
(src/examples/org/apache/hadoop/examples/Grep.java: a RegexMapper +
LongSumReducer job into a temp SequenceFile, then an InverseMapper sort job
with LongWritable.DecreasingComparator and one reducer)."""
from __future__ import annotations

import argparse
import os
import shutil
import tempfile

from ..io.writable import LongWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.formats import SequenceFileInputFormat, SequenceFileOutputFormat
from ..mapred.lib.basic import InverseMapper, LongSumReducer, RegexMapper


class DecreasingLong:
    """LongWritable.DecreasingComparator as a sort key over serialised keys."""

    def sort_key(self, kb):
        return -int.from_bytes(kb[:8], "big", signed=True)


def run(inp, out, regex, group=0, conf=None, cluster=None, verbose=False):
    tmp = tempfile.mkdtemp(prefix="grep-temp-")
    try:
        grep = JobConf(conf)
        grep.set_job_name("grep-search")
        FileInputFormat.setInputPaths(grep, *([inp] if isinstance(inp, str) else inp))
        grep.set_mapper_class(RegexMapper)
        grep.set("mapred.mapper.regex", regex)
        grep.set_int("mapred.mapper.regex.group", group)
        grep.set_combiner_class(LongSumReducer)
        grep.set_reducer_class(LongSumReducer)
        FileOutputFormat.setOutputPath(grep, os.path.join(tmp, "out"))
        grep.set_output_format(SequenceFileOutputFormat)
        grep.set_output_key_class(Text)
        grep.set_output_value_class(LongWritable)
        JobClient.runJob(grep, cluster=cluster, verbose=verbose)

        sort = JobConf(conf)
        sort.set_job_name("grep-sort")
        FileInputFormat.setInputPaths(sort, os.path.join(tmp, "out"))
        sort.set_input_format(SequenceFileInputFormat)
        sort.set_mapper_class(InverseMapper)
        sort.set_num_reduce_tasks(1)
        FileOutputFormat.setOutputPath(sort, out)
        sort.set_map_output_key_class(LongWritable)
        sort.set_map_output_value_class(Text)
        sort.set_output_key_class(LongWritable)
        sort.set_output_value_class(Text)
        sort.set_output_key_comparator_class(DecreasingLong)
        return JobClient.runJob(sort, cluster=cluster, verbose=verbose)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr grep")
    ap.add_argument("indir")
    ap.add_argument("outdir")
    ap.add_argument("regex")
    ap.add_argument("group", nargs="?", type=int, default=0)
    a = ap.parse_args(argv)
    rj = run(a.indir, a.outdir, a.regex, a.group, cluster=cluster, verbose=True)
    return 0 if rj.isSuccessful() else 1
