"""MultiFileWordCount (src/examples/org/apache/hadoop/examples/MultiFileWordCount.java):
word count where each map reads several whole files (MultiFileInputFormat)."""
from __future__ import annotations

import argparse

from ..io.writable import LongWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.lib.basic import LongSumReducer, TokenCountMapper
from ..mapred.lib.combine import MultiFileInputFormat


def make_job(inp, out, maps=2, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name("MultiFileWordCount")
    job.set_input_format(MultiFileInputFormat)
    job.set_num_map_tasks(maps)
    job.set_mapper_class(TokenCountMapper)
    job.set_combiner_class(LongSumReducer)
    job.set_reducer_class(LongSumReducer)
    job.set_output_key_class(Text)
    job.set_output_value_class(LongWritable)
    FileInputFormat.setInputPaths(job, *([inp] if isinstance(inp, str) else inp))
    FileOutputFormat.setOutputPath(job, out)
    return job


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr multifilewc")
    ap.add_argument("input")
    ap.add_argument("output")
    a = ap.parse_args(argv)
    rj = JobClient.runJob(make_job(a.input, a.output), cluster=cluster)
    return 0 if rj.isSuccessful() else 1
