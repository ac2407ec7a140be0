"""WordCount — BASELINE config 1 (CPU-only mappers on the LocalJobRunner).

Same job as hadoop-1.0.3/src/examples/org/apache/hadoop/examples/WordCount.java:
map emits (word, 1) per whitespace token, combiner + reducer sum.
"""
from __future__ import annotations

from ..io.writable import IntWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper, Reducer


class WordCountMapper(Mapper):
    one = IntWritable(1)

    def map(self, key, value, output, reporter):
        for w in value.bytes.split():
            output.collect(Text(w), self.one)


class IntSumReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(key, IntWritable(sum(v.value for v in values)))


def make_job(inputs, output, reduces=1, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name("wordcount")
    job.set_output_key_class(Text)
    job.set_output_value_class(IntWritable)
    job.set_mapper_class(WordCountMapper)
    job.set_combiner_class(IntSumReducer)
    job.set_reducer_class(IntSumReducer)
    job.set_num_reduce_tasks(reduces)
    FileInputFormat.setInputPaths(job, *([inputs] if isinstance(inputs, str) else inputs))
    FileOutputFormat.setOutputPath(job, output)
    return job


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr wordcount")
    ap.add_argument("input", nargs="+")
    ap.add_argument("output")
    ap.add_argument("-r", "--reduces", type=int, default=1)
    a = ap.parse_args(argv)
    job = make_job(a.input, a.output, a.reduces)
    rj = JobClient.runJob(job)
    return 0 if rj.isSuccessful() else 1
