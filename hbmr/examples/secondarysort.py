"""SecondarySort (src/examples/org/apache/hadoop/examples/SecondarySort.java):
input lines "a b" (two ints); keys are IntPair(a, b) sorted by (a, b),
partitioned and grouped by a only, so each reduce call sees one a with its b
values in increasing order.  Output: a separator line, then "a b" lines."""
from __future__ import annotations

import argparse
import struct

from ..io.writable import IntWritable, Text, WritableComparable
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from ..mapred.api import Partitioner

SEPARATOR = Text("------------------------------------------------")


class IntPair(WritableComparable):
    """Two ints, serialised as offset-binary big-endian so raw bytes sort like
    the pair (IntPair.write in the reference adds Integer.MIN_VALUE)."""

    def __init__(self, first=0, second=0):
        self.first, self.second = int(first), int(second)

    def set(self, a, b):
        self.first, self.second = int(a), int(b)

    def getFirst(self):  # noqa: N802
        return self.first

    def getSecond(self):  # noqa: N802
        return self.second

    def serialize(self):
        return struct.pack(">II", (self.first + (1 << 31)) & 0xFFFFFFFF,
                           (self.second + (1 << 31)) & 0xFFFFFFFF)

    def readFields(self, inp):  # noqa: N802
        a, b = struct.unpack(">II", inp.read(8))
        self.first, self.second = a - (1 << 31), b - (1 << 31)

    @classmethod
    def raw_sort_key(cls, raw):
        return raw[:8]

    def hash_code(self):
        return (self.first * 157 + self.second) & 0xFFFFFFFF

    def __str__(self):
        return f"{self.first} {self.second}"


class FirstPartitioner(Partitioner):
    def getPartition(self, key, value, n):  # noqa: N802
        return abs(key.first * 127) % n


class FirstGroupingComparator:
    def sort_key(self, kb):
        return kb[:4]


class MapClass(Mapper):
    def map(self, key, value, output, reporter):
        parts = str(value).split()
        if len(parts) >= 2:
            a, b = int(parts[0]), int(parts[1])
            output.collect(IntPair(a, b), IntWritable(b))


class Reduce(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(SEPARATOR, None)
        first = IntWritable(key.first)
        for v in values:
            output.collect(first, v)


def make_job(inp, out, reduces=1, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name("secondary sort")
    FileInputFormat.setInputPaths(job, inp)
    FileOutputFormat.setOutputPath(job, out)
    job.set_mapper_class(MapClass)
    job.set_reducer_class(Reduce)
    job.set_partitioner_class(FirstPartitioner)
    job.set_output_value_grouping_comparator(FirstGroupingComparator)
    job.set_map_output_key_class(IntPair)
    job.set_map_output_value_class(IntWritable)
    job.set_output_key_class(Text)
    job.set_output_value_class(IntWritable)
    job.set_num_reduce_tasks(reduces)
    return job


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr secondarysort")
    ap.add_argument("input")
    ap.add_argument("output")
    a = ap.parse_args(argv)
    rj = JobClient.runJob(make_job(a.input, a.output), cluster=cluster)
    return 0 if rj.isSuccessful() else 1
