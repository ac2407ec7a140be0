"""Stock mappers, reducers and partitioners (hadoop-1.0.3/src/mapred/org/apache/
hadoop/mapred/lib/*): IdentityMapper, IdentityReducer, HashPartitioner,
TokenCountMapper, LongSumReducer, InverseMapper, RegexMapper,
KeyFieldBasedPartitioner, FieldSelection-style helpers, TotalOrderPartitioner and
InputSampler (the TeraSort/Sort range partitioning path)."""
from __future__ import annotations

import bisect
import random
import re

from ...io.serializer import hash_code as serializer_hash
from ...io.writable import IntWritable, LongWritable, Text, hash_bytes
from ..api import Mapper, Partitioner, Reducer


class IdentityMapper(Mapper):
    def map(self, key, value, output, reporter):
        output.collect(key, value)


class IdentityReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        for v in values:
            output.collect(key, v)


class HashPartitioner(Partitioner):
    """(key.hashCode() & Integer.MAX_VALUE) % numReduceTasks (HashPartitioner.java:31-34)."""

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        h = key.hash_code() if hasattr(key, "hash_code") else serializer_hash(key)
        return (h & 0x7FFFFFFF) % num_partitions


class TokenCountMapper(Mapper):
    """Emits (token, 1) for every whitespace token (lib/TokenCountMapper.java)."""

    def map(self, key, value, output, reporter):
        one = LongWritable(1)
        for tok in str(value).split():
            output.collect(Text(tok), one)


class LongSumReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(key, LongWritable(sum(v.get() for v in values)))


class IntSumReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(key, IntWritable(sum(v.get() for v in values)))


class InverseMapper(Mapper):
    def map(self, key, value, output, reporter):
        output.collect(value, key)


class RegexMapper(Mapper):
    """Emits (match, 1) for each match of ``mapred.mapper.regex`` (group
    ``mapred.mapper.regex.group``), as lib/RegexMapper.java."""

    def configure(self, job):
        self.pattern = re.compile(job.get("mapred.mapper.regex", ".*"))
        self.group = job.get_int("mapred.mapper.regex.group", 0)

    def map(self, key, value, output, reporter):
        one = LongWritable(1)
        for m in self.pattern.finditer(str(value)):
            output.collect(Text(m.group(self.group)), one)


from .keyfield import KeyFieldBasedComparator, KeyFieldBasedPartitioner  # noqa: E402,F401


class TotalOrderPartitioner(Partitioner):
    """Range partitioner over sorted split points (lib/TotalOrderPartitioner.java).

    Split points are the serialized-key sort keys of R-1 boundary keys, read
    from ``total.order.partitioner.path`` (written by :func:`write_partition_file`)
    or set in-process via :meth:`set_split_points`."""

    _inproc: dict = {}

    def configure(self, job):
        self.kcls = job.get_map_output_key_class()
        path = job.get("total.order.partitioner.path")
        if path and path in TotalOrderPartitioner._inproc:
            self.points = TotalOrderPartitioner._inproc[path]
        elif path:
            from ...io import sequencefile as seqf
            pts = []
            with seqf.Reader(path) as r:
                while True:
                    raw = r.next_raw()
                    if raw is None:
                        break
                    pts.append(self.kcls.raw_sort_key(raw[0]))
            self.points = pts
        else:
            self.points = []

    @classmethod
    def set_split_points(cls, job, keys, path="inproc:default"):
        kc = job.get_map_output_key_class()
        cls._inproc[path] = sorted(kc.raw_sort_key(k.serialize()) for k in keys)
        job.set("total.order.partitioner.path", path)

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        k = type(key).raw_sort_key(key.serialize())
        return bisect.bisect_right(self.points, k)


def write_partition_file(job, keys, path):
    from ...io import sequencefile as seqf
    from ...io.writable import NullWritable
    with seqf.Writer(path, job.get_map_output_key_class(), NullWritable) as w:
        for k in sorted(keys, key=lambda k: type(k).raw_sort_key(k.serialize())):
            w.append(k, NullWritable())
    job.set("total.order.partitioner.path", path)


class InputSampler:
    """Samples input keys to build TotalOrderPartitioner split points
    (lib/InputSampler.java: RandomSampler / SplitSampler / IntervalSampler)."""

    def __init__(self, freq=0.1, num_samples=10000, max_splits=10, seed=0):
        self.freq = freq
        self.num_samples = num_samples
        self.max_splits = max_splits
        self.rng = random.Random(seed)

    def get_sample(self, input_format, job):
        splits = input_format.getSplits(job, job.get_num_map_tasks())
        self.rng.shuffle(splits)
        samples = []
        for sp in splits[:self.max_splits]:
            rr = input_format.getRecordReader(sp, job, None)
            for k, _v in rr:
                if self.rng.random() <= self.freq:
                    if len(samples) < self.num_samples:
                        samples.append(k)
                    else:
                        i = self.rng.randrange(self.num_samples)
                        samples[i] = k
            rr.close()
        return samples

    def split_points(self, samples, num_partitions):
        if num_partitions <= 1 or not samples:
            return []
        s = sorted(samples, key=lambda k: type(k).raw_sort_key(k.serialize()))
        step = len(s) / num_partitions
        return [s[min(len(s) - 1, int(round(step * i)))] for i in range(1, num_partitions)]

    def write_partition_file(self, input_format, job, path):
        pts = self.split_points(self.get_sample(input_format, job), job.get_num_reduce_tasks())
        write_partition_file(job, pts, path)
        return pts
