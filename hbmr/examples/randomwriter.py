"""RandomWriter and RandomTextWriter (src/examples/org/apache/hadoop/examples/
{RandomWriter,RandomTextWriter}.java): map-only jobs over empty splits, each map
writing ``test.randomwrite.bytes_per_map`` bytes of random records into a
SequenceFile.

RandomWriter: BytesWritable keys/values, lengths uniform in
[min_key, max_key] / [min_value, max_value] (test.randomwrite.{min,max}_{key,value}).
RandomTextWriter: Text keys/values of random words from a fixed vocabulary.
"""
from __future__ import annotations

import argparse
import random

from ..io.writable import BytesWritable, Text
from ..mapred import FileOutputFormat, JobClient, JobConf
from ..mapred.api import InputFormat, Mapper, RecordReader
from ..mapred.formats import SequenceFileOutputFormat
from .sleepjob import EmptySplit


class _CounterReader(RecordReader):
    def __init__(self, name):
        self.name = name
        self.done = False

    def next(self):
        if self.done:
            return None
        self.done = True
        return Text(self.name), Text(self.name)


class RandomInputFormat(InputFormat):
    """One empty split per map; each yields one record (the map's name)."""

    def getSplits(self, job, num_splits):  # noqa: N802
        return [EmptySplit() for _ in range(max(1, num_splits))]

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return _CounterReader(job.get("mapred.task.id", "map"))


class RandomMapper(Mapper):
    def configure(self, job):
        self.total = job.get_long("test.randomwrite.bytes_per_map", 1 << 20)
        self.kmin = job.get_int("test.randomwrite.min_key", 10)
        self.kmax = job.get_int("test.randomwrite.max_key", 1000)
        self.vmin = job.get_int("test.randomwrite.min_value", 0)
        self.vmax = job.get_int("test.randomwrite.max_value", 20000)
        self.rng = random.Random(hash(job.get("mapred.task.id", "")) & 0xFFFFFFFF)

    def map(self, key, value, output, reporter):
        left = self.total
        n = 0
        while left > 0:
            kl = self.rng.randint(self.kmin, self.kmax)
            vl = self.rng.randint(self.vmin, self.vmax)
            output.collect(BytesWritable(self.rng.randbytes(kl)),
                           BytesWritable(self.rng.randbytes(vl)))
            left -= kl + vl
            n += 1
            if n % 200 == 0:
                reporter.setStatus(f"wrote record {n}. {left} bytes left.")
        reporter.incrCounter("RandomWriter", "RECORDS_WRITTEN", n)
        reporter.incrCounter("RandomWriter", "BYTES_WRITTEN", self.total - left)


_WORDS = ("diurnalness Homoiousian spiranthic tetragynian silverhead ungreat lithograph "
          "exploiter physiologian by hellbender Filipendula undeterring antiscolic pentagamist "
          "hypoid cacuminal sertularian schoolmasterism nonuple gallybeggar phytonic swearingly "
          "nebular Confervales thermochemically atomizer afterpressure infranodal Ghent "
          "gorilloid enterectomy pyxie mesophyte seraphism unpremonished charioteer").split()


class RandomTextMapper(Mapper):
    def configure(self, job):
        self.total = job.get_long("test.randomtextwrite.bytes_per_map", 1 << 20)
        self.kmin = job.get_int("test.randomtextwrite.min_words_key", 5)
        self.kmax = job.get_int("test.randomtextwrite.max_words_key", 10)
        self.vmin = job.get_int("test.randomtextwrite.min_words_value", 10)
        self.vmax = job.get_int("test.randomtextwrite.max_words_value", 100)
        self.rng = random.Random(hash(job.get("mapred.task.id", "")) & 0xFFFFFFFF)

    def _words(self, lo, hi):
        return " ".join(self.rng.choice(_WORDS) for _ in range(self.rng.randint(lo, hi)))

    def map(self, key, value, output, reporter):
        left = self.total
        while left > 0:
            k = Text(self._words(self.kmin, self.kmax))
            v = Text(self._words(self.vmin, self.vmax))
            output.collect(k, v)
            left -= len(k.bytes) + len(v.bytes)
        reporter.incrCounter("RandomTextWriter", "BYTES_WRITTEN", self.total - left)


def make_job(out, maps=2, bytes_per_map=1 << 20, text=False, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name("random-text-writer" if text else "random-writer")
    job.set_input_format(RandomInputFormat)
    job.set_mapper_class(RandomTextMapper if text else RandomMapper)
    job.set_num_map_tasks(maps)
    job.set_num_reduce_tasks(0)
    job.set_output_format(SequenceFileOutputFormat)
    job.set_output_key_class(Text if text else BytesWritable)
    job.set_output_value_class(Text if text else BytesWritable)
    job.set_long("test.randomtextwrite.bytes_per_map" if text else
                 "test.randomwrite.bytes_per_map", bytes_per_map)
    FileOutputFormat.setOutputPath(job, out)
    return job


def main(argv=None, cluster=None, text=False):
    ap = argparse.ArgumentParser(prog="hbmr randomtextwriter" if text else "hbmr randomwriter")
    ap.add_argument("outdir")
    ap.add_argument("-m", "--maps", type=int, default=2)
    ap.add_argument("-b", "--bytes-per-map", type=int, default=1 << 20)
    a = ap.parse_args(argv)
    rj = JobClient.runJob(make_job(a.outdir, a.maps, a.bytes_per_map, text), cluster=cluster)
    return 0 if rj.isSuccessful() else 1


def main_text(argv=None, cluster=None):
    return main(argv, cluster, text=True)
