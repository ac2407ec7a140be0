"""Logalyzer: archive daemon logs into the DFS and analyse them with a job.

Behaviour from hadoop-1.0.3/src/tools/org/apache/hadoop/tools/Logalyzer.java:
``-archive -logs URLS -archiveDir D`` copies logs with DistCp; ``-analysis D
-grep PATTERN -sort COLS -separator SEP`` runs a job whose map emits every log
line matching PATTERN keyed by the chosen separator-delimited columns
(LogRegexMapper + LogComparator), and whose reduce counts them (LongSumReducer),
so the output is ``<sort columns>\\t<count>`` in sort-column order.
"""
from __future__ import annotations

import argparse
import re

from ..io.writable import LongWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.api import Mapper
from ..mapred.lib.basic import LongSumReducer
from . import distcp


class LogRegexMapper(Mapper):
    def configure(self, job):
        self.pattern = re.compile(job.get("mapred.mapper.regex", ".*"))
        cols = job.get("logalizer.logcomparator.sort.columns", "")
        self.cols = [int(c) for c in cols.split(",") if c.strip()] if cols else []
        self.sep = job.get("logalizer.logcomparator.column.separator", " ")

    def map(self, key, value, output, reporter):
        line = str(value)
        if not self.pattern.search(line):
            return
        if self.cols:
            parts = line.split(self.sep)
            line = self.sep.join(parts[c] for c in self.cols if c < len(parts))
        output.collect(Text(line), LongWritable(1))


def archive(log_urls, archive_dir, conf=None, cluster=None):
    return distcp.copy(list(log_urls), archive_dir, conf=conf, cluster=cluster, update=True)


def analyze(input_dir, output_dir, grep=".*", sort_columns="", separator=" ", conf=None,
            cluster=None, reduces=1):
    job = JobConf(conf)
    job.set_job_name(f"logalyzer: {grep}")
    FileInputFormat.setInputPaths(job, input_dir)
    FileOutputFormat.setOutputPath(job, output_dir)
    job.set_mapper_class(LogRegexMapper)
    job.set_combiner_class(LongSumReducer)
    job.set_reducer_class(LongSumReducer)
    job.set_output_key_class(Text)
    job.set_output_value_class(LongWritable)
    job.set("mapred.mapper.regex", grep)
    job.set("logalizer.logcomparator.sort.columns", sort_columns)
    job.set("logalizer.logcomparator.column.separator", separator)
    job.set_num_reduce_tasks(reduces)
    return JobClient.runJob(job, cluster=cluster, verbose=False)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr logalyzer")
    ap.add_argument("-archive", action="store_true")
    ap.add_argument("-logs", default="")
    ap.add_argument("-archiveDir", default=None)
    ap.add_argument("-analysis", default=None, help="output dir of the analysis")
    ap.add_argument("-grep", default=".*")
    ap.add_argument("-sort", default="")
    ap.add_argument("-separator", default=" ")
    a = ap.parse_args(argv)
    if a.archive:
        archive([u for u in a.logs.split(",") if u], a.archiveDir, cluster=cluster)
    if a.analysis:
        analyze(a.archiveDir, a.analysis, a.grep, a.sort, a.separator, cluster=cluster)
    return 0
