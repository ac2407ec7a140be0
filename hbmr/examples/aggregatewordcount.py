"""AggregateWordCount / AggregateWordHistogram (src/examples/org/apache/hadoop/
examples/AggregateWord{Count,Histogram}.java) on the aggregate framework."""
from __future__ import annotations

import argparse

from ..io.writable import Text
from ..mapred import JobClient
from ..mapred.lib.aggregate import ValueAggregatorBaseDescriptor, ValueAggregatorJob


class WordCountPlugIn(ValueAggregatorBaseDescriptor):
    def generateKeyValPairs(self, key, val):  # noqa: N802
        one = Text("1")
        return [self.generateEntry(self.LONG_VALUE_SUM, w, one) for w in str(val).split()]


class WordHistogramPlugIn(ValueAggregatorBaseDescriptor):
    def generateKeyValPairs(self, key, val):  # noqa: N802
        return [self.generateEntry(self.VALUE_HISTOGRAM, "WORD_HISTOGRAM", Text(f"{w}\t1"))
                for w in str(val).split()]


def main(argv=None, cluster=None, histogram=False):
    ap = argparse.ArgumentParser(prog="hbmr aggregatewordcount")
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("reduces", nargs="?", type=int, default=1)
    a = ap.parse_args(argv)
    job = ValueAggregatorJob.createValueAggregatorJob(
        a.input, a.output, [WordHistogramPlugIn if histogram else WordCountPlugIn], a.reduces)
    rj = JobClient.runJob(job, cluster=cluster)
    return 0 if rj.isSuccessful() else 1


def main_histogram(argv=None, cluster=None):
    return main(argv, cluster, histogram=True)
