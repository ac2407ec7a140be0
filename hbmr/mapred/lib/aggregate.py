"""The aggregate framework (hadoop-1.0.3 mapred/lib/aggregate/*.java).

A job is described by aggregator descriptors: each turns an input (key, value)
into (``"TYPE:id"``, value) pairs, where TYPE names an aggregator.  The
generic mapper emits them, the combiner and reducer fold values per id with
the named aggregator and the reducer writes ``id \\t result``.

Aggregators: LongValueSum, LongValueMax, LongValueMin, DoubleValueSum,
StringValueMax, StringValueMin, UniqValueCount, ValueHistogram.
Descriptors are configured as ``aggregator.descriptor.num`` /
``aggregator.descriptor.<i>`` = ``UserDefined,<module:Class>``.
"""
from __future__ import annotations

from ...io.writable import Text
from ...utils.reflection import load_class
from ..api import Mapper, Reducer


class LongValueSum:
    def __init__(self):
        self.v = 0

    def addNextValue(self, x):  # noqa: N802
        self.v += int(str(x))

    def getReport(self):  # noqa: N802
        return str(self.v)

    def getCombinerOutput(self):  # noqa: N802
        return [self.getReport()]


class LongValueMax(LongValueSum):
    def __init__(self):
        self.v = None

    def addNextValue(self, x):  # noqa: N802
        x = int(str(x))
        self.v = x if self.v is None else max(self.v, x)


class LongValueMin(LongValueMax):
    def addNextValue(self, x):  # noqa: N802
        x = int(str(x))
        self.v = x if self.v is None else min(self.v, x)


class DoubleValueSum(LongValueSum):
    def __init__(self):
        self.v = 0.0

    def addNextValue(self, x):  # noqa: N802
        self.v += float(str(x))


class StringValueMax(LongValueSum):
    def __init__(self):
        self.v = None

    def addNextValue(self, x):  # noqa: N802
        x = str(x)
        self.v = x if self.v is None or x > self.v else self.v


class StringValueMin(StringValueMax):
    def addNextValue(self, x):  # noqa: N802
        x = str(x)
        self.v = x if self.v is None or x < self.v else self.v


class UniqValueCount:
    def __init__(self):
        self.items = set()

    def addNextValue(self, x):  # noqa: N802
        self.items.add(str(x))

    def getReport(self):  # noqa: N802
        return str(len(self.items))

    def getCombinerOutput(self):  # noqa: N802
        return sorted(self.items)


class ValueHistogram:
    """value "v" or "v\\tcount"; report: number of distinct values, then
    min/median/max/average/stddev of the counts (ValueHistogram.java)."""

    def __init__(self):
        self.counts = {}

    def addNextValue(self, x):  # noqa: N802
        s = str(x)
        v, _, c = s.partition("\t")
        self.counts[v] = self.counts.get(v, 0) + (int(c) if c else 1)

    def getReport(self):  # noqa: N802
        if not self.counts:
            return "0"
        cs = sorted(self.counts.values())
        n = len(cs)
        avg = sum(cs) / n
        sd = (sum((c - avg) ** 2 for c in cs) / n) ** 0.5
        return f"{n}\t{cs[0]}\t{cs[n // 2]}\t{cs[-1]}\t{avg}\t{sd}"

    def getCombinerOutput(self):  # noqa: N802
        return [f"{v}\t{c}" for v, c in sorted(self.counts.items())]


AGGREGATORS = {c.__name__: c for c in (LongValueSum, LongValueMax, LongValueMin, DoubleValueSum,
                                       StringValueMax, StringValueMin, UniqValueCount,
                                       ValueHistogram)}


class ValueAggregatorBaseDescriptor:
    LONG_VALUE_SUM = "LongValueSum"
    VALUE_HISTOGRAM = "ValueHistogram"
    UNIQ_VALUE_COUNT = "UniqValueCount"

    @staticmethod
    def generateEntry(typ, id_, val):  # noqa: N802
        return Text(f"{typ}:{id_}"), val

    def configure(self, job):
        pass

    def generateKeyValPairs(self, key, val):  # noqa: N802
        # default: count each input record under "record_count"
        return [self.generateEntry(self.LONG_VALUE_SUM, "record_count", Text("1"))]


def _descriptors(job):
    out = []
    for i in range(job.get_int("aggregator.descriptor.num", 0)):
        spec = job.get(f"aggregator.descriptor.{i}", "")
        kind, _, cls = spec.partition(",")
        if kind == "UserDefined" and cls:
            d = load_class(cls)()
            if hasattr(d, "configure"):
                d.configure(job)
            out.append(d)
    return out or [ValueAggregatorBaseDescriptor()]


def _split(key):
    s = str(key)
    typ, _, id_ = s.partition(":")
    return typ, id_


class ValueAggregatorMapper(Mapper):
    def configure(self, job):
        self.descs = _descriptors(job)

    def map(self, key, value, output, reporter):
        for d in self.descs:
            for k, v in d.generateKeyValPairs(key, value):
                output.collect(k, v)


class ValueAggregatorCombiner(Reducer):
    def reduce(self, key, values, output, reporter):
        typ, _ = _split(key)
        agg = AGGREGATORS[typ]()
        for v in values:
            agg.addNextValue(v)
        for out in agg.getCombinerOutput():
            output.collect(key, Text(out))


class ValueAggregatorReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        typ, id_ = _split(key)
        agg = AGGREGATORS[typ]()
        for v in values:
            agg.addNextValue(v)
        output.collect(Text(id_), Text(agg.getReport()))


class ValueAggregatorJob:
    @staticmethod
    def createValueAggregatorJob(inputs, output, descriptors, reduces=1, conf=None):  # noqa: N802
        from ...utils.reflection import class_name
        from ..formats import set_input_paths, set_output_path
        from ..jobconf import JobConf
        job = JobConf(conf)
        job.set_job_name("ValueAggregatorJob")
        set_input_paths(job, *([inputs] if isinstance(inputs, str) else inputs))
        set_output_path(job, output)
        job.set_mapper_class(ValueAggregatorMapper)
        job.set_combiner_class(ValueAggregatorCombiner)
        job.set_reducer_class(ValueAggregatorReducer)
        job.set_output_key_class(Text)
        job.set_output_value_class(Text)
        job.set_num_reduce_tasks(reduces)
        job.set_int("aggregator.descriptor.num", len(descriptors))
        for i, d in enumerate(descriptors):
            job.set(f"aggregator.descriptor.{i}", f"UserDefined,{class_name(d)}")
        return job
