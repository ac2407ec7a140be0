"""Run new-API (hbmr.mapreduce) classes on the task runtime.

The runtime drives old-API interfaces (MapRunnable, Reducer, Partitioner,
InputFormat, OutputFormat); these adapters wrap the user's new-API classes,
named under the ``mapreduce.*.class`` keys (the keys of
hadoop-1.0.3 mapreduce/JobContext.java:49-58), so Job-based programs run on
the same MapTask/ReduceTask, CPU and GPU slots, local runner and cluster.
"""
from __future__ import annotations

from ..mapred import api as old
from ..mapred import counters as C
from ..mapred.formats import TextOutputFormat as _OldTextOut
from ..utils.reflection import new_instance
from . import api

MAP_KEY = "mapreduce.map.class"
REDUCE_KEY = "mapreduce.reduce.class"
COMBINE_KEY = "mapreduce.combine.class"
PARTITION_KEY = "mapreduce.partitioner.class"
INPUT_KEY = "mapreduce.inputformat.class"
OUTPUT_KEY = "mapreduce.outputformat.class"


class _CountingReader:
    def __init__(self, reader):
        self.r = reader
        self.n = 0

    def next(self):
        kv = self.r.next()
        if kv is not None:
            self.n += 1
        return kv


class NewMapperRunner(old.MapRunnable):
    """MapRunnable that runs a new-API Mapper's run(context)."""

    def configure(self, job):
        self.job = job

    def run(self, reader, output, reporter):
        m = new_instance(self.job.get_class(MAP_KEY, "hbmr.mapreduce.api:Mapper"), self.job)
        cr = _CountingReader(reader)
        ctx = api.MapContext(self.job, self.job.get("mapred.task.id"), reporter, output, cr,
                             getattr(reporter, "split", None))
        try:
            m.run(ctx)
        finally:
            reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, cr.n)


class NewReducerAdapter(old.Reducer):
    key = REDUCE_KEY

    def configure(self, job):
        self.job = job
        self.r = new_instance(job.get_class(self.key, "hbmr.mapreduce.api:Reducer"), job)
        self.ctx = None

    def reduce(self, key, values, output, reporter):
        if self.ctx is None:
            self.ctx = api.ReduceContext(self.job, self.job.get("mapred.task.id"), reporter,
                                         output)
            self.r.setup(self.ctx)
        self.ctx._out = output
        self.ctx._key = key
        self.ctx._values = values
        self.r.reduce(key, values, self.ctx)

    def close(self):
        if self.ctx is not None:
            self.r.cleanup(self.ctx)


class NewCombinerAdapter(NewReducerAdapter):
    key = COMBINE_KEY


class NewPartitionerAdapter(old.Partitioner):
    def configure(self, job):
        self.p = new_instance(job.get_class(PARTITION_KEY,
                                            "hbmr.mapreduce.lib.partition:HashPartitioner"), job)

    def getPartition(self, key, value, n):  # noqa: N802
        return self.p.getPartition(key, value, n)


class _OldRecordReader(old.RecordReader):
    def __init__(self, rr):
        self.rr = rr

    def next(self):
        if not self.rr.nextKeyValue():
            return None
        return self.rr.getCurrentKey(), self.rr.getCurrentValue()

    def getProgress(self):  # noqa: N802
        return self.rr.getProgress()

    def close(self):
        self.rr.close()


class NewInputFormatAdapter(old.InputFormat):
    def configure(self, job):
        self.job = job
        self.fmt = new_instance(job.get_class(INPUT_KEY,
                                              "hbmr.mapreduce.lib.input:TextInputFormat"), job)

    def getSplits(self, job, num_splits):  # noqa: N802
        return self.fmt.getSplits(api.JobContext(job))

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        ctx = api.TaskAttemptContext(job, job.get("mapred.task.id"), reporter)
        rr = self.fmt.createRecordReader(split, ctx)
        rr.initialize(split, ctx)
        return _OldRecordReader(rr)


class _OldRecordWriter(old.RecordWriter):
    def __init__(self, w, ctx):
        self.w, self.ctx = w, ctx

    def write(self, key, value):
        self.w.write(key, value)

    def close(self, reporter):
        self.w.close(self.ctx)


class NewOutputFormatAdapter(old.OutputFormat):
    def configure(self, job):
        self.job = job
        self.fmt = new_instance(job.get_class(OUTPUT_KEY,
                                              "hbmr.mapreduce.lib.output:TextOutputFormat"), job)

    def getRecordWriter(self, fs, job, name, progress):  # noqa: N802
        # new-API file names: part-m-NNNNN (map-only) / part-r-NNNNN
        if name.startswith("part-") and name[5:].isdigit():
            name = f"part-{'m' if job.get_num_reduce_tasks() == 0 else 'r'}-{name[5:]}"
        ctx = api.TaskAttemptContext(job, job.get("mapred.task.id"), progress)
        ctx.output_name = name
        return _OldRecordWriter(self.fmt.getRecordWriter(ctx), ctx)

    def checkOutputSpecs(self, fs, job):  # noqa: N802
        self.fmt.checkOutputSpecs(api.JobContext(job))


class OldWriterAsNew(api.RecordWriter):
    """A new-API RecordWriter over an old-API one (used by lib.output formats)."""

    def __init__(self, w, reporter):
        self.w, self.rep = w, reporter

    def write(self, key, value):
        self.w.write(key, value)

    def close(self, context):
        self.w.close(self.rep)


_ = _OldTextOut
