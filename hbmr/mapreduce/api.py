"""The new ("mapreduce") user API: context-object Mapper/Reducer and the
InputFormat/RecordReader/OutputFormat/RecordWriter/OutputCommitter contracts.

Mirrors hadoop-1.0.3/src/mapred/org/apache/hadoop/mapreduce/{Mapper,Reducer,
Partitioner,InputFormat,RecordReader,InputSplit,OutputFormat,RecordWriter,
OutputCommitter,JobContext,TaskAttemptContext,MapContext,ReduceContext,
TaskInputOutputContext}.java.  Jobs written against it run on the same
runtime as old-API jobs (hbmr.mapreduce.adapters translates), and — unlike the
reference, whose runNewMapper had no GPU branch (MapTask.java:725, SURVEY.md
G15) — a new-API job may name a split-level GPU map as well.
"""
from __future__ import annotations

import enum


class Counter:
    """A live counter handle (Counter.increment / getValue)."""

    def __init__(self, reporter, group, name):
        self._rep, self.group, self.name = reporter, group, name

    def increment(self, amount=1):
        self._rep.incrCounter(self.group, self.name, amount)

    def getValue(self):  # noqa: N802
        c = self._rep.getCounter(self.group, self.name)
        return getattr(c, "value", c) if c is not None else 0

    getDisplayName = lambda self: self.name  # noqa: E731, N815

    def getName(self):  # noqa: N802
        return self.name


class JobContext:
    def __init__(self, conf, job_id=None):
        self.conf = conf
        self.job_id = job_id

    def getConfiguration(self):  # noqa: N802
        return self.conf

    def getJobID(self):  # noqa: N802
        return self.job_id

    def getNumReduceTasks(self):  # noqa: N802
        return self.conf.get_num_reduce_tasks()

    def getJobName(self):  # noqa: N802
        return self.conf.get_job_name()


class TaskAttemptContext(JobContext):
    def __init__(self, conf, attempt_id=None, reporter=None):
        super().__init__(conf)
        self.attempt_id = attempt_id
        self.reporter = reporter

    def getTaskAttemptID(self):  # noqa: N802
        return self.attempt_id

    def setStatus(self, msg):  # noqa: N802
        if self.reporter is not None:
            self.reporter.setStatus(msg)

    def progress(self):
        if self.reporter is not None:
            self.reporter.progress()


class TaskInputOutputContext(TaskAttemptContext):
    def __init__(self, conf, attempt_id, reporter, output):
        super().__init__(conf, attempt_id, reporter)
        self._out = output

    def write(self, key, value):
        self._out.collect(key, value)

    def getCounter(self, group, name=None):  # noqa: N802
        if name is None:
            if isinstance(group, enum.Enum):
                return Counter(self.reporter, type(group).__qualname__, group.name)
            raise TypeError("getCounter(enum) or getCounter(group, name)")
        return Counter(self.reporter, group, name)

    def getOutputCommitter(self):  # noqa: N802
        return None


class MapContext(TaskInputOutputContext):
    def __init__(self, conf, attempt_id, reporter, output, reader, split):
        super().__init__(conf, attempt_id, reporter, output)
        self._reader = reader
        self._split = split
        self._kv = None

    def nextKeyValue(self) -> bool:  # noqa: N802
        self._kv = self._reader.next()
        return self._kv is not None

    def getCurrentKey(self):  # noqa: N802
        return self._kv[0]

    def getCurrentValue(self):  # noqa: N802
        return self._kv[1]

    def getInputSplit(self):  # noqa: N802
        return self._split


class ReduceContext(TaskInputOutputContext):
    """The reduce-side context; values for one key are an iterable."""

    def __init__(self, conf, attempt_id, reporter, output):
        super().__init__(conf, attempt_id, reporter, output)
        self._key = None
        self._values = None

    def getCurrentKey(self):  # noqa: N802
        return self._key

    def getValues(self):  # noqa: N802
        return self._values


class Mapper:
    """setup → map(key, value, context) per record → cleanup (Mapper.run)."""

    Context = MapContext

    def setup(self, context):
        pass

    def map(self, key, value, context):
        context.write(key, value)

    def cleanup(self, context):
        pass

    def run(self, context):
        self.setup(context)
        try:
            while context.nextKeyValue():
                self.map(context.getCurrentKey(), context.getCurrentValue(), context)
        finally:
            self.cleanup(context)


class Reducer:
    """setup → reduce(key, values, context) per key group → cleanup."""

    Context = ReduceContext

    def setup(self, context):
        pass

    def reduce(self, key, values, context):
        for v in values:
            context.write(key, v)

    def cleanup(self, context):
        pass


class Partitioner:
    def getPartition(self, key, value, num_partitions: int) -> int:  # noqa: N802
        raise NotImplementedError


class InputSplit:
    def getLength(self) -> int:  # noqa: N802
        return 0

    def getLocations(self) -> list:  # noqa: N802
        return []

    def serialize(self) -> bytes:
        raise NotImplementedError


class RecordReader:
    def initialize(self, split, context):
        pass

    def nextKeyValue(self) -> bool:  # noqa: N802
        raise NotImplementedError

    def getCurrentKey(self):  # noqa: N802
        raise NotImplementedError

    def getCurrentValue(self):  # noqa: N802
        raise NotImplementedError

    def getProgress(self) -> float:  # noqa: N802
        return 0.0

    def close(self):
        pass


class InputFormat:
    def getSplits(self, context: JobContext) -> list:  # noqa: N802
        raise NotImplementedError

    def createRecordReader(self, split, context) -> RecordReader:  # noqa: N802
        raise NotImplementedError


class RecordWriter:
    def write(self, key, value):
        raise NotImplementedError

    def close(self, context):
        pass


class OutputCommitter:
    def setupJob(self, context):  # noqa: N802
        pass

    def cleanupJob(self, context):  # noqa: N802
        pass

    def setupTask(self, context):  # noqa: N802
        pass

    def needsTaskCommit(self, context) -> bool:  # noqa: N802
        return False

    def commitTask(self, context):  # noqa: N802
        pass

    def abortTask(self, context):  # noqa: N802
        pass


class OutputFormat:
    def getRecordWriter(self, context) -> RecordWriter:  # noqa: N802
        raise NotImplementedError

    def checkOutputSpecs(self, context):  # noqa: N802
        pass

    def getOutputCommitter(self, context):  # noqa: N802
        return OutputCommitter()
