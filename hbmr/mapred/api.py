"""The old ("mapred") user API: Mapper, Reducer, Partitioner, OutputCollector,
Reporter, RecordReader/Writer, InputFormat/OutputFormat, InputSplit, MapRunnable.

Interfaces mirror hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/{Mapper,
Reducer,Partitioner,OutputCollector,Reporter,RecordReader,RecordWriter,
InputFormat,OutputFormat,InputSplit,MapRunnable}.java.  Python duck typing
replaces generics; method names keep Hadoop's camelCase so user code ports
line-for-line, with snake_case aliases.

GPU additions (hbmr-native): :class:`GpuMapper` is the
split-level map interface — it receives a whole HBM-resident split as device
tensors instead of one record per call, which is how a GPU map task avoids the
reference's per-record Pipes messages (SURVEY.md §2.9 "Pipes socket").
"""
from __future__ import annotations


class JobConfigurable:
    def configure(self, job) -> None:
        pass


class Closeable:
    def close(self) -> None:
        pass


class Mapper(JobConfigurable, Closeable):
    """map(key, value, output, reporter) is called once per input record."""

    def map(self, key, value, output, reporter):
        raise NotImplementedError


class Reducer(JobConfigurable, Closeable):
    """reduce(key, values_iterator, output, reporter) once per key group."""

    def reduce(self, key, values, output, reporter):
        raise NotImplementedError


class Partitioner(JobConfigurable):
    def getPartition(self, key, value, num_partitions: int) -> int:  # noqa: N802
        raise NotImplementedError

    def get_partition(self, key, value, num_partitions):
        return self.getPartition(key, value, num_partitions)


class OutputCollector:
    def collect(self, key, value) -> None:
        raise NotImplementedError

    def __call__(self, key, value):
        self.collect(key, value)


class Reporter:
    """Progress / status / counter sink handed to user code."""

    def setStatus(self, status: str):  # noqa: N802
        pass

    def progress(self):
        pass

    def getCounter(self, group, name=None):  # noqa: N802
        return None

    def incrCounter(self, group, name, amount=1):  # noqa: N802
        pass

    def getInputSplit(self):  # noqa: N802
        raise NotImplementedError

    def getProgress(self):  # noqa: N802
        return 0.0


class _NullReporter(Reporter):
    def getInputSplit(self):  # noqa: N802
        return None


NULL_REPORTER = _NullReporter()


class InputSplit:
    def getLength(self) -> int:  # noqa: N802
        return 0

    def getLocations(self) -> list[str]:  # noqa: N802
        return []

    def serialize(self) -> bytes:
        raise NotImplementedError


class RecordReader(Closeable):
    def next(self):
        """Return the next (key, value) or None at end of input."""
        raise NotImplementedError

    def getPos(self) -> int:  # noqa: N802
        return 0

    def getProgress(self) -> float:  # noqa: N802
        return 0.0

    def __iter__(self):
        while True:
            kv = self.next()
            if kv is None:
                return
            yield kv


class RecordWriter:
    def write(self, key, value):
        raise NotImplementedError

    def close(self, reporter=None):
        pass


class InputFormat:
    def getSplits(self, job, num_splits: int) -> list:  # noqa: N802
        raise NotImplementedError

    def getRecordReader(self, split, job, reporter) -> RecordReader:  # noqa: N802
        raise NotImplementedError


class OutputFormat:
    def getRecordWriter(self, fs, job, name: str, progress) -> RecordWriter:  # noqa: N802
        raise NotImplementedError

    def checkOutputSpecs(self, fs, job):  # noqa: N802
        pass


class MapRunnable(JobConfigurable):
    """Drives a map task: run(record_reader, output_collector, reporter)."""

    def run(self, reader, output, reporter):
        raise NotImplementedError


class GpuMapper(JobConfigurable, Closeable):
    """Split-level GPU map function (hbmr extension).

    ``map_split(ctx)`` runs one whole input split on the task's device.  ``ctx``
    is a :class:`hbmr.gpu.runner.GpuTaskContext` exposing the split as an
    HBM-resident tensor, the device/stream, the job's broadcast side data
    (DistributedCache analogue) and an ``emit_partial`` sink for combined map
    output.  Kernels launched on ``ctx.stream`` are asynchronous; the runtime
    records completion events around the call.
    """

    #: dtype/feature layout the split cache should materialise for this mapper
    split_layout: dict = {}

    def setup(self, ctx):
        pass

    def map_split(self, ctx):
        raise NotImplementedError

    def cpu_map_split(self, ctx):
        """Optional CPU implementation of the same split-level map (for CPU slots)."""
        raise NotImplementedError


# snake_case conveniences --------------------------------------------------------
Mapper.map_record = Mapper.map
