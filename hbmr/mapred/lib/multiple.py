"""Multiple inputs and outputs (hadoop-1.0.3 mapred/lib/{MultipleInputs,
DelegatingInputFormat,DelegatingMapper,TaggedInputSplit,MultipleOutputs,
MultipleOutputFormat,MultipleTextOutputFormat,MultipleSequenceFileOutputFormat}.java).
"""
from __future__ import annotations

import io
import os
import struct

from ...io.writable import Text
from ...utils.reflection import class_name, load_class, new_instance
from .. import formats as F
from ..api import InputFormat, InputSplit, Mapper, OutputCollector, RecordWriter

_INPUTS = "mapred.input.dir.formats"
_MAPPERS = "mapred.input.dir.mappers"


# ----------------------------------------------------------------------- inputs
class MultipleInputs:
    @staticmethod
    def addInputPath(job, path, input_format, mapper=None):  # noqa: N802
        path = os.path.abspath(str(path))
        fmts = job.get(_INPUTS)
        job.set(_INPUTS, (fmts + "," if fmts else "") + f"{path};{class_name(input_format)}")
        job.set_input_format(DelegatingInputFormat)
        if mapper is not None:
            ms = job.get(_MAPPERS)
            job.set(_MAPPERS, (ms + "," if ms else "") + f"{path};{class_name(mapper)}")
            job.set_mapper_class(DelegatingMapper)

    @staticmethod
    def _table(job, key):
        out = {}
        for item in (job.get(key) or "").split(","):
            if item:
                p, c = item.split(";", 1)
                out[p] = c
        return out


class TaggedInputSplit(InputSplit):
    """A split plus the input format and mapper that own it."""

    def __init__(self, split, fmt_cls: str, mapper_cls: str | None):
        self.split, self.fmt_cls, self.mapper_cls = split, fmt_cls, mapper_cls or ""

    def getLength(self):  # noqa: N802
        return self.split.getLength()

    def getLocations(self):  # noqa: N802
        return self.split.getLocations()

    def serialize(self):
        inner = self.split.serialize()
        cls = f"{type(self.split).__module__}:{type(self.split).__qualname__}"
        parts = [Text(cls).serialize(), Text(self.fmt_cls).serialize(),
                 Text(self.mapper_cls).serialize(), struct.pack(">i", len(inner)), inner]
        return b"".join(parts)

    @classmethod
    def deserialize(cls, raw):
        b = io.BytesIO(raw)
        vals = []
        for _ in range(3):
            t = Text()
            t.readFields(b)
            vals.append(str(t))
        n = struct.unpack(">i", b.read(4))[0]
        split = load_class(vals[0]).deserialize(b.read(n))
        return cls(split, vals[1], vals[2] or None)


class DelegatingInputFormat(InputFormat):
    def getSplits(self, job, num_splits):  # noqa: N802
        from ..jobconf import JobConf
        fmts = MultipleInputs._table(job, _INPUTS)
        mappers = MultipleInputs._table(job, _MAPPERS)
        out = []
        for path, fcls in fmts.items():
            sub = JobConf(job)
            F.set_input_paths(sub, path)
            fmt = new_instance(load_class(fcls), sub)
            for s in fmt.getSplits(sub, num_splits):
                out.append(TaggedInputSplit(s, fcls, mappers.get(path)))
        return out

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        fmt = new_instance(load_class(split.fmt_cls), job)
        reporter.tagged_split = split
        return fmt.getRecordReader(split.split, job, reporter)


class DelegatingMapper(Mapper):
    def configure(self, job):
        self.job = job
        self.mapper = None

    def map(self, key, value, output, reporter):
        if self.mapper is None:
            split = getattr(reporter, "tagged_split", None) or getattr(reporter, "split", None)
            cls = getattr(split, "mapper_cls", None)
            if not cls:
                # find the mapper by the split's path
                path = getattr(getattr(reporter, "split", None), "path", "")
                table = MultipleInputs._table(self.job, _MAPPERS)
                cls = next((c for p, c in table.items() if path.startswith(p)), None)
            self.mapper = new_instance(load_class(cls) if cls else
                                       "hbmr.mapred.lib.basic:IdentityMapper", self.job)
        self.mapper.map(key, value, output, reporter)

    def close(self):
        if self.mapper is not None:
            self.mapper.close()


# ----------------------------------------------------------------------- outputs
class MultipleOutputFormat(F.FileOutputFormat):
    """Routes each record to a file chosen by generateFileNameForKeyValue."""

    def generateFileNameForKeyValue(self, key, value, name):  # noqa: N802
        return name

    def generateActualKey(self, key, value):  # noqa: N802
        return key

    def generateActualValue(self, key, value):  # noqa: N802
        return value

    def getBaseRecordWriter(self, fs, job, name, progress):  # noqa: N802
        raise NotImplementedError

    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        fmt = self
        writers = {}

        class _W(RecordWriter):
            def write(self_inner, key, value):
                fn = fmt.generateFileNameForKeyValue(key, value, name)
                w = writers.get(fn)
                if w is None:
                    w = writers[fn] = fmt.getBaseRecordWriter(fs, job, fn, progress)
                w.write(fmt.generateActualKey(key, value), fmt.generateActualValue(key, value))

            def close(self_inner, reporter=None):
                for w in writers.values():
                    w.close(reporter)
        return _W()


class MultipleTextOutputFormat(MultipleOutputFormat):
    def getBaseRecordWriter(self, fs, job, name, progress):  # noqa: N802
        return F.TextOutputFormat().getRecordWriter(fs, job, name, progress)


class MultipleSequenceFileOutputFormat(MultipleOutputFormat):
    def getBaseRecordWriter(self, fs, job, name, progress):  # noqa: N802
        return F.SequenceFileOutputFormat().getRecordWriter(fs, job, name, progress)


class MultipleOutputs:
    """Named extra outputs of a task: ``addNamedOutput(job, "errors",
    TextOutputFormat, Text, Text)`` then ``mos.getCollector("errors", reporter)``.
    Files are ``<name>-m-NNNNN`` / ``<name>-r-NNNNN`` in the task's output dir."""

    @staticmethod
    def addNamedOutput(job, name, output_format, key_class, value_class):  # noqa: N802
        if not name.isalnum():
            raise ValueError(f"named output must be alphanumeric: {name!r}")
        names = job.get("mo.namedOutputs", "")
        if name in names.split():
            raise ValueError(f"named output {name!r} already defined")
        job.set("mo.namedOutputs", (names + " " + name).strip())
        job.set(f"mo.namedOutput.{name}.format", class_name(output_format))
        job.set(f"mo.namedOutput.{name}.key", class_name(key_class))
        job.set(f"mo.namedOutput.{name}.value", class_name(value_class))

    @staticmethod
    def getNamedOutputsList(job):  # noqa: N802
        return job.get("mo.namedOutputs", "").split()

    def __init__(self, job):
        self.job = job
        self.writers = {}

    def getCollector(self, name, reporter):  # noqa: N802
        if name not in self.getNamedOutputsList(self.job):
            raise ValueError(f"undefined named output {name!r}")
        w = self.writers.get(name)
        if w is None:
            from ..jobconf import JobConf
            sub = JobConf(self.job)
            sub.set("mapred.output.key.class", self.job.get(f"mo.namedOutput.{name}.key"))
            sub.set("mapred.output.value.class", self.job.get(f"mo.namedOutput.{name}.value"))
            fmt = new_instance(self.job.get_class(f"mo.namedOutput.{name}.format"), sub)
            is_map = str(self.job.get("mapred.task.is.map", "true")).lower() == "true"
            part = int(self.job.get("mapred.task.partition", 0) or 0)
            fn = f"{name}-{'m' if is_map else 'r'}-{part:05d}"
            w = self.writers[name] = fmt.getRecordWriter(None, sub, fn, reporter)

        class _C(OutputCollector):
            def collect(self_inner, k, v):
                w.write(k, v)
        return _C()

    def close(self):
        for w in self.writers.values():
            w.close(None)
        self.writers.clear()
