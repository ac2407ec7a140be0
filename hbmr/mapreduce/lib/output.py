"""New-API output formats (mapreduce/lib/output/*.java)."""
from __future__ import annotations

from ...mapred import formats as F
from .. import api
from ..adapters import OldWriterAsNew


def _conf(job):
    return job.getConfiguration() if hasattr(job, "getConfiguration") else job


class FileOutputFormat(api.OutputFormat):
    _old = F.TextOutputFormat

    @staticmethod
    def setOutputPath(job, path):  # noqa: N802
        F.set_output_path(_conf(job), str(path))

    @staticmethod
    def getOutputPath(job):  # noqa: N802
        return F.get_output_path(_conf(job))

    @staticmethod
    def setCompressOutput(job, b):  # noqa: N802
        _conf(job).set_boolean("mapred.output.compress", b)

    @staticmethod
    def setOutputCompressorClass(job, codec):  # noqa: N802
        _conf(job).set("mapred.output.compression.codec", getattr(codec, "JAVA_NAME", codec))

    def checkOutputSpecs(self, context):  # noqa: N802
        self._old().checkOutputSpecs(None, _conf(context))

    def getRecordWriter(self, context):  # noqa: N802
        name = getattr(context, "output_name", "part-r-00000")
        w = self._old().getRecordWriter(None, _conf(context), name, context.reporter)
        return OldWriterAsNew(w, context.reporter)


class TextOutputFormat(FileOutputFormat):
    """key \\t value lines (mapred.textoutputformat.separator)."""
    _old = F.TextOutputFormat


class SequenceFileOutputFormat(FileOutputFormat):
    _old = F.SequenceFileOutputFormat


class NullOutputFormat(api.OutputFormat):
    def getRecordWriter(self, context):  # noqa: N802
        class _Null(api.RecordWriter):
            def write(self, k, v):
                pass
        return _Null()


class SequenceFileAsBinaryOutputFormat(FileOutputFormat):
    """BytesWritable keys/values written as raw record bytes under the real
    class names (mapred.SequenceFileAsBinaryOutputFormat)."""
    _old = F.SequenceFileAsBinaryOutputFormat
    setSequenceFileOutputKeyClass = staticmethod(  # noqa: N815
        lambda job, c: F.SequenceFileAsBinaryOutputFormat.setSequenceFileOutputKeyClass(_conf(job), c))
    setSequenceFileOutputValueClass = staticmethod(  # noqa: N815
        lambda job, c: F.SequenceFileAsBinaryOutputFormat.setSequenceFileOutputValueClass(
            _conf(job), c))


class FilterOutputFormat(api.OutputFormat):
    """Wraps another output format and forwards to it
    (mapreduce/lib/output/FilterOutputFormat.java); subclasses override the
    writer to filter or transform records.  The wrapped class is
    ``mapreduce.output.filteroutputformat.class``."""

    KEY = "mapreduce.output.filteroutputformat.class"

    @staticmethod
    def setOutputFormatClass(job, cls):  # noqa: N802
        from ...utils.reflection import class_name
        conf = _conf(job)
        conf.set(FilterOutputFormat.KEY, class_name(cls))

    def _base(self, context):
        from ...utils.reflection import new_instance
        cls = _conf(context).get(self.KEY)
        if not cls:
            raise ValueError("FilterOutputFormat: no output format to wrap "
                             f"({self.KEY} unset)")
        return new_instance(cls, _conf(context))

    def getRecordWriter(self, context):  # noqa: N802
        return self._base(context).getRecordWriter(context)

    def checkOutputSpecs(self, context):  # noqa: N802
        self._base(context).checkOutputSpecs(context)


class LazyOutputFormat(FilterOutputFormat):
    """Creates the wrapped format's file only when the first record is
    written (mapreduce/lib/output/LazyOutputFormat.java): tasks that emit
    nothing leave no empty part files."""

    KEY = "mapreduce.output.lazyoutputformat.outputformat"

    @staticmethod
    def setOutputFormatClass(job, cls):  # noqa: N802
        from ...utils.reflection import class_name
        conf = _conf(job)
        conf.set(LazyOutputFormat.KEY, class_name(cls))
        conf.set("mapreduce.outputformat.class", class_name(LazyOutputFormat))

    def getRecordWriter(self, context):  # noqa: N802
        fmt = self

        class _Lazy(api.RecordWriter):
            w = None

            def write(self_inner, k, v):
                if self_inner.w is None:
                    self_inner.w = fmt._base(context).getRecordWriter(context)
                self_inner.w.write(k, v)

            def close(self_inner, ctx=None):
                if self_inner.w is not None:
                    self_inner.w.close(ctx)
        return _Lazy()


class MultipleOutputs:
    """Named outputs of a new-API task (mapreduce/lib/output/MultipleOutputs.java):
    ``addNamedOutput(job, "errors", TextOutputFormat, Text, Text)``; in the
    task ``mos = MultipleOutputs(context)``, ``mos.write("errors", k, v)`` (to
    ``errors-m-NNNNN``) or ``mos.write("errors", k, v, "sub/base")`` (to
    ``sub/base-m-NNNNN``), then ``mos.close()``."""

    @staticmethod
    def addNamedOutput(job, name, output_format, key_class, value_class):  # noqa: N802
        from ...mapred.lib.multiple import MultipleOutputs as _Old
        _Old.addNamedOutput(_conf(job), name, output_format, key_class, value_class)

    @staticmethod
    def setCountersEnabled(job, enabled):  # noqa: N802
        _conf(job).set_boolean("mo.counters", enabled)

    def __init__(self, context):
        self.ctx = context
        self.conf = context.getConfiguration()
        self.writers = {}
        self.counters = self.conf.get_boolean("mo.counters", False)

    def _writer(self, name, base):
        from ...mapred.jobconf import JobConf
        from ...utils.reflection import new_instance
        w = self.writers.get(base)
        if w is None:
            names = self.conf.get("mo.namedOutputs", "").split()
            if name not in names:
                raise ValueError(f"undefined named output {name!r}")
            sub = JobConf(self.conf)
            sub.set("mapred.output.key.class", self.conf.get(f"mo.namedOutput.{name}.key"))
            sub.set("mapred.output.value.class", self.conf.get(f"mo.namedOutput.{name}.value"))
            fmt = new_instance(self.conf.get(f"mo.namedOutput.{name}.format"), sub)
            is_map = str(self.conf.get("mapred.task.is.map", "true")).lower() == "true"
            part = int(self.conf.get("mapred.task.partition", 0) or 0)
            fn = f"{base}-{'m' if is_map else 'r'}-{part:05d}"
            ctx = api.TaskAttemptContext(sub, self.conf.get("mapred.task.id"),
                                         getattr(self.ctx, "reporter", None))
            ctx.output_name = fn
            if hasattr(fmt, "_old"):            # a new-API FileOutputFormat
                w = fmt.getRecordWriter(ctx)
            else:                               # an old-API format named directly
                from ..adapters import OldWriterAsNew
                w = OldWriterAsNew(fmt.getRecordWriter(None, sub, fn, ctx.reporter), ctx.reporter)
            self.writers[base] = w
        return w

    def write(self, name, key, value, base_output_path=None):
        self._writer(name, base_output_path or name).write(key, value)
        if self.counters:
            self.ctx.getCounter("org.apache.hadoop.mapreduce.lib.output.MultipleOutputs",
                                name).increment(1)

    def close(self):
        for w in self.writers.values():
            w.close(self.ctx)
        self.writers.clear()
