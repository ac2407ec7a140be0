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
