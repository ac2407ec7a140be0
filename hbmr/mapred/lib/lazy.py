"""Old-API LazyOutputFormat (hadoop-1.0.3 mapred/lib/LazyOutputFormat.java):
wraps the real output format (``mapred.lazy.output.format.class``) and only
creates a task's output file when its first record is written — tasks with
no output leave no empty part files.  ``set_output_format_class`` installs it."""
from __future__ import annotations

from ..api import OutputFormat, RecordWriter
from ...utils.reflection import class_name, load_class

KEY = "mapred.lazy.output.format.class"


def set_output_format_class(job, cls):
    job.set("mapred.output.format.class", class_name(LazyOutputFormat))
    job.set(KEY, class_name(cls))


class _LazyRecordWriter(RecordWriter):
    def __init__(self, fmt, fs, job, name, progress):
        self.args = (fs, job, name, progress)
        self.fmt = fmt
        self.w = None

    def write(self, key, value):
        if self.w is None:
            self.w = self.fmt.getRecordWriter(*self.args)
        self.w.write(key, value)

    def close(self, reporter=None):
        if self.w is not None:
            self.w.close(reporter)


class LazyOutputFormat(OutputFormat):
    def _base(self, job):
        name = job.get(KEY)
        if not name:
            raise ValueError(f"LazyOutputFormat needs {KEY}")
        return load_class(name)()

    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        return _LazyRecordWriter(self._base(job), fs, job, name, progress)

    def checkOutputSpecs(self, fs, job):  # noqa: N802
        self._base(job).checkOutputSpecs(fs, job)
