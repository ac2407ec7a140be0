"""New-API input formats (mapreduce/lib/input/*.java)."""
from __future__ import annotations

from ...io.writable import LongWritable, Text
from ...mapred import formats as F
from .. import api

SPLIT_MIN = "mapred.min.split.size"
SPLIT_MAX = "mapred.max.split.size"


def _conf(job):
    return job.getConfiguration() if hasattr(job, "getConfiguration") else job


class FileInputFormat(api.InputFormat):
    """Splits of size max(minSize, min(maxSize, blockSize)) with the 1.1 slop
    (mapreduce/lib/input/FileInputFormat.java:238-275)."""

    @staticmethod
    def addInputPath(job, path):  # noqa: N802
        F.add_input_path(_conf(job), str(path))

    @staticmethod
    def setInputPaths(job, *paths):  # noqa: N802
        F.set_input_paths(_conf(job), *[str(p) for p in paths])

    @staticmethod
    def getInputPaths(job):  # noqa: N802
        return F.get_input_paths(_conf(job))

    @staticmethod
    def setMinInputSplitSize(job, n):  # noqa: N802
        _conf(job).set_long(SPLIT_MIN, n)

    @staticmethod
    def setMaxInputSplitSize(job, n):  # noqa: N802
        _conf(job).set_long(SPLIT_MAX, n)

    def isSplitable(self, context, path):  # noqa: N802
        return F.codec_for_path(path) is None

    def listStatus(self, context):  # noqa: N802
        return F.FileInputFormat().list_status(_conf(context))

    def getSplits(self, context):  # noqa: N802
        conf = _conf(context)
        min_size = max(1, conf.get_long(SPLIT_MIN, 1))
        max_size = conf.get_long(SPLIT_MAX, (1 << 63) - 1)
        splits = []
        for f in self.listStatus(context):
            length = f.length
            if length and self.isSplitable(context, f.path):
                size = max(min_size, min(max_size, f.block_size))
                rem = length
                while rem / size > F.SPLIT_SLOP:
                    splits.append(F.FileSplit(f.path, length - rem, size))
                    rem -= size
                if rem:
                    splits.append(F.FileSplit(f.path, length - rem, rem))
            else:
                splits.append(F.FileSplit(f.path, 0, length))
        return splits


class _WrapOld(api.RecordReader):
    """A new-API RecordReader over an old-API one."""

    def __init__(self, make):
        self.make = make
        self.rr = None
        self.kv = None

    def initialize(self, split, context):
        self.rr = self.make(_conf(context), split)

    def nextKeyValue(self):  # noqa: N802
        self.kv = self.rr.next()
        return self.kv is not None

    def getCurrentKey(self):  # noqa: N802
        return self.kv[0]

    def getCurrentValue(self):  # noqa: N802
        return self.kv[1]

    def getProgress(self):  # noqa: N802
        return self.rr.getProgress()

    def close(self):
        if self.rr is not None:
            self.rr.close()


class LineRecordReader(_WrapOld):
    def __init__(self):
        super().__init__(F.LineRecordReader)


class TextInputFormat(FileInputFormat):
    """(LongWritable offset, Text line)."""

    def createRecordReader(self, split, context):  # noqa: N802
        return LineRecordReader()


class KeyValueTextInputFormat(FileInputFormat):
    def createRecordReader(self, split, context):  # noqa: N802
        return _WrapOld(F.KeyValueLineRecordReader)


class SequenceFileInputFormat(FileInputFormat):
    def listStatus(self, context):  # noqa: N802
        return F.SequenceFileInputFormat().list_status(_conf(context))

    def isSplitable(self, context, path):  # noqa: N802
        return True

    def createRecordReader(self, split, context):  # noqa: N802
        return _WrapOld(F.SequenceFileRecordReader)


class NLineInputFormat(FileInputFormat):
    """N lines per split (mapreduce/lib/input/NLineInputFormat.java)."""

    @staticmethod
    def setNumLinesPerSplit(job, n):  # noqa: N802
        _conf(job).set_int("mapred.line.input.format.linespermap", n)

    def getSplits(self, context):  # noqa: N802
        return F.NLineInputFormat().getSplits(_conf(context), 0)

    def createRecordReader(self, split, context):  # noqa: N802
        return LineRecordReader()


_ = (LongWritable, Text)
