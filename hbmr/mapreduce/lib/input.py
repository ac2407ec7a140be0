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


# ------------------------------------------------------------------ old formats, new API
class _OldFormatReader(api.RecordReader):
    """A new-API RecordReader over an old-API InputFormat's reader."""

    def __init__(self, old_fmt):
        self.fmt = old_fmt
        self.rr = None
        self.kv = None

    def initialize(self, split, context):
        self.rr = self.fmt.getRecordReader(split, _conf(context),
                                           getattr(context, "reporter", None))

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


class _OldBacked(FileInputFormat):
    """New-API file input format whose records come from an old-API format."""
    _old = None

    def listStatus(self, context):  # noqa: N802
        return self._old().list_status(_conf(context))

    def createRecordReader(self, split, context):  # noqa: N802
        return _OldFormatReader(self._old())


class SequenceFileAsTextInputFormat(_OldBacked):
    """Keys and values as Text (their toString)."""
    _old = F.SequenceFileAsTextInputFormat


class SequenceFileAsBinaryInputFormat(_OldBacked):
    """Keys and values as the raw BytesWritable record bytes."""
    _old = F.SequenceFileAsBinaryInputFormat


class SequenceFileInputFilter(_OldBacked):
    """Records whose key passes ``sequencefile.filter.class`` (Regex / Percent
    / MD5 filters of mapred.SequenceFileInputFilter)."""
    _old = F.SequenceFileInputFilter
    RegexFilter = F.SequenceFileInputFilter.RegexFilter
    PercentFilter = F.SequenceFileInputFilter.PercentFilter
    MD5Filter = F.SequenceFileInputFilter.MD5Filter
    setFilterClass = staticmethod(lambda job, cls: F.SequenceFileInputFilter.setFilterClass(  # noqa: E731,N815
        _conf(job), cls))


class CombineFileInputFormat(api.InputFormat):
    """Packs many small files (or max-split-size chunks of them) into each
    split (mapreduce/lib/input/CombineFileInputFormat.java); subclasses set
    ``record_reader``, a ``make(conf, FileSplit)`` per-chunk reader (default
    lines).  Split planning is mapred.lib.CombineFileInputFormat's."""

    record_reader = staticmethod(F.LineRecordReader)

    def __init__(self):
        self.max_split_size = 0

    def setMaxSplitSize(self, n):  # noqa: N802
        self.max_split_size = int(n)

    def _old(self):
        from ...mapred.lib.combine import CombineFileInputFormat as _Old

        class _O(_Old):
            record_reader = staticmethod(type(self).record_reader)
        return _O()

    def getSplits(self, context):  # noqa: N802
        from ...mapred.jobconf import JobConf
        conf = JobConf(_conf(context))
        if self.max_split_size:
            conf.set_long("mapred.max.split.size", self.max_split_size)
        return self._old().getSplits(conf, conf.get_num_map_tasks())

    def createRecordReader(self, split, context):  # noqa: N802
        return _OldFormatReader(self._old())


# ------------------------------------------------------------------ MultipleInputs
_NEW_INPUTS = "mapreduce.input.multipleinputs.dir.formats"
_NEW_MAPPERS = "mapreduce.input.multipleinputs.dir.mappers"


class MultipleInputs:
    """A new-API input format (and optionally a mapper) per input path
    (mapreduce/lib/input/MultipleInputs.java)."""

    @staticmethod
    def addInputPath(job, path, input_format, mapper=None):  # noqa: N802
        import os

        from ...utils.reflection import class_name
        conf = _conf(job)
        path = os.path.abspath(str(path))
        cur = conf.get(_NEW_INPUTS)
        conf.set(_NEW_INPUTS, (cur + "," if cur else "") + f"{path};{class_name(input_format)}")
        conf.set("mapreduce.inputformat.class", class_name(DelegatingInputFormat))
        if mapper is not None:
            ms = conf.get(_NEW_MAPPERS)
            conf.set(_NEW_MAPPERS, (ms + "," if ms else "") + f"{path};{class_name(mapper)}")
            conf.set("mapreduce.map.class", class_name(DelegatingMapper))

    @staticmethod
    def _table(conf, key):
        out = {}
        for item in (conf.get(key) or "").split(","):
            if item:
                p, c = item.split(";", 1)
                out[p] = c
        return out


class DelegatingInputFormat(api.InputFormat):
    def getSplits(self, context):  # noqa: N802
        from ...mapred.jobconf import JobConf
        from ...mapred.lib.multiple import TaggedInputSplit
        from ...utils.reflection import new_instance
        conf = _conf(context)
        mappers = MultipleInputs._table(conf, _NEW_MAPPERS)
        out = []
        for path, fcls in MultipleInputs._table(conf, _NEW_INPUTS).items():
            sub = JobConf(conf)
            F.set_input_paths(sub, path)
            fmt = new_instance(fcls, sub)
            for s in fmt.getSplits(api.JobContext(sub)):
                out.append(TaggedInputSplit(s, fcls, mappers.get(path)))
        return out

    def createRecordReader(self, split, context):  # noqa: N802
        from ...utils.reflection import new_instance
        fmt = new_instance(split.fmt_cls, _conf(context))
        rep = getattr(context, "reporter", None)
        if rep is not None:
            rep.tagged_split = split

        class _R(api.RecordReader):
            def __init__(self_inner):
                self_inner.rr = fmt.createRecordReader(split.split, context)

            def initialize(self_inner, s, ctx):
                self_inner.rr.initialize(split.split, ctx)

            def nextKeyValue(self_inner):  # noqa: N802
                return self_inner.rr.nextKeyValue()

            def getCurrentKey(self_inner):  # noqa: N802
                return self_inner.rr.getCurrentKey()

            def getCurrentValue(self_inner):  # noqa: N802
                return self_inner.rr.getCurrentValue()

            def getProgress(self_inner):  # noqa: N802
                return self_inner.rr.getProgress()

            def close(self_inner):
                self_inner.rr.close()
        return _R()


class DelegatingMapper(api.Mapper):
    """Runs the mapper named for the split's input path."""

    def run(self, context):
        from ...utils.reflection import new_instance
        conf = context.getConfiguration()
        split = getattr(context.reporter, "tagged_split", None) or context.getInputSplit()
        cls = getattr(split, "mapper_cls", None)
        if not cls:
            path = getattr(getattr(split, "split", split), "path", "")
            cls = next((c for p, c in MultipleInputs._table(conf, _NEW_MAPPERS).items()
                        if str(path).startswith(p)), "hbmr.mapreduce.api:Mapper")
        new_instance(cls, conf).run(context)
