"""Input and output formats.

* FileInputFormat split math follows hadoop-1.0.3/src/mapred/org/apache/hadoop/
  mapred/FileInputFormat.java:206-261: goalSize = totalSize / numSplits,
  splitSize = max(minSize, min(goalSize, blockSize)), keep cutting while
  remaining/splitSize > SPLIT_SLOP (1.1); hidden files (_ or . prefix) skipped.
* TextInputFormat/LineRecordReader: key = byte offset (LongWritable), value = line
  (Text); a split that does not start at 0 skips its first (partial) line and
  every split reads one line past its end, so each line is read exactly once.
* NLineInputFormat (mapred/lib/NLineInputFormat.java:78,120): N lines per split —
  the reference configuration's input format (conf/mapred-site.xml:15-20).
* SequenceFileInputFormat / SequenceFileRecordReader: splits honoured via sync
  markers (``pos >= end && syncSeen`` ends a split).
* TextOutputFormat ("key\\tvalue\\n"), SequenceFileOutputFormat, NullOutputFormat.
"""
from __future__ import annotations

import io
import os
import struct

from .. import fs as F
from ..fs import get_fs, hidden, strip_scheme
from ..io import sequencefile as seqf
from ..io.compress import codec_for_path, get_codec
from ..io.writable import LongWritable, NullWritable, Text, Writable
from .api import InputFormat, InputSplit, OutputFormat, RecordReader, RecordWriter

SPLIT_SLOP = 1.1


# --------------------------------------------------------------------------- splits
class FileSplit(InputSplit):
    def __init__(self, path: str, start: int, length: int, hosts=None):
        self.path = str(path)
        self.start = int(start)
        self.length = int(length)
        self.hosts = list(hosts or [])

    def getPath(self):  # noqa: N802
        return self.path

    def getStart(self):  # noqa: N802
        return self.start

    def getLength(self):  # noqa: N802
        return self.length

    def getLocations(self):  # noqa: N802
        return self.hosts

    def serialize(self) -> bytes:
        """Java FileSplit.write: Text path, long start, long length."""
        return Text(self.path).serialize() + struct.pack(">qq", self.start, self.length)

    @classmethod
    def deserialize(cls, raw: bytes) -> "FileSplit":
        b = io.BytesIO(raw)
        t = Text()
        t.readFields(b)
        start, length = struct.unpack(">qq", b.read(16))
        return cls(str(t), start, length)

    def __repr__(self):
        return f"{self.path}:{self.start}+{self.length}"

    def __eq__(self, o):
        return isinstance(o, FileSplit) and (self.path, self.start, self.length) == \
            (o.path, o.start, o.length)

    def __hash__(self):
        return hash((self.path, self.start, self.length))


# --------------------------------------------------------------------------- inputs
def get_input_paths(job) -> list[str]:
    v = job.get("mapred.input.dir", "")
    return [p for p in (s.strip() for s in v.split(",")) if p]


def set_input_paths(job, *paths):
    job.set("mapred.input.dir", ",".join(strip_scheme(p) for p in paths))


def add_input_path(job, path):
    cur = get_input_paths(job)
    cur.append(strip_scheme(path))
    job.set("mapred.input.dir", ",".join(cur))


def get_output_path(job):
    v = job.get("mapred.output.dir")
    return strip_scheme(v) if v else None


def set_output_path(job, path):
    job.set("mapred.output.dir", strip_scheme(path))


class FileInputFormat(InputFormat):
    setInputPaths = staticmethod(set_input_paths)  # noqa: N815
    addInputPath = staticmethod(add_input_path)  # noqa: N815
    getInputPaths = staticmethod(get_input_paths)  # noqa: N815

    def is_splitable(self, fs, path) -> bool:
        return codec_for_path(path) is None

    def list_status(self, job):
        out = []
        for p in get_input_paths(job):
            fs = get_fs(p, job)
            matches = fs.glob_status(p) if any(ch in p for ch in "*?[") else \
                [fs.get_file_status(p)]
            if not matches:
                raise FileNotFoundError(f"Input path does not exist: {p}")
            for st in matches:
                if st.is_dir:
                    for c in fs.list_status(st.path):
                        if not c.is_dir and not hidden(c.path):
                            out.append(c)
                elif not hidden(st.path):
                    out.append(st)
        return out

    listStatus = list_status  # noqa: N815

    def compute_split_size(self, goal, min_size, block_size):
        return max(min_size, min(goal, block_size))

    def getSplits(self, job, num_splits: int):  # noqa: N802
        files = self.list_status(job)
        total = sum(f.length for f in files)
        goal = total // (num_splits if num_splits > 0 else 1)
        min_size = max(job.get_long("mapred.min.split.size", 1), 1)
        splits = []
        for f in files:
            fs = get_fs(f.path, job)
            length = f.length
            # split hosts = the DataNodes holding the split's first block
            # (FileInputFormat.getBlockIndex), for data-local scheduling
            hosts = (lambda s, n: F.block_hosts(fs, f.path, s, n)) if F.is_dfs(f.path) else \
                (lambda s, n: None)
            if length != 0 and self.is_splitable(fs, f.path):
                split_size = self.compute_split_size(goal, min_size, f.block_size)
                remaining = length
                while remaining / split_size > SPLIT_SLOP:
                    st = length - remaining
                    splits.append(FileSplit(f.path, st, split_size, hosts(st, split_size)))
                    remaining -= split_size
                if remaining != 0:
                    st = length - remaining
                    splits.append(FileSplit(f.path, st, remaining, hosts(st, remaining)))
            elif length != 0:
                splits.append(FileSplit(f.path, 0, length, hosts(0, length)))
            else:
                splits.append(FileSplit(f.path, 0, 0))
        return splits

    get_splits = getSplits


class LineRecordReader(RecordReader):
    """Lines of a split (LineRecordReader.java: a split owns every line that
    starts at or before its end; the first partial line belongs to the previous
    split).  Reads 1 MiB chunks and splits them into lines in C (bytes.split)
    instead of one readline() per record; keys and values are fresh objects."""
    CHUNK = 1 << 20

    def __init__(self, job, split: FileSplit):
        self.start = split.start
        self.end = split.start + split.length
        self.path = split.path
        self.codec = codec_for_path(split.path)
        if self.codec is not None:
            with F.fopen(split.path, "rb") as f:
                self.f = io.BytesIO(self.codec.decompress(f.read()))
            self.end = 1 << 62
        else:
            self.f = F.fopen(split.path, "rb", buffering=1 << 20)
        self.f.seek(self.start)
        self.pos = self.start
        if self.start != 0:
            # skip the first (partial) line; the previous split owns it
            skipped = self.f.readline()
            self.pos += len(skipped)
        self._lines = []        # lines of the current chunk (newline stripped)
        self._i = 0
        self._nl = 1            # 1: the chunk's lines each ended with "\n"
        self._tail = b""        # partial last line of the chunk read so far

    def _fill(self):
        while True:
            data = self.f.read(self.CHUNK)
            if not data:
                if self._tail:
                    self._lines, self._tail, self._i, self._nl = [self._tail], b"", 0, 0
                    return True
                return False
            parts = (self._tail + data if self._tail else data).split(b"\n")
            self._tail = parts.pop()
            if parts:
                self._lines, self._i, self._nl = parts, 0, 1
                return True

    def next(self):
        pos = self.pos
        if pos > self.end:
            return None
        if self._i >= len(self._lines) and not self._fill():
            return None
        line = self._lines[self._i]
        self._i += 1
        self.pos = pos + len(line) + self._nl
        if line.endswith(b"\r"):
            line = line[:-1]
        key = LongWritable.__new__(LongWritable)
        key.value = pos
        val = Text.__new__(Text)
        val.bytes = line
        return key, val

    def getPos(self):  # noqa: N802
        return self.pos

    def getProgress(self):  # noqa: N802
        if self.end == self.start:
            return 0.0
        return min(1.0, (self.pos - self.start) / max(1, self.end - self.start))

    def close(self):
        self.f.close()


class TextInputFormat(FileInputFormat):
    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return LineRecordReader(job, split)


class KeyValueLineRecordReader(RecordReader):
    def __init__(self, job, split):
        self.lr = LineRecordReader(job, split)
        sep = job.get("key.value.separator.in.input.line", "\t")
        self.sep = sep.encode()[:1] or b"\t"

    def next(self):
        kv = self.lr.next()
        if kv is None:
            return None
        line = kv[1].bytes
        i = line.find(self.sep)
        if i < 0:
            return Text(line), Text(b"")
        return Text(line[:i]), Text(line[i + 1:])

    def getProgress(self):  # noqa: N802
        return self.lr.getProgress()

    def close(self):
        self.lr.close()


class KeyValueTextInputFormat(FileInputFormat):
    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return KeyValueLineRecordReader(job, split)


class NLineInputFormat(FileInputFormat):
    """Each split holds N lines (``mapred.line.input.format.linespermap``)."""

    def getSplits(self, job, num_splits):  # noqa: N802
        n = max(1, job.get_int("mapred.line.input.format.linespermap", 1))
        splits = []
        for st in self.list_status(job):
            begin = 0
            length = 0
            count = 0
            with F.fopen(st.path, "rb") as f:
                for line in f:
                    count += 1
                    length += len(line)
                    if count == n:
                        splits.append(self._mk(st.path, begin, length))
                        begin += length
                        length = 0
                        count = 0
            if count:
                splits.append(self._mk(st.path, begin, length))
        return splits

    @staticmethod
    def _mk(path, begin, length):
        # the reference shifts every split but the first back by one byte so the
        # LineRecordReader's "skip first partial line" lands on the intended line
        # (NLineInputFormat.java:97-110)
        if begin == 0:
            return FileSplit(path, 0, length - 1)
        return FileSplit(path, begin - 1, length)

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return LineRecordReader(job, split)


class SequenceFileRecordReader(RecordReader):
    def __init__(self, job, split: FileSplit):
        self.reader = seqf.Reader(split.path)
        self.start = split.start
        self.end = split.start + split.length
        if self.start > self.reader.get_position():
            self.reader.sync_to(self.start)
        self.start = self.reader.get_position()
        self.more = self.start < self.end
        self.kcls = self.reader.key_class
        self.vcls = self.reader.value_class

    def next_raw(self):
        if not self.more:
            return None
        pos = self.reader.get_position()
        raw = self.reader.next_raw()
        if raw is None or (pos >= self.end and self.reader.sync_seen):
            self.more = False
            return None
        return raw

    def next(self):
        raw = self.next_raw()
        if raw is None:
            return None
        return self.kcls.deserialize(raw[0]), self.vcls.deserialize(raw[1])

    def getPos(self):  # noqa: N802
        return self.reader.get_position()

    def getProgress(self):  # noqa: N802
        if self.end == self.start:
            return 0.0
        return min(1.0, (self.reader.get_position() - self.start) / (self.end - self.start))

    def close(self):
        self.reader.close()


class SequenceFileInputFormat(FileInputFormat):
    def __init__(self):
        pass

    def list_status(self, job):
        files = super().list_status(job)
        out = []
        fs = get_fs(conf=job)
        for f in files:
            # a MapFile directory contributes its data file
            if f.is_dir:
                data = os.path.join(f.path, "data")
                out.append(fs.get_file_status(data))
            else:
                out.append(f)
        return out

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return SequenceFileRecordReader(job, split)


class SequenceFileAsTextInputFormat(SequenceFileInputFormat):
    def getRecordReader(self, split, job, reporter):  # noqa: N802
        rr = SequenceFileRecordReader(job, split)

        class _AsText(RecordReader):
            def next(self_inner):
                kv = rr.next()
                return None if kv is None else (Text(str(kv[0])), Text(str(kv[1])))

            def getProgress(self_inner):  # noqa: N802
                return rr.getProgress()

            def close(self_inner):
                rr.close()

        return _AsText()


class SequenceFileAsBinaryInputFormat(SequenceFileInputFormat):
    """Keys and values as raw BytesWritable, not deserialised
    (SequenceFileAsBinaryInputFormat.java): the record bytes exactly as stored
    (after RECORD/BLOCK decompression), for jobs that move records unread."""

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        from ..io.writable import BytesWritable
        rr = SequenceFileRecordReader(job, split)

        class _AsBinary(RecordReader):
            def next(self_inner):
                raw = rr.next_raw()
                return None if raw is None else (BytesWritable(raw[0]), BytesWritable(raw[1]))

            def getKeyClassName(self_inner):  # noqa: N802,N805
                return rr.reader.key_class_name

            def getValueClassName(self_inner):  # noqa: N802,N805
                return rr.reader.value_class_name

            def getProgress(self_inner):  # noqa: N802
                return rr.getProgress()

            def getPos(self_inner):  # noqa: N802
                return rr.getPos()

            def close(self_inner):
                rr.close()

        return _AsBinary()


FILTER_CLASS = "sequencefile.filter.class"
FILTER_FREQUENCY = "sequencefile.filter.frequency"
FILTER_REGEX = "sequencefile.filter.regex"


class SequenceFileInputFilter(SequenceFileInputFormat):
    """Only the records whose KEY passes ``sequencefile.filter.class``
    (SequenceFileInputFilter.java): RegexFilter (``sequencefile.filter.regex``
    must match the whole key), PercentFilter (the 1st of every
    ``sequencefile.filter.frequency`` records, default 10) or MD5Filter (keys
    whose MD5's first 8 bytes, as a signed long, are a multiple of the
    frequency — a stable sample of keys)."""

    class Filter:
        def configure(self, conf):
            pass

        def accept(self, key) -> bool:
            raise NotImplementedError

    class RegexFilter(Filter):
        @staticmethod
        def setPattern(conf, regex):  # noqa: N802
            import re
            try:
                re.compile(regex)
            except re.error as e:
                raise ValueError(f"Invalid pattern: {regex}") from e
            conf.set(FILTER_REGEX, regex)

        def configure(self, conf):
            import re
            regex = conf.get(FILTER_REGEX)
            if regex is None:
                raise RuntimeError(f"{FILTER_REGEX} not set")
            self.p = re.compile(regex)

        def accept(self, key):
            return self.p.fullmatch(str(key)) is not None

    class PercentFilter(Filter):
        @staticmethod
        def setFrequency(conf, f):  # noqa: N802
            if f <= 0:
                raise ValueError(f"Negative {FILTER_FREQUENCY}: {f}")
            conf.set_int(FILTER_FREQUENCY, f)

        def configure(self, conf):
            self.frequency = conf.get_int(FILTER_FREQUENCY, 10)
            if self.frequency <= 0:
                raise RuntimeError(f"Negative {FILTER_FREQUENCY}: {self.frequency}")
            self.count = 0

        def accept(self, key):
            ok = self.count == 0
            self.count += 1
            if self.count == self.frequency:
                self.count = 0
            return ok

    class MD5Filter(Filter):
        setFrequency = staticmethod(lambda conf, f: SequenceFileInputFilter.PercentFilter  # noqa: E731,N815
                                    .setFrequency(conf, f))

        def configure(self, conf):
            self.frequency = conf.get_int(FILTER_FREQUENCY, 10)
            if self.frequency <= 0:
                raise RuntimeError(f"Negative {FILTER_FREQUENCY}: {self.frequency}")

        @staticmethod
        def md5_hashcode(b: bytes) -> int:
            import hashlib
            h = int.from_bytes(hashlib.md5(b).digest()[:8], "big")
            return h - (1 << 64) if h & (1 << 63) else h

        def accept(self, key):
            from ..io.writable import BytesWritable
            if isinstance(key, Text):
                b = key.bytes
            elif isinstance(key, BytesWritable):
                b = key.get()
            else:
                b = str(key).encode("utf-8")
            h = self.md5_hashcode(bytes(b))
            # Java's h / f * f == h: integer division truncates toward zero
            q = abs(h) // self.frequency * (1 if h >= 0 else -1)
            return q * self.frequency == h

    @staticmethod
    def setFilterClass(conf, cls):  # noqa: N802
        from ..utils.reflection import class_name
        conf.set(FILTER_CLASS, class_name(cls))

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        from ..utils.reflection import new_instance
        rr = SequenceFileRecordReader(job, split)
        flt = new_instance(job.get_class(FILTER_CLASS, SequenceFileInputFilter.PercentFilter),
                           job)

        class _Filtered(RecordReader):
            def next(self_inner):
                while True:
                    kv = rr.next()
                    if kv is None or flt.accept(kv[0]):
                        return kv

            def getProgress(self_inner):  # noqa: N802
                return rr.getProgress()

            def getPos(self_inner):  # noqa: N802
                return rr.getPos()

            def close(self_inner):
                rr.close()

        return _Filtered()


# --------------------------------------------------------------------------- outputs
def get_task_output_path(job, name: str) -> str:
    """Where a task attempt writes: the committer's work dir if set."""
    work = job.get("mapred.work.output.dir") or get_output_path(job)
    return os.path.join(work, name)


class FileOutputFormat(OutputFormat):
    setOutputPath = staticmethod(set_output_path)  # noqa: N815
    getOutputPath = staticmethod(get_output_path)  # noqa: N815

    def checkOutputSpecs(self, fs, job):  # noqa: N802
        out = get_output_path(job)
        if out is None and job.get_num_reduce_tasks() != 0:
            raise ValueError("Output directory not set in JobConf.")
        if out is not None and F.exists(out) and F.listdir(out):
            raise FileExistsError(f"Output directory {out} already exists")

    @staticmethod
    def get_compress_output(job):
        return job.get_boolean("mapred.output.compress", False)

    @staticmethod
    def set_compress_output(job, b):
        job.set_boolean("mapred.output.compress", b)


class _TextRecordWriter(RecordWriter):
    def __init__(self, f, sep=b"\t", codec=None):
        self.f = f
        self.sep = sep
        self.codec = codec
        self.buf = io.BytesIO() if codec else None

    @staticmethod
    def _b(x):
        if x is None or isinstance(x, NullWritable):
            return None
        if isinstance(x, Text):
            return x.bytes
        if isinstance(x, (bytes, bytearray)):
            return bytes(x)
        return str(x).encode("utf-8")

    def write(self, key, value):
        k, v = self._b(key), self._b(value)
        out = self.buf if self.buf is not None else self.f
        if k is None and v is None:
            return
        if k is None:
            out.write(v + b"\n")
        elif v is None:
            out.write(k + b"\n")
        else:
            out.write(k + self.sep + v + b"\n")

    def close(self, reporter=None):
        if self.buf is not None:
            self.f.write(self.codec.compress(self.buf.getvalue()))
        self.f.close()


class TextOutputFormat(FileOutputFormat):
    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        sep = job.get("mapred.textoutputformat.separator", "\t").encode()
        codec = None
        path = get_task_output_path(job, name)
        if self.get_compress_output(job):
            codec = get_codec(job.get("mapred.output.compression.codec",
                                      "org.apache.hadoop.io.compress.DefaultCodec"))
            path += codec.getDefaultExtension()
        F.makedirs(os.path.dirname(path))
        return _TextRecordWriter(F.fopen(path, "wb"), sep, codec)


class _SeqRecordWriter(RecordWriter):
    def __init__(self, w):
        self.w = w

    def write(self, key, value):
        self.w.append(key, value)

    def close(self, reporter=None):
        self.w.close()


class SequenceFileOutputFormat(FileOutputFormat):
    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        path = get_task_output_path(job, name)
        comp = seqf.NONE
        codec = None
        if self.get_compress_output(job):
            comp = job.get("mapred.output.compression.type", "RECORD").upper()
            codec = job.get("mapred.output.compression.codec",
                            "org.apache.hadoop.io.compress.DefaultCodec")
        w = seqf.Writer(path, job.get_output_key_class(), job.get_output_value_class(), comp, codec)
        return _SeqRecordWriter(w)

    @staticmethod
    def get_readers(path):
        files = sorted(p for p in F.listdir(path) if p.startswith("part-"))
        return [seqf.Reader(os.path.join(path, p)) for p in files]


SEQBINARY_KEY_CLASS = "mapred.seqbinary.output.key.class"
SEQBINARY_VALUE_CLASS = "mapred.seqbinary.output.value.class"


class _RawSeqWriter(RecordWriter):
    def __init__(self, w):
        self.w = w

    def write(self, key, value):
        # BytesWritable payloads go into the file as the record's key/value bytes
        self.w.append_raw(bytes(key.get()), bytes(value.get()))

    def close(self, reporter=None):
        self.w.close()


class SequenceFileAsBinaryOutputFormat(SequenceFileOutputFormat):
    """Writes BytesWritable keys/values as the raw record bytes of a
    SequenceFile whose header names the real classes
    (``mapred.seqbinary.output.{key,value}.class``, default the job's output
    classes) — SequenceFileAsBinaryOutputFormat.java; the output of
    SequenceFileAsBinaryInputFormat round-trips unchanged."""

    @staticmethod
    def setSequenceFileOutputKeyClass(conf, cls):  # noqa: N802
        conf.set_class(SEQBINARY_KEY_CLASS, cls)

    @staticmethod
    def setSequenceFileOutputValueClass(conf, cls):  # noqa: N802
        conf.set_class(SEQBINARY_VALUE_CLASS, cls)

    @staticmethod
    def getSequenceFileOutputKeyClass(conf):  # noqa: N802
        return conf.get(SEQBINARY_KEY_CLASS) or conf.get_output_key_class()

    @staticmethod
    def getSequenceFileOutputValueClass(conf):  # noqa: N802
        return conf.get(SEQBINARY_VALUE_CLASS) or conf.get_output_value_class()

    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        path = get_task_output_path(job, name)
        comp, codec = seqf.NONE, None
        if self.get_compress_output(job):
            comp = job.get("mapred.output.compression.type", "RECORD").upper()
            codec = job.get("mapred.output.compression.codec",
                            "org.apache.hadoop.io.compress.DefaultCodec")
        w = seqf.Writer(path, self.getSequenceFileOutputKeyClass(job),
                        self.getSequenceFileOutputValueClass(job), comp, codec)
        return _RawSeqWriter(w)

    def checkOutputSpecs(self, fs, job):  # noqa: N802
        super().checkOutputSpecs(fs, job)
        if self.get_compress_output(job) and \
                job.get("mapred.output.compression.type", "RECORD").upper() == seqf.RECORD:
            raise ValueError("SequenceFileAsBinaryOutputFormat doesn't support Record "
                             "Compression")


class MapFileOutputFormat(FileOutputFormat):
    """Reduce output as one MapFile per partition (MapFileOutputFormat.java):
    reduce keys arrive sorted, so each part-NNNNN is a directly indexable map;
    ``get_entry`` routes a lookup to the right part with the job's partitioner."""

    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        from ..io.mapfile import MapFile
        path = get_task_output_path(job, name)
        comp = seqf.NONE
        codec = None
        if self.get_compress_output(job):
            comp = job.get("mapred.output.compression.type", "RECORD").upper()
            codec = job.get("mapred.output.compression.codec",
                            "org.apache.hadoop.io.compress.DefaultCodec")
        w = MapFile.Writer(path, job.get_output_key_class(), job.get_output_value_class(),
                           comp, codec, conf=job)
        return _SeqRecordWriter(w)

    @staticmethod
    def get_readers(path, conf=None):
        from ..io.mapfile import MapFile
        parts = sorted(p for p in os.listdir(path) if p.startswith("part-"))
        return [MapFile.Reader(os.path.join(path, p), conf) for p in parts]

    getReaders = get_readers  # noqa: N815

    @staticmethod
    def get_entry(readers, partitioner, key, value=None):
        part = partitioner.getPartition(key, value, len(readers))
        return readers[part].get(key, value)

    getEntry = get_entry  # noqa: N815


class NullOutputFormat(OutputFormat):
    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        class _Null(RecordWriter):
            def write(self, k, v):
                pass
        return _Null()


class _CollectingWriter(RecordWriter):
    def __init__(self, sink):
        self.sink = sink

    def write(self, key, value):
        self.sink.append((key, value))


class MemoryOutputFormat(OutputFormat):
    """Keeps reduce output in memory (hbmr extension, used by iterative drivers
    such as K-Means so centroids never round-trip through files)."""
    _sinks: dict = {}

    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        key = job.get("hbmr.memory.output.id", "default")
        sink = MemoryOutputFormat._sinks.setdefault(key, [])
        return _CollectingWriter(sink)

    @classmethod
    def take(cls, key="default"):
        return cls._sinks.pop(key, [])


def writable_bytes(x) -> bytes:
    return x.serialize() if isinstance(x, Writable) else bytes(x)
