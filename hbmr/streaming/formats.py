"""Streaming input formats (hadoop-1.0.3 contrib/streaming:
StreamInputFormat.java, StreamBaseRecordReader.java,
StreamXmlRecordReader.java, AutoInputFormat.java).

* :class:`StreamInputFormat` — text input whose record reader is
  ``stream.recordreader.class`` (``-inputreader CLASS,k=v,...`` sets it and the
  ``stream.recordreader.<k>`` options); without one, plain lines
  (LineRecordReader).
* :class:`StreamXmlRecordReader` — ``-inputreader
  "StreamXmlRecord,begin=<tag>,end=</tag>"``: each record is the text from a
  ``stream.recordreader.begin`` match through the next
  ``stream.recordreader.end`` match (key = the record, value = empty).  A split
  owns the records that begin before its end; the last may run past it.
  ``stream.recordreader.slowmatch=true`` treats ``begin``/``end`` as regular
  expressions and ignores matches inside ``<![CDATA[ ... ]]>`` sections;
  ``stream.recordreader.maxrec`` caps a record (default 50,000 bytes: a
  longer one is truncated there, as the reference's lookahead buffer does).
* :class:`AutoInputFormat` — per file: SequenceFile (header ``SEQ``) records
  as they are, anything else as text lines (LongWritable offset, Text line).
"""
from __future__ import annotations

import re

from .. import fs as F
from ..io.writable import Text
from ..mapred.api import RecordReader
from ..mapred.formats import (FileInputFormat, LineRecordReader, SequenceFileRecordReader,
                              TextInputFormat)
from ..utils.reflection import load_class

_READER_ALIASES = {
    "StreamXmlRecordReader": "hbmr.streaming.formats:StreamXmlRecordReader",
    "StreamXmlRecord": "hbmr.streaming.formats:StreamXmlRecordReader",
    "org.apache.hadoop.streaming.StreamXmlRecordReader":
        "hbmr.streaming.formats:StreamXmlRecordReader",
}


def reader_class(name: str):
    return load_class(_READER_ALIASES.get(name, name))


class StreamXmlRecordReader(RecordReader):
    CHUNK = 1 << 20

    def __init__(self, job, split):
        self.start = split.start
        self.end = split.start + split.length
        g = lambda k, d=None: job.get(f"stream.recordreader.{k}", d)  # noqa: E731
        begin, end = g("begin"), g("end")
        if not begin or not end:
            raise ValueError("StreamXmlRecordReader needs stream.recordreader.begin and .end "
                             "(-inputreader \"StreamXmlRecord,begin=<tag>,end=</tag>\")")
        self.slow = (g("slowmatch", "false") or "false").lower() == "true"
        self.maxrec = int(g("maxrec", "50000"))
        if self.slow:
            self.begin_re = re.compile(begin.encode())
            self.end_re = re.compile(end.encode())
        else:
            self.begin_b, self.end_b = begin.encode(), end.encode()
        with F.fopen(split.path, "rb") as f:
            # the split plus a record's worth past its end (a record that begins
            # inside the split is read to its end tag)
            f.seek(self.start)
            self.buf = f.read(split.length + self.maxrec + len(end.encode()) + 16)
        self.pos = 0            # offset into buf
        self.limit = split.length

    # begin / end searches; the slow form skips matches inside CDATA sections
    def _find(self, which, frm):
        if not self.slow:
            pat = self.begin_b if which == "begin" else self.end_b
            i = self.buf.find(pat, frm)
            return (i, i + len(pat)) if i >= 0 else (-1, -1)
        rx = self.begin_re if which == "begin" else self.end_re
        cd = re.compile(rb"<!\[CDATA\[|\]\]>")
        pos = frm
        in_cdata = False
        while True:
            m = rx.search(self.buf, pos)
            c = cd.search(self.buf, pos)
            if m is None:
                return -1, -1
            if c is not None and c.start() <= m.start():
                in_cdata = c.group(0) == b"<![CDATA["
                pos = c.end()
                continue
            if in_cdata:
                pos = m.end()
                continue
            return m.start(), m.end()

    def next(self):
        if self.pos >= self.limit:
            return None
        b0, _ = self._find("begin", self.pos)
        if b0 < 0 or b0 >= self.limit:
            self.pos = self.limit
            return None
        _, e1 = self._find("end", b0 + 1)
        if e1 < 0:
            self.pos = self.limit
            return None
        rec = self.buf[b0:min(e1, b0 + self.maxrec)]
        self.pos = e1
        return Text(rec), Text(b"")

    def getProgress(self):  # noqa: N802
        return min(1.0, self.pos / max(1, self.limit))

    def close(self):
        self.buf = b""


class StreamInputFormat(TextInputFormat):
    """TextInputFormat, or the ``stream.recordreader.class`` reader."""

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        name = job.get("stream.recordreader.class")
        if not name:
            return LineRecordReader(job, split)
        return reader_class(name)(job, split)


def _is_sequence_file(path) -> bool:
    try:
        with F.fopen(path, "rb") as f:
            return f.read(3) == b"SEQ"
    except OSError:
        return False


class AutoInputFormat(FileInputFormat):
    """AutoInputFormat.java: SequenceFiles and text files in one input."""

    def is_splitable(self, fs, path) -> bool:
        return super().is_splitable(fs, path)

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        if _is_sequence_file(split.path):
            return SequenceFileRecordReader(job, split)
        return LineRecordReader(job, split)
