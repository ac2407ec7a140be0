"""Compression codecs named like Hadoop's (org.apache.hadoop.io.compress.*).

DefaultCodec = zlib stream (ZlibCompressor with header), GzipCodec = gzip
member, BZip2Codec = bzip2 stream, SnappyCodec = Hadoop block framing of raw
Snappy (SnappyCodec.java).  (Hadoop's JNI zlib/snappy live in libhadoop.so:
src/native/src/org/apache/hadoop/io/compress/{zlib,snappy}/*.c; Python's
zlib/bz2 wrap the same C libraries; Snappy is native/io/snappy.cc since the
image has no libsnappy.)
"""
from __future__ import annotations

import bz2
import gzip
import zlib


class CompressionCodec:
    JAVA_NAME = ""
    EXT = ""

    def compress(self, data: bytes) -> bytes:
        raise NotImplementedError

    def decompress(self, data: bytes) -> bytes:
        raise NotImplementedError

    def getDefaultExtension(self):  # noqa: N802
        return self.EXT


class DefaultCodec(CompressionCodec):
    JAVA_NAME = "org.apache.hadoop.io.compress.DefaultCodec"
    EXT = ".deflate"

    def __init__(self, level: int = 6):
        self.level = level

    def compress(self, data):
        return zlib.compress(data, self.level)

    def decompress(self, data):
        return zlib.decompress(data)


class GzipCodec(CompressionCodec):
    JAVA_NAME = "org.apache.hadoop.io.compress.GzipCodec"
    EXT = ".gz"

    def compress(self, data):
        return gzip.compress(data, mtime=0)

    def decompress(self, data):
        return gzip.decompress(data)


class BZip2Codec(CompressionCodec):
    JAVA_NAME = "org.apache.hadoop.io.compress.BZip2Codec"
    EXT = ".bz2"

    def compress(self, data):
        return bz2.compress(data)

    def decompress(self, data):
        return bz2.decompress(data)


class SnappyCodec(CompressionCodec):
    """Each compress() is one BlockCompressorStream write + finish: a block of
    [int uncompressed length][int chunk length][snappy]… with chunks of at most
    bufferSize - (bufferSize/6 + 32) input bytes (SnappyCodec.java:95-110);
    decompress() reads any sequence of such blocks."""
    JAVA_NAME = "org.apache.hadoop.io.compress.SnappyCodec"
    EXT = ".snappy"

    def __init__(self, buffer_size: int | None = None, conf=None):
        from . import snappy
        if buffer_size is None:
            buffer_size = (conf.get_int(snappy.BUFFER_SIZE_KEY, snappy.BUFFER_SIZE_DEFAULT)
                           if conf is not None else snappy.BUFFER_SIZE_DEFAULT)
        self.buffer_size = int(buffer_size)

    def compress(self, data):
        from . import snappy
        return snappy.hadoop_compress(data, self.buffer_size)

    def decompress(self, data):
        from . import snappy
        return snappy.hadoop_decompress(data)


_CODECS = {c.JAVA_NAME: c for c in (DefaultCodec, GzipCodec, BZip2Codec, SnappyCodec)}
_BY_NAME = {"default": DefaultCodec, "zlib": DefaultCodec, "deflate": DefaultCodec,
            "gzip": GzipCodec, "bzip2": BZip2Codec, "bz2": BZip2Codec, "snappy": SnappyCodec}


def get_codec(name_or_codec) -> CompressionCodec | None:
    if name_or_codec is None or isinstance(name_or_codec, CompressionCodec):
        return name_or_codec
    if isinstance(name_or_codec, type):
        return name_or_codec()
    cls = _CODECS.get(name_or_codec) or _BY_NAME.get(str(name_or_codec).lower())
    if cls is None:
        raise ValueError(f"unsupported codec {name_or_codec!r}")
    return cls()


def codec_for_path(path: str) -> CompressionCodec | None:
    """CompressionCodecFactory.getCodec: choose by file extension."""
    for cls in (GzipCodec, BZip2Codec, SnappyCodec, DefaultCodec):
        if str(path).endswith(cls.EXT):
            return cls()
    return None
