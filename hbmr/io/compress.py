"""Compression codecs named like Hadoop's (org.apache.hadoop.io.compress.*).

DefaultCodec = zlib stream (ZlibCompressor with header), GzipCodec = gzip
member, BZip2Codec = bzip2 stream.  (Hadoop's JNI zlib/snappy live in
libhadoop.so: src/native/src/org/apache/hadoop/io/compress/zlib/*.c; Python's
zlib/bz2 wrap the same C libraries.)  Snappy has no library in this image.
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


_CODECS = {c.JAVA_NAME: c for c in (DefaultCodec, GzipCodec, BZip2Codec)}
_BY_NAME = {"default": DefaultCodec, "zlib": DefaultCodec, "deflate": DefaultCodec,
            "gzip": GzipCodec, "bzip2": BZip2Codec, "bz2": BZip2Codec}


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
    for cls in (GzipCodec, BZip2Codec, DefaultCodec):
        if str(path).endswith(cls.EXT):
            return cls()
    return None
