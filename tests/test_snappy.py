"""SnappyCodec (native/io/snappy.cc): raw Snappy against an independent
decoder written here from the format, hand-built streams for every element
form, malformed input, Hadoop's BlockCompressorStream framing
(SnappyCodec.java:95-110, BlockCompressorStream.java:76-153), SequenceFile
RECORD/BLOCK files and a job with Snappy map output and text output
(TestCodec.java's codec round trips over SequenceFiles).  No libsnappy in the
image: byte-level parity with Google's compressor is unpinned (its match
choices are an implementation detail); the decoder side is pinned by the
hand-built streams and the Python decoder."""
import collections
import os
import struct

import numpy as np
import pytest

from hbmr.io import compress as C
from hbmr.io import sequencefile as seqf
from hbmr.io import snappy as S
from hbmr.io.writable import BytesWritable, Text
from hbmr.mapred import JobClient
from hbmr.models import wordcount


def py_decode(buf: bytes) -> bytes:
    """Snappy format decoder, written independently of the C++ one."""
    n = shift = i = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if b < 0x80:
            break
    out = bytearray()
    while i < len(buf):
        tag = buf[i]
        i += 1
        t = tag & 3
        if t == 0:
            ln = tag >> 2
            if ln >= 60:
                k = ln - 59
                ln = int.from_bytes(buf[i:i + k], "little")
                i += k
            ln += 1
            out += buf[i:i + ln]
            i += ln
            continue
        if t == 1:
            ln, off = 4 + ((tag >> 2) & 7), ((tag >> 5) << 8) | buf[i]
            i += 1
        elif t == 2:
            ln, off = 1 + (tag >> 2), int.from_bytes(buf[i:i + 2], "little")
            i += 2
        else:
            ln, off = 1 + (tag >> 2), int.from_bytes(buf[i:i + 4], "little")
            i += 4
        assert 0 < off <= len(out)
        for _ in range(ln):
            out.append(out[-off])
    assert len(out) == n
    return bytes(out)


def _inputs():
    rng = np.random.default_rng(0)
    text = open(C.__file__, "rb").read()
    words = b" ".join(rng.choice([b"map", b"reduce", b"shuffle", b"gpu", b"hadoop"], 40000))
    return {
        "empty": b"", "one": b"x", "short": b"abcabcabcabcab", "zeros": bytes(200_000),
        "random": rng.integers(0, 256, 150_000, dtype=np.uint8).tobytes(),
        "text": text * 20, "words": words,
        "periodic": bytes(range(7)) * 30_000,
        "mixed": rng.integers(0, 4, 90_000, dtype=np.uint8).tobytes() + text,
    }


@pytest.mark.parametrize("name", list(_inputs()))
def test_raw_roundtrip_and_independent_decoder(name):
    d = _inputs()[name]
    c = S.compress(d)
    assert S.decompress(c) == d
    assert py_decode(c) == d
    assert len(c) <= 32 + len(d) + len(d) // 6
    if name in ("zeros", "periodic", "words", "text"):
        assert len(c) < len(d) // 3, (name, len(c), len(d))


def _varint(n):
    out = bytearray()
    while n >= 0x80:
        out.append(n & 0x7F | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def test_hand_built_streams_every_element_form():
    lit = bytes(range(256)) * 4
    cases = []
    # short literal, copy-1 (len 4..11, 11-bit offset), overlapping run
    cases.append((_varint(17) + bytes([(3 - 1) << 2]) + b"abc" + bytes([1 | (6 << 2), 3]) +
                  bytes([1 | (0 << 2), 1]), b"abc" + b"abcabcabca" + b"aaaa"))
    # literal with 1..4 length bytes (tags 60..63)
    for k in (1, 2, 3, 4):
        ln = 61 if k == 1 else 300
        s = lit[:ln]
        cases.append((_varint(ln) + bytes([(59 + k) << 2]) + (ln - 1).to_bytes(k, "little") + s, s))
    # copy-2 (len 1..64, 16-bit offset) and copy-4 (32-bit offset)
    body = lit[:1000]
    want = body + body[300:364] + body[0:5]
    s = (_varint(len(want)) + bytes([61 << 2]) + (999).to_bytes(2, "little") + body +
         bytes([2 | (63 << 2)]) + (700).to_bytes(2, "little") +
         bytes([3 | (4 << 2)]) + (1064).to_bytes(4, "little"))
    cases.append((s, want))
    for stream, expect in cases:
        assert py_decode(stream) == expect
        assert S.decompress(stream) == expect


@pytest.mark.parametrize("bad", [
    _varint(5) + bytes([4 << 2]) + b"abc",             # literal runs past the end
    _varint(4) + bytes([0]) + b"a" + bytes([1, 0]),     # offset 0
    _varint(9) + bytes([0]) + b"a" + bytes([1 | (4 << 2), 2]),  # offset beyond output
    _varint(3) + bytes([8]) + b"abc",                   # well formed (control)
    _varint(10) + bytes([8]) + b"abc",                  # stream shorter than its preamble
    _varint(2) + bytes([8]) + b"abc",                   # output overrun
    bytes([0x80, 0x80, 0x80, 0x80, 0x80]),              # bad varint
    _varint(8) + bytes([2 | (7 << 2), 1]),              # truncated copy-2
])
def test_malformed_raw_streams_are_rejected(bad):
    if bad == _varint(3) + bytes([8]) + b"abc":
        assert S.decompress(bad) == b"abc"
        return
    with pytest.raises(IOError):
        S.decompress(bad)


def _blocks(framed):
    """Parse BlockCompressorStream framing: [(orig, [chunk bytes...])...]."""
    out, i = [], 0
    while i < len(framed):
        orig = struct.unpack(">i", framed[i:i + 4])[0]
        i += 4
        chunks, got = [], 0
        while got < orig:
            ln = struct.unpack(">i", framed[i:i + 4])[0]
            i += 4
            chunks.append(framed[i:i + ln])
            got += len(py_decode(framed[i:i + ln]))
            i += ln
        out.append((orig, chunks))
    return out


def test_hadoop_block_framing():
    bs = S.BUFFER_SIZE_DEFAULT
    max_in = bs - (bs // 6 + 32)
    assert max_in == 218422
    for d in (b"", b"hello hadoop", bytes(max_in), bytes(max_in + 1),
              np.random.default_rng(1).integers(0, 9, 3 * max_in + 17, dtype=np.uint8).tobytes()):
        f = S.hadoop_compress(d)
        blocks = _blocks(f)
        assert len(blocks) == 1 and blocks[0][0] == len(d)
        chunks = blocks[0][1]
        assert len(chunks) == -(-len(d) // max_in)
        dec = b"".join(py_decode(c) for c in chunks)
        assert dec == d and all(len(py_decode(c)) <= max_in for c in chunks)
        assert S.hadoop_decompress(f) == d
    assert S.hadoop_compress(b"") == b"\x00\x00\x00\x00"
    # a stream of several write()+finish() blocks decodes to their concatenation
    a, b = b"first block " * 100, b"second" * 7
    assert S.hadoop_decompress(S.hadoop_compress(a) + S.hadoop_compress(b)) == a + b
    # a small buffer size splits into more chunks
    small = S.hadoop_compress(bytes(10_000), buffer_size=1024)
    assert len(_blocks(small)[0][1]) == -(-10_000 // (1024 - (1024 // 6 + 32)))
    for cut in (3, 6, len(small) - 1):
        with pytest.raises(IOError):
            S.hadoop_decompress(small[:cut])


def test_codec_names_and_factory():
    c = C.get_codec("org.apache.hadoop.io.compress.SnappyCodec")
    assert isinstance(c, C.SnappyCodec) and c.getDefaultExtension() == ".snappy"
    assert isinstance(C.get_codec("snappy"), C.SnappyCodec)
    assert isinstance(C.codec_for_path("/x/part-00000.snappy"), C.SnappyCodec)
    from hbmr.mapred.jobconf import JobConf
    conf = JobConf()
    conf.set_int(S.BUFFER_SIZE_KEY, 4096)
    assert C.SnappyCodec(conf=conf).buffer_size == 4096


@pytest.mark.parametrize("comp", [seqf.RECORD, seqf.BLOCK])
def test_sequencefile_snappy_roundtrip(tmp_path, comp):
    p = tmp_path / "f.seq"
    rng = np.random.default_rng(2)
    toks = [b"map ", b"reduce ", b"split ", b"gpu "]
    vals = [b"".join(rng.choice(toks, int(rng.integers(0, 600)))) for _ in range(400)]
    with seqf.Writer(p, Text, BytesWritable, compression=comp, codec="snappy",
                     block_size=20_000) as w:
        for i, v in enumerate(vals):
            w.append(Text(f"k{i:04d}"), BytesWritable(v))
    raw = open(p, "rb").read()
    assert b"org.apache.hadoop.io.compress.SnappyCodec" in raw[:200]
    assert len(raw) < sum(map(len, vals)) // 2
    r = seqf.Reader(p)
    assert r.compression == comp and isinstance(r.codec, C.SnappyCodec)
    got = [(str(k), bytes(v.get() if hasattr(v, "get") else v.value)) for k, v in r]
    assert got == [(f"k{i:04d}", v) for i, v in enumerate(vals)]


def test_job_with_snappy_map_output_and_text_output(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    words = ["alpha", "beta", "gamma", "delta"]
    rng = np.random.default_rng(4)
    lines = [" ".join(rng.choice(words, 9)) for _ in range(3000)]
    (inp / "a.txt").write_text("\n".join(lines) + "\n")
    out = tmp_path / "out"
    job = wordcount.make_job(str(inp), str(out), reduces=2)
    job.set_boolean("mapred.compress.map.output", True)
    job.set("mapred.map.output.compression.codec", "org.apache.hadoop.io.compress.SnappyCodec")
    job.set_boolean("mapred.output.compress", True)
    job.set("mapred.output.compression.codec", "org.apache.hadoop.io.compress.SnappyCodec")
    rj = JobClient.runJob(job, verbose=False)
    assert rj.isSuccessful()
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert parts and all(f.endswith(".snappy") for f in parts)
    got = collections.Counter()
    for f in parts:
        for ln in S.hadoop_decompress((out / f).read_bytes()).decode().splitlines():
            w, n = ln.split("\t")
            got[w] += int(n)
    assert got == collections.Counter(" ".join(lines).split())


def test_mutated_streams_never_crash():
    """Bit flips, truncations and spliced lengths of valid streams: the
    decoders either raise IOError or return bytes (never read/write out of
    bounds — a crash would take the test process down)."""
    rng = np.random.default_rng(7)
    base = [S.compress(d) for d in _inputs().values() if d]
    framed = [S.hadoop_compress(d, buffer_size=2048) for d in (b"abc" * 999, bytes(5000))]
    for _ in range(3000):
        src = base[int(rng.integers(len(base)))]
        b = bytearray(src[:int(rng.integers(1, len(src) + 1))])
        for _ in range(int(rng.integers(0, 4))):
            b[int(rng.integers(len(b)))] = int(rng.integers(256))
        try:
            S.decompress(bytes(b))
        except IOError:
            pass
    for _ in range(500):
        src = framed[int(rng.integers(len(framed)))]
        b = bytearray(src)
        b[int(rng.integers(len(b)))] = int(rng.integers(256))
        try:
            S.hadoop_decompress(bytes(b))
        except IOError:
            pass
