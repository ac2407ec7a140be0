"""Core I/O: VInt codec, Writables, SequenceFile, IFile, Configuration."""
import io
import os
import struct

import numpy as np
import pytest

from hbmr.conf.configuration import Configuration
from hbmr.io import sequencefile as seqf
from hbmr.io.ifile import IFileWriter, SpillRecord, read_segment
from hbmr.io.vint import decode_vlong, encode_vlong, read_vlong
from hbmr.io.writable import (BytesWritable, DoubleWritable, FloatVectorWritable, IntWritable,
                              LongWritable, NullWritable, Text, hash_bytes)
from hbmr.mapred.jobconf import JobConf


# Golden encodings from WritableUtils.writeVLong (hadoop-1.0.3/src/core/org/apache/
# hadoop/io/WritableUtils.java) — computed by hand from the algorithm.
GOLDEN = {
    0: b"\x00", 1: b"\x01", 127: b"\x7f", -112: b"\x90", -113: b"\x87\x70",
    128: b"\x8f\x80", 255: b"\x8f\xff", 256: b"\x8e\x01\x00", -1: b"\xff",
    -129: b"\x87\x80", 2**31 - 1: b"\x8c\x7f\xff\xff\xff", -2**31: b"\x84\x7f\xff\xff\xff",
    2**63 - 1: b"\x88\x7f\xff\xff\xff\xff\xff\xff\xff",
}


@pytest.mark.parametrize("v,enc", list(GOLDEN.items()))
def test_vlong_golden(v, enc):
    assert encode_vlong(v) == enc
    assert decode_vlong(enc) == (v, len(enc))
    assert read_vlong(io.BytesIO(enc)) == v


def test_vlong_roundtrip_random():
    rng = np.random.default_rng(0)
    for v in list(rng.integers(-2**62, 2**62, 2000)) + list(range(-300, 300)):
        v = int(v)
        e = encode_vlong(v)
        assert decode_vlong(e)[0] == v


def test_text_hash_and_order():
    # Java: "hello".getBytes() hashed by WritableComparator.hashBytes
    h = 1
    for b in b"hello":
        h = (31 * h + b) & 0xFFFFFFFF
    h = h - (1 << 32) if h >= 1 << 31 else h
    assert Text("hello").hash_code() == h == hash_bytes(b"hello")
    assert Text("abc") < Text("abd") < Text("b")
    assert Text("é").serialize() == b"\x02\xc3\xa9"
    assert IntWritable(-5) < IntWritable(3)
    assert LongWritable(2**40).hash_code() == (2**40 ^ (2**40 >> 32)) & 0x7FFFFFFF


def test_writable_roundtrip():
    for w in [Text("x y"), IntWritable(-7), LongWritable(1 << 50), DoubleWritable(1.25),
              BytesWritable(b"\x00\x01"), FloatVectorWritable([1.5, -2.0, 3.25])]:
        back = type(w).deserialize(w.serialize())
        assert back.serialize() == w.serialize()
    assert NullWritable().serialize() == b""


@pytest.mark.parametrize("comp", [seqf.NONE, seqf.RECORD, seqf.BLOCK])
def test_sequencefile_roundtrip(tmp_path, comp):
    p = tmp_path / "f.seq"
    n = 3000
    with seqf.Writer(p, Text, IntWritable, compression=comp, metadata={"a": "b"},
                     block_size=4096) as w:
        for i in range(n):
            w.append(Text(f"key-{i:05d}"), IntWritable(i))
    raw = open(p, "rb").read()
    assert raw[:4] == b"SEQ\x06"
    r = seqf.Reader(p)
    assert r.key_class_name == "org.apache.hadoop.io.Text"
    assert r.value_class_name == "org.apache.hadoop.io.IntWritable"
    assert r.metadata == {"a": "b"}
    assert r.compression == comp
    got = [(str(k), v.get()) for k, v in r]
    assert got == [(f"key-{i:05d}", i) for i in range(n)]


@pytest.mark.parametrize("comp", [seqf.NONE, seqf.BLOCK])
def test_sequencefile_splits_cover_exactly_once(tmp_path, comp):
    from hbmr.mapred.formats import FileSplit, SequenceFileRecordReader
    p = tmp_path / "f.seq"
    n = 5000
    with seqf.Writer(p, LongWritable, Text, compression=comp, block_size=2000) as w:
        for i in range(n):
            w.append(LongWritable(i), Text("v" * (i % 17)))
    size = os.path.getsize(p)
    job = JobConf()
    for nsplits in (1, 3, 7, 20):
        step = size // nsplits + 1
        seen = []
        for s in range(0, size, step):
            rr = SequenceFileRecordReader(job, FileSplit(str(p), s, min(step, size - s)))
            seen += [k.get() for k, _ in rr]
            rr.close()
        assert seen == list(range(n)), nsplits


def test_ifile_and_spill_index(tmp_path):
    p = tmp_path / "file.out"
    rec = SpillRecord(3)
    with open(p, "wb") as f:
        for part in range(3):
            w = IFileWriter(f)
            for i in range(part * 10):
                w.append(f"k{i}".encode(), f"v{part}".encode())
            rec.put(part, *w.close())
    rec.write(str(p) + ".index")
    rec2 = SpillRecord.read(str(p) + ".index")
    assert rec2.entries == rec.entries
    data = open(p, "rb").read()
    for part in range(3):
        s, raw, plen = rec2.get(part)
        kv = read_segment(data[s:s + plen])
        assert len(kv) == part * 10
        assert all(v == f"v{part}".encode() for _, v in kv)
    # corrupt a byte -> checksum error
    s, raw, plen = rec2.get(2)
    bad = bytearray(data[s:s + plen])
    bad[3] ^= 0xFF
    with pytest.raises(IOError):
        read_segment(bytes(bad))


def test_configuration_layering(tmp_path, monkeypatch):
    site = tmp_path / "core-site.xml"
    site.write_text("""<configuration>
      <property><name>a.b</name><value>site</value><final>true</final></property>
      <property><name>x.dir</name><value>${hadoop.tmp.dir}/x</value></property>
    </configuration>""")
    extra = tmp_path / "extra.xml"
    extra.write_text("<configuration><property><name>a.b</name><value>extra</value></property>"
                     "<property><name>c</name><value>7</value></property></configuration>")
    monkeypatch.setenv("HBMR_CONF_DIR", str(tmp_path))
    monkeypatch.setenv("USER", "tester")
    conf = Configuration()
    assert conf.get("a.b") == "site"
    conf.add_resource(str(extra))
    assert conf.get("a.b") == "site"   # final wins over later resources
    assert conf.get_int("c") == 7
    assert conf.get("x.dir") == "/tmp/hbmr-tester/x"
    conf.set("c", 9)
    assert conf.get_int("c") == 9
    buf = io.StringIO()
    conf.write_xml(buf)
    assert "<name>c</name>" in buf.getvalue()


def test_configuration_default_snapshot_tracks_site_files(tmp_path, monkeypatch):
    """New Configurations copy a cached layering of the default resources;
    editing (or adding) a site file in the conf dir invalidates it."""
    import os
    monkeypatch.setenv("HBMR_CONF_DIR", str(tmp_path))
    assert Configuration().get("snap.k") is None
    site = tmp_path / "core-site.xml"
    site.write_text("<configuration><property><name>snap.k</name><value>1</value>"
                    "</property></configuration>")
    assert Configuration().get("snap.k") == "1"
    a = Configuration()
    a.set("snap.k", "local")            # a copy, not the shared snapshot
    assert Configuration().get("snap.k") == "1"
    site.write_text("<configuration><property><name>snap.k</name><value>2</value>"
                    "</property></configuration>")
    st = os.stat(site)
    os.utime(site, ns=(st.st_atime_ns, st.st_mtime_ns + 1_000_000))
    assert Configuration().get("snap.k") == "2"
    monkeypatch.delenv("HBMR_CONF_DIR")
    assert Configuration().get("snap.k") is None


def test_jobconf_gpu_keys_and_typo_alias():
    job = JobConf()
    assert job.get_int("mapred.tasktracker.map.gpu.tasks.maximum") == 0
    assert job.get_int("mapred.tasktracker.map.cpu.tasks.maximum") == 2
    # the reference's getter read a misspelled key: both spellings alias
    job.set("mapred.map.runnner.gpu.class", "hbmr.mapred.maprunner:MapRunner")
    from hbmr.mapred.maprunner import MapRunner
    assert job.get_gpu_map_runner_class() is MapRunner
    job.set_gpu_executable("/bin/gpu")
    assert job.getGPUExecutable() == "/bin/gpu" and job.is_gpu_capable()


@pytest.mark.parametrize("comp", [seqf.NONE, seqf.BLOCK])
def test_sequencefile_sorter_multi_run(tmp_path, comp):
    """SequenceFile.Sorter (SequenceFile.java:2269): many inputs, a memory
    budget that forces several runs and a factor that forces merge passes;
    the output is sorted by the key comparator and stable for equal keys."""
    rng = np.random.default_rng(3)
    ins, recs = [], []
    for f in range(4):
        p = tmp_path / f"in{f}.seq"
        with seqf.Writer(p, IntWritable, Text, compression=comp, block_size=1500) as w:
            for i in range(700):
                k = int(rng.integers(-50, 50))
                w.append(IntWritable(k), Text(f"{f}-{i}"))
                recs.append((k, f"{f}-{i}"))
        ins.append(p)
    conf = Configuration()
    conf.set("hbmr.io.sort.bytes", "4000")
    conf.set("io.sort.factor", "3")
    s = seqf.Sorter(IntWritable, Text, conf)
    out = tmp_path / "sorted.seq"
    assert s.sort(ins, out) == len(recs)
    assert s.runs_written > 3 and s.merge_passes >= 2
    got = [(k.get(), str(v)) for k, v in seqf.Reader(out)]
    assert got == sorted(recs, key=lambda r: r[0])          # Python sort is stable
    assert not (tmp_path / "sorted.seq.sort-tmp").exists()
    assert all(p.exists() for p in ins)


def test_sequencefile_sorter_text_and_merge(tmp_path):
    """Text keys order by raw bytes (Text.Comparator); merge of sorted files."""
    words = ["pear", "apple", "Zeta", "apricot", "", "é", "b", "apple"]
    parts = []
    for j in range(3):
        p = tmp_path / f"s{j}.seq"
        ws = sorted((w + str(j) for w in words), key=lambda s: s.encode())
        with seqf.Writer(p, Text, IntWritable) as w:
            for i, x in enumerate(ws):
                w.append(Text(x), IntWritable(j))
        parts.append(p)
    out = tmp_path / "m.seq"
    s = seqf.Sorter(Text, IntWritable)
    n = s.merge(parts, out)
    assert n == 3 * len(words)
    got = [str(k) for k, _ in seqf.Reader(out)]
    assert got == sorted((w + str(j) for j in range(3) for w in words), key=lambda s: s.encode())
    # sort with delete_input removes the inputs
    out2 = tmp_path / "m2.seq"
    assert seqf.Sorter(Text, IntWritable).sort(parts, out2, delete_input=True) == n
    assert [str(k) for k, _ in seqf.Reader(out2)] == got
    assert not any(p.exists() for p in parts)
