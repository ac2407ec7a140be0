"""Streaming breadth (hadoop-1.0.3 contrib/streaming): output field separators
and key-field counts (PipeMapper.java:78-80, PipeReducer.java:75-77),
-inputreader StreamXmlRecord (StreamXmlRecordReader.java), -io typedbytes /
rawbytes (streaming/io/*, typedbytes/*), DumpTypedBytes / LoadTypedBytes,
AutoInputFormat, -reducer aggregate and -lazyOutput."""
import io
import os
import struct
import sys

import pytest

from hbmr import streaming, typedbytes as tb
from hbmr.io import sequencefile as seqf
from hbmr.io.writable import IntWritable, Text
from hbmr.mapred import JobClient
from hbmr.streaming import dumptb

PY = sys.executable
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    job = streaming.stream_job_conf(args)
    rj = JobClient.runJob(job, verbose=False)
    assert rj.isSuccessful(), rj.getFailureInfo() if hasattr(rj, "getFailureInfo") else ""
    return rj


def _lines(out):
    res = []
    for fn in sorted(os.listdir(out)):
        if fn.startswith("part-"):
            res += open(os.path.join(out, fn), encoding="utf-8").read().splitlines()
    return res


def _script(tmp_path, name, body):
    p = tmp_path / name
    p.write_text(f"import sys\nsys.path.insert(0, {ROOT!r})\n" + body)
    return f"{PY} {p}"


def test_typed_bytes_codec_roundtrip():
    vals = [0, -5, 2 ** 40, tb.Long(7), "héllo", 1.25, tb.Float(0.5), True, tb.Byte(-2),
            tb.Buffer(b"\x00\x01"), (1, "a"), [1, [2, 3]], {"k": 1, 2: "v"}]
    raw = b"".join(tb.dumps(v) for v in vals)
    got = list(tb.iter_values(io.BytesIO(raw)))
    assert got == vals
    assert [type(g) for g in got[:4]] == [int, int, tb.Long, tb.Long]
    # raw reads are value-exact, codes included (list = 9 ... 255 marker)
    tin = tb.TypedBytesInput(io.BytesIO(raw))
    assert b"".join(iter(tin.read_raw, None)) == raw
    assert tb.dumps([1])[0] == tb.LIST and tb.dumps([1])[-1] == tb.MARKER
    assert tb.dumps("ab") == b"\x07\x00\x00\x00\x02ab"


def test_output_field_separator_and_key_fields(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    (inp / "a").write_text("x\n")
    mapper = _script(tmp_path, "m.py", "for l in sys.stdin:\n"
                     "  print('a.b.c'); print('a.b.d'); print('q'); print('z.y.w')\n")
    out = tmp_path / "out"
    _run(["-input", str(inp), "-output", str(out), "-mapper", mapper,
          "-reducer", "hbmr.mapred.lib.basic:IdentityReducer", "-numReduceTasks", "1",
          "-D", "stream.map.output.field.separator=.",
          "-D", "stream.num.map.output.key.fields=2"])
    assert sorted(_lines(out)) == ["a.b\tc", "a.b\td", "q\t", "z.y\tw"]
    # the reduce side: a reducer that prints "k|v1|v2" with a 1-field '|' key
    red = _script(tmp_path, "r.py", "for l in sys.stdin:\n"
                  "  k, v = l.rstrip('\\n').split('\\t')\n  print(k + '|' + v + '|end')\n")
    out2 = tmp_path / "out2"
    _run(["-input", str(inp), "-output", str(out2), "-mapper", mapper, "-reducer", red,
          "-D", "stream.map.output.field.separator=.", "-D", "stream.num.map.output.key.fields=2",
          "-D", "stream.reduce.output.field.separator=|",
          "-D", "stream.num.reduce.output.key.fields=2"])
    assert sorted(_lines(out2)) == ["a.b|c\tend", "a.b|d\tend", "q|\tend", "z.y|w\tend"]


def test_split_key_value_rules():
    f = streaming.split_key_value
    assert [x.bytes for x in f(b"a\tb\tc", b"\t", 1)] == [b"a", b"b\tc"]
    assert [x.bytes for x in f(b"a\tb\tc", b"\t", 2)] == [b"a\tb", b"c"]
    assert [x.bytes for x in f(b"a\tb", b"\t", 3)] == [b"a\tb", b""]
    assert [x.bytes for x in f(b"k::v", b"::", 1)] == [b"k", b"v"]


def test_xml_input_reader(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    pages = [f"<page>\n  <title>t{i}</title>\n</page>" for i in range(40)]
    body = "<root>junk\n" + "\nbetween\n".join(pages) + "\ntail</root>\n"
    (inp / "x.xml").write_text(body)
    mapper = _script(tmp_path, "m.py", "d = sys.stdin.read()\n"
                     "print(d.count('<page>'), d.count('</page>'), d.count('junk'),"
                     " d.count('between'), d.count('<title>t'))\n")
    out = tmp_path / "out"
    _run(["-input", str(inp), "-output", str(out), "-mapper", mapper, "-reducer", "NONE",
          "-inputreader", "StreamXmlRecord,begin=<page>,end=</page>",
          "-D", "mapred.min.split.size=1", "-D", "mapred.map.tasks=3"])
    tot = [0] * 5
    for ln in _lines(out):
        for i, v in enumerate(ln.split()):
            tot[i] += int(v)
    assert tot == [40, 40, 0, 0, 40]   # every page exactly once, nothing between
    # slowmatch: an end tag inside CDATA does not end the record
    (inp / "x.xml").write_text("<page><![CDATA[ </page> ]]>body</page>\n<page>b</page>\n")
    out2 = tmp_path / "out2"
    mapper2 = _script(tmp_path, "m2.py", "d = sys.stdin.read()\nprint(d.count('body'),"
                      " d.count('<page>'))\n")
    _run(["-input", str(inp), "-output", str(out2), "-mapper", mapper2, "-reducer", "NONE",
          "-inputreader", "StreamXmlRecord,begin=<page>,end=</page>,slowmatch=true"])
    sums = [sum(int(ln.split()[i]) for ln in _lines(out2)) for i in range(2)]
    assert sums == [1, 2]


def test_typedbytes_io_wordcount(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    (inp / "a").write_text("x y x\ny z\n")
    mapper = _script(tmp_path, "m.py",
                     "from hbmr import typedbytes as tb\n"
                     "out = tb.TypedBytesOutput(sys.stdout.buffer)\n"
                     "vals = list(tb.iter_values(sys.stdin.buffer))\n"
                     "for k, line in zip(vals[::2], vals[1::2]):\n"
                     "    assert isinstance(k, tb.Long)\n"
                     "    for w in line.split():\n        out.write(w); out.write(1)\n")
    reducer = _script(tmp_path, "r.py",
                      "from hbmr import typedbytes as tb\n"
                      "out = tb.TypedBytesOutput(sys.stdout.buffer)\n"
                      "vals = list(tb.iter_values(sys.stdin.buffer))\nc = {}\n"
                      "for k, v in zip(vals[::2], vals[1::2]):\n    c[k] = c.get(k, 0) + v\n"
                      "for k in sorted(c):\n    out.write(k); out.write(tb.Long(c[k]))\n")
    out = tmp_path / "out"
    _run(["-input", str(inp), "-output", str(out), "-mapper", mapper, "-reducer", reducer,
          "-io", "typedbytes", "-inputformat", "SequenceFileInputFormat",
          "-D", "stream.map.input=typedbytes"] if False else
         ["-input", str(inp), "-output", str(out), "-mapper", mapper, "-reducer", reducer,
          "-io", "typedbytes", "-D", "stream.map.input.ignoreKey=false"])
    assert sorted(_lines(out)) == ["x\t2", "y\t2", "z\t1"]


def test_rawbytes_io(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    (inp / "a").write_text("p\nq\n")
    mapper = _script(tmp_path, "m.py",
                     "import struct\nb = sys.stdin.buffer.read()\ni = 0\n"
                     "o = sys.stdout.buffer\n"
                     "while i < len(b):\n"
                     "    n = struct.unpack('>i', b[i:i+4])[0]; v = b[i+4:i+4+n]; i += 4 + n\n"
                     "    o.write(struct.pack('>i', len(v)) + v + struct.pack('>i', 3) + b'\\x00\\xff\\n')\n")
    out = tmp_path / "out"
    _run(["-input", str(inp), "-output", str(out), "-mapper", mapper, "-reducer", "NONE",
          "-io", "rawbytes", "-outputformat", "SequenceFileOutputFormat"])
    got = []
    for fn in sorted(os.listdir(out)):
        if fn.startswith("part-"):
            for k, v in seqf.Reader(str(out / fn)):
                got.append((k.bytes, v.bytes))
    assert sorted(got) == [(b"p", b"\x00\xff\n"), (b"q", b"\x00\xff\n")]


def test_dump_and_load_typed_bytes(tmp_path):
    src = tmp_path / "src"
    src.mkdir()
    with seqf.Writer(str(src / "part-00000"), Text, IntWritable) as w:
        for i in range(5):
            w.append(Text(f"k{i}"), IntWritable(i * i))
    (src / "notes.txt").write_text("line one\nline two\n")
    buf = io.BytesIO()
    n = dumptb.dump_typed_bytes(str(src), buf)
    assert n == 7
    vals = list(tb.iter_values(io.BytesIO(buf.getvalue())))
    pairs = list(zip(vals[::2], vals[1::2]))
    assert ("k3", 9) in pairs and (0, "line one") in pairs
    dst = tmp_path / "tb.seq"
    assert dumptb.load_typed_bytes(str(dst), io.BytesIO(buf.getvalue())) == 7
    back = [(k.get_value(), v.get_value()) for k, v in seqf.Reader(str(dst))]
    assert back == pairs
    r = seqf.Reader(str(dst))
    assert r.key_class.JAVA_NAME == "org.apache.hadoop.typedbytes.TypedBytesWritable"


def test_auto_input_format(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    with seqf.Writer(str(inp / "s.seq"), Text, Text) as w:
        w.append(Text("sk"), Text("sv"))
    (inp / "t.txt").write_text("tline\n")
    out = tmp_path / "out"
    _run(["-input", str(inp), "-output", str(out), "-mapper", "cat", "-reducer", "NONE",
          "-inputformat", "AutoInputFormat"])
    got = sorted(_lines(out))
    assert got == ["0\ttline", "sk\tsv"]


def test_aggregate_reducer_and_lazy_output(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    (inp / "a").write_text("a b a\n")
    mapper = _script(tmp_path, "m.py", "for l in sys.stdin:\n"
                     "  [print('LongValueSum:' + w + '\\t1') for w in l.split()]\n")
    out = tmp_path / "out"
    _run(["-input", str(inp), "-output", str(out), "-mapper", mapper, "-reducer", "aggregate",
          "-numReduceTasks", "3"])
    assert sorted(_lines(out)) == ["a\t2", "b\t1"]
    # -lazyOutput: a map-only job whose maps emit nothing leaves no part files
    (inp / "b").write_text("zz\n")
    out2 = tmp_path / "out2"
    quiet = _script(tmp_path, "q.py", "for l in sys.stdin:\n  pass\n")
    _run(["-input", str(inp), "-output", str(out2), "-mapper", quiet, "-reducer", "NONE",
          "-lazyOutput"])
    assert not [f for f in os.listdir(out2) if f.startswith("part-")]


def test_bad_io_identifier_and_missing_reader(tmp_path):
    with pytest.raises(ValueError):
        streaming.stream_job_conf(["-input", "x", "-output", "y", "-io", "json"])
    with pytest.raises((ImportError, AttributeError, ModuleNotFoundError)):
        streaming.stream_job_conf(["-input", "x", "-output", "y",
                                   "-inputreader", "no.such:Reader,begin=a"])
    assert struct.calcsize(">i") == 4
