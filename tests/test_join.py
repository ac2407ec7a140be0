"""Map-side joins (hbmr/mapred/join; the reference's mapred/join package and
examples/Join.java): sources sorted by key and partitioned alike are joined
inside the map tasks; the output equals the reduce-side join's."""
import io
import os

import pytest

from hbmr.examples import driver, join
from hbmr.io import sequencefile as seqf
from hbmr.io.writable import IntWritable, Text, hash_bytes
from hbmr.mapred import JobClient
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.formats import SequenceFileInputFormat, TextOutputFormat
from hbmr.mapred.jobconf import JobConf
from hbmr.mapred.join import (CompositeInputFormat, CompositeInputSplit, TupleWritable, parse,
                              tokenize)

PARTS = 3


def _part(key: str) -> int:
    return (hash_bytes(Text(key).serialize()[1:]) & 0x7FFFFFFF) % PARTS


def _source(d, records):
    """A sorted, hash-partitioned SequenceFile dataset (like a job's output)."""
    d.mkdir()
    parts = [[] for _ in range(PARTS)]
    for k, v in records:
        parts[_part(k)].append((k, v))
    for i, recs in enumerate(parts):
        with seqf.Writer(str(d / f"part-{i:05d}"), Text, Text) as w:
            for k, v in sorted(recs, key=lambda kv: Text(kv[0]).serialize()):
                w.append(Text(k), Text(v))
    return str(d)


A = [("k1", "a1"), ("k2", "a2"), ("k3", "a3"), ("k5", "a5"), ("k7", "a7"), ("k8", "a8")]
B = [("k1", "b1"), ("k1", "b1x"), ("k3", "b3"), ("k4", "b4"), ("k7", "b7"), ("k9", "b9")]
C = [("k1", "c1"), ("k4", "c4"), ("k7", "c7"), ("k10", "c10")]


@pytest.fixture(scope="module")
def cluster():
    cl = LocalCluster(JobConf(), num_trackers=2, cpu_slots=2)
    yield cl
    cl.shutdown()


def _run_join(cluster, inputs, out, op):
    job = join.make_job(inputs, out, op, reduces=0, out_format=TextOutputFormat,
                        out_key=Text, out_value=TupleWritable)
    rj = JobClient.runJob(job, cluster=cluster, verbose=False)
    assert rj.isSuccessful()
    rows = []
    for fn in sorted(os.listdir(out)):
        if fn.startswith("part-"):
            for line in open(os.path.join(out, fn)):
                k, v = line.rstrip("\n").split("\t")
                rows.append((k, tuple(v[1:-1].split(","))))
    return sorted(rows)


def test_inner_join_equals_the_reduce_side_join(tmp_path, cluster):
    a, b = _source(tmp_path / "a", A), _source(tmp_path / "b", B)
    got = _run_join(cluster, [a, b], str(tmp_path / "out"), "inner")
    assert got == [("k1", ("a1", "b1")), ("k1", ("a1", "b1x")), ("k3", ("a3", "b3")),
                   ("k7", ("a7", "b7"))]
    # the same pairs as the reduce-side join of the text form of the inputs
    for name, recs in (("ta", A), ("tb", B)):
        (tmp_path / name).mkdir()
        (tmp_path / name / "x").write_text("".join(f"{k}\t{v}\n" for k, v in recs))
    JobClient.runJob(join.make_reduce_side_job([str(tmp_path / "ta"), str(tmp_path / "tb")],
                                               str(tmp_path / "rs")), cluster=cluster,
                     verbose=False)
    rs = []
    for fn in sorted(os.listdir(tmp_path / "rs")):
        if fn.startswith("part-"):
            for line in open(tmp_path / "rs" / fn):
                k, x, y = line.rstrip("\n").split("\t")
                rs.append((k, (x, y)))
    assert got == sorted(rs)


def test_outer_and_override_joins(tmp_path, cluster):
    a, b = _source(tmp_path / "a", A), _source(tmp_path / "b", B)
    got = _run_join(cluster, [a, b], str(tmp_path / "outer"), "outer")
    keys = sorted({k for k, _ in A} | {k for k, _ in B})
    assert sorted({k for k, _ in got}) == keys
    assert ("k2", ("a2", "")) in got and ("k4", ("", "b4")) in got
    assert [t for k, t in got if k == "k1"] == [("a1", "b1"), ("a1", "b1x")]
    # override: per key the rightmost source that has it
    job = join.make_job([a, b], str(tmp_path / "ov"), "override", out_format=TextOutputFormat,
                        out_key=Text, out_value=Text)
    assert JobClient.runJob(job, cluster=cluster, verbose=False).isSuccessful()
    rows = sorted(tuple(line.rstrip("\n").split("\t")) for fn in os.listdir(tmp_path / "ov")
                  if fn.startswith("part-") for line in open(tmp_path / "ov" / fn))
    want = {}
    for k, v in A:
        want.setdefault(k, []).append(v)
    bmap = {}
    for k, v in B:
        bmap.setdefault(k, []).append(v)
    want.update(bmap)
    assert rows == sorted((k, v) for k, vs in want.items() for v in vs)


def test_nested_expression_and_key_comparator(tmp_path, cluster):
    a, b, c = (_source(tmp_path / n, r) for n, r in (("a", A), ("b", B), ("c", C)))
    fmt = "hbmr.mapred.formats:SequenceFileInputFormat"
    job = join.make_job([a, b], str(tmp_path / "o"), "inner", out_format=TextOutputFormat,
                        out_key=Text, out_value=TupleWritable)
    job.set("mapred.join.expr", f'outer(inner(tbl({fmt},"{a}"),tbl({fmt},"{b}")),'
                                f'tbl(org.apache.hadoop.mapred.SequenceFileInputFormat,"{c}"))')
    assert JobClient.runJob(job, cluster=cluster, verbose=False).isSuccessful()
    rows = sorted(line.rstrip("\n") for fn in os.listdir(tmp_path / "o")
                  if fn.startswith("part-") for line in open(tmp_path / "o" / fn))
    # k1: inner(a,b) gives two tuples, c has c1 -> both combined with c1
    assert "k1\t[[a1,b1],c1]" in rows and "k1\t[[a1,b1x],c1]" in rows
    assert "k4\t[,c4]" in rows and "k10\t[,c10]" in rows
    assert "k3\t[[a3,b3],]" in rows
    assert not any(r.startswith("k2\t") for r in rows)      # only in a: not in inner(a,b)


def test_parser_splits_and_tuple_writable(tmp_path):
    toks = tokenize('inner(tbl(org.apache.hadoop.mapred.SequenceFileInputFormat,"/x/y"),'
                    'tbl(pkg.mod:Cls,"z"))')
    assert toks[0] == ("IDENT", "inner") and ("QUOT", "/x/y") in toks
    a = _source(tmp_path / "a", A)
    d = tmp_path / "two"
    d.mkdir()
    with seqf.Writer(str(d / "part-00000"), Text, Text) as w:
        w.append(Text("k1"), Text("v"))
    job = JobConf()
    job.set("mapred.join.expr", CompositeInputFormat.compose("inner", SequenceFileInputFormat,
                                                             a, str(d)))
    with pytest.raises(IOError, match="Inconsistent split cardinality"):
        CompositeInputFormat().getSplits(job, 1)
    job.set("mapred.join.expr", CompositeInputFormat.compose("inner", SequenceFileInputFormat,
                                                             a, a))
    splits = CompositeInputFormat().getSplits(job, 1)
    assert len(splits) == PARTS
    s2 = CompositeInputSplit.deserialize(splits[1].serialize())
    assert [repr(x) for x in s2.splits] == [repr(x) for x in splits[1].splits]
    with pytest.raises(ValueError):
        parse("inner(tbl(x,\"a\")", job)
    with pytest.raises(ValueError, match="no node type"):
        parse('bogus(tbl(x,"a"))', job)
    t = TupleWritable([Text("a"), None, IntWritable(7)])
    assert t.has(0) and not t.has(1) and t.has(2) and list(t) == [Text("a"), IntWritable(7)]
    t2 = TupleWritable()
    t2.readFields(io.BytesIO(t.serialize()))
    assert t2 == t and str(t2) == "[a,,7]"


def test_join_example_through_the_driver(tmp_path, cluster):
    a, b = _source(tmp_path / "a", A), _source(tmp_path / "b", B)
    out = str(tmp_path / "out")
    assert driver.run("join", ["-outFormat", "org.apache.hadoop.mapred.SequenceFileOutputFormat",
                               "-outKey", "org.apache.hadoop.io.Text", a, b, out],
                      cluster=cluster) == 0
    got = []
    for fn in sorted(os.listdir(out)):
        if fn.startswith("part-"):
            with seqf.Reader(os.path.join(out, fn)) as r:
                while True:
                    kv = r.next()
                    if kv is None:
                        break
                    got.append((str(kv[0]), str(kv[1])))
    assert sorted(got) == [("k1", "[a1,b1]"), ("k1", "[a1,b1x]"), ("k3", "[a3,b3]"),
                           ("k7", "[a7,b7]")]
