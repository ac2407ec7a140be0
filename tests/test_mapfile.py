"""MapFile / ArrayFile / SetFile / BloomMapFile (the reference's TestMapFile,
TestArrayFile, TestSetFile, TestBloomMapFile behaviours)."""
import os

import pytest

from hbmr.io import sequencefile as SF
from hbmr.io.mapfile import ArrayFile, BloomMapFile, MapFile, SetFile
from hbmr.io.writable import IntWritable, LongWritable, Text


def _keys(n):
    return [f"k{i:05d}" for i in range(0, 2 * n, 2)]     # even numbers only


@pytest.mark.parametrize("comp", [SF.NONE, SF.RECORD, SF.BLOCK])
def test_mapfile_get_seek_closest(tmp_path, comp):
    d = tmp_path / "mf"
    keys = _keys(1000)
    with MapFile.Writer(d, Text, IntWritable, compression=comp, index_interval=16) as w:
        for i, k in enumerate(keys):
            w.append(Text(k), IntWritable(i))
    assert sorted(os.listdir(d)) == ["data", "index"]
    with MapFile.Reader(d) as r:
        for i in (0, 1, 15, 16, 17, 500, 999):
            assert r.get(Text(keys[i])).get() == i
        assert r.get(Text("k00001")) is None            # odd: absent
        assert r.get(Text("zzz")) is None
        v = IntWritable()
        assert str(r.get_closest(Text("k00001"), v)) == "k00002" and v.get() == 1
        assert str(r.get_closest(Text("k00001"), v, before=True)) == "k00000" and v.get() == 0
        assert r.get_closest(Text("zzz")) is None
        assert str(r.get_closest(Text("zzz"), before=True)) == keys[-1]
        assert r.get_closest(Text("a"), before=True) is None
        assert str(r.final_key()) == keys[-1]
        assert str(r.mid_key()) in keys
        # sequential scan after a seek continues from the sought key
        assert r.seek(Text(keys[100]))
        k, val = r.next()
        assert str(k) == keys[100] and val.get() == 100
        k, val = r.next()
        assert str(k) == keys[101]
        assert [str(k) for k, _ in r] == keys


def test_mapfile_rejects_out_of_order_and_allows_duplicates(tmp_path):
    with MapFile.Writer(tmp_path / "m", Text, IntWritable) as w:
        w.append(Text("b"), IntWritable(1))
        w.append(Text("b"), IntWritable(2))
        with pytest.raises(IOError, match="out of order"):
            w.append(Text("a"), IntWritable(3))


def test_mapfile_duplicates_across_index_entries(tmp_path):
    d = tmp_path / "dup"
    with MapFile.Writer(d, IntWritable, IntWritable, index_interval=4) as w:
        for i in range(40):
            w.append(IntWritable(i // 10), IntWritable(i))
    with MapFile.Reader(d) as r:
        assert r.get(IntWritable(2)).get() == 20          # first of the run


@pytest.mark.parametrize("comp", [SF.NONE, SF.BLOCK])
def test_mapfile_fix_rebuilds_index(tmp_path, comp):
    d = tmp_path / "fix"
    with MapFile.Writer(d, LongWritable, Text, compression=comp) as w:
        for i in range(3000):
            w.append(LongWritable(i * 3), Text(f"v{i}"))
    os.unlink(d / "index")
    assert MapFile.fix(d, dry_run=True) == 3000
    assert not (d / "index").exists()
    assert MapFile.fix(d) == 3000
    with MapFile.Reader(d) as r:
        assert str(r.get(LongWritable(2997 * 3))) == "v2997"
        assert r.get(LongWritable(1)) is None
    assert MapFile.fix(d) == -1


def test_arrayfile_and_setfile(tmp_path):
    with ArrayFile.Writer(tmp_path / "af", Text) as w:
        for i in range(300):
            w.append(Text(f"item{i}"))
    with ArrayFile.Reader(tmp_path / "af") as r:
        assert str(r.get(123)) == "item123"
        assert r.seek(250) and r.key() == 250 and str(r.next()) == "item250"
        assert r.get(300) is None
    with SetFile.Writer(tmp_path / "sf", Text) as w:
        for k in _keys(200):
            w.append(Text(k))
    with SetFile.Reader(tmp_path / "sf") as r:
        assert r.contains(Text("k00010")) and not r.contains(Text("k00011"))
        assert str(r.next()) == "k00012"


def test_bloom_mapfile(tmp_path):
    d = tmp_path / "bmf"
    with BloomMapFile.Writer(d, Text, IntWritable, expected_keys=2000) as w:
        for i, k in enumerate(_keys(2000)):
            w.append(Text(k), IntWritable(i))
    with BloomMapFile.Reader(d) as r:
        assert all(r.probably_has_key(Text(k)) for k in _keys(2000))
        fp = sum(r.probably_has_key(Text(f"k{i:05d}")) for i in range(1, 4000, 2))
        assert fp < 60                                       # ~0.5 % of 2000 absent keys
        assert r.get(Text("k00400")).get() == 200
        assert r.get(Text("k00401")) is None


def test_mapfile_output_format_lookup(tmp_path):
    from hbmr.mapred import JobClient, MapFileOutputFormat
    from hbmr.mapred.lib.basic import HashPartitioner
    from hbmr.models import wordcount
    d = tmp_path / "in"
    d.mkdir()
    (d / "a").write_text("x y z x\ny y q\n")
    job = wordcount.make_job(str(d), str(tmp_path / "out"), reduces=3)
    job.set_output_format(MapFileOutputFormat)
    rj = JobClient.runJob(job, verbose=False)
    assert rj.isSuccessful()
    readers = MapFileOutputFormat.get_readers(str(tmp_path / "out"))
    assert len(readers) == 3
    part = HashPartitioner()
    assert MapFileOutputFormat.get_entry(readers, part, Text("y")).get() == 3
    assert MapFileOutputFormat.get_entry(readers, part, Text("x")).get() == 2
    assert MapFileOutputFormat.get_entry(readers, part, Text("nope")) is None
