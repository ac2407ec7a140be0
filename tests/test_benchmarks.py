"""Benchmarks/validators of the reference's test tree: TestDFSIO
(fs/TestDFSIO.java), NNBench (hdfs/NNBench.java), MRBench, SortValidator,
BigMapOutput, ThreadedMapBenchmark (mapred/*.java)."""
from __future__ import annotations

import os

import pytest

from hbmr.benchmarks import bigmapoutput, dfsio, mrbench, nnbench, sortvalidator
from hbmr.examples import randomwriter, sort
from hbmr.io import sequencefile as seqf
from hbmr.mapred import JobClient, JobConf


@pytest.mark.parametrize("target", ["local", "dfs"])
def test_dfsio_write_then_read(tmp_path, target):
    if target == "dfs":
        from hbmr.dfs.cluster import MiniDFSCluster
        ctx = MiniDFSCluster(num_datanodes=2, base_dir=str(tmp_path / "dfs"))
    else:
        import contextlib
        ctx = contextlib.nullcontext()
    with ctx as dfs:
        base = (dfs.uri + "/benchmarks/TestDFSIO") if dfs else str(tmp_path / "TestDFSIO")
        res_file = str(tmp_path / "res.log")
        w = dfsio.run("write", nr_files=3, file_size_mb=2, base_dir=base, res_file=res_file)
        assert w["totalMBytes"] == 6 and w["throughput_mb_s"] > 0
        r = dfsio.run("read", nr_files=3, file_size_mb=2, base_dir=base)
        assert r["totalMBytes"] == 6 and r["avg_io_rate_mb_s"] > 0 and r["io_rate_std_dev"] >= 0
        assert "Throughput mb/sec" in open(res_file).read()
        dfsio.clean(base)


def test_nnbench_operations_in_order(tmp_path):
    from hbmr.dfs.cluster import MiniDFSCluster
    with MiniDFSCluster(num_datanodes=1, base_dir=str(tmp_path / "dfs")) as dfs:
        base = dfs.uri + "/benchmarks/NNBench"
        for op in nnbench.OPS:
            r = nnbench.run(op, maps=2, files_per_map=5, bytes_to_write=10, base_dir=base,
                            start_delay_s=0.05)
            assert r["successful_file_ops"] == 10 and r["exceptions"] == 0, r
            assert r["tps"] > 0
        # everything renamed and deleted
        from hbmr.fs import get_fs
        assert get_fs(base).list_status(base + "/data") == []


def test_mrbench_runs(tmp_path):
    r = mrbench.run(num_runs=2, maps=2, reduces=1, input_lines=20, input_type="random",
                    base_dir=str(tmp_path))
    assert len(r["times_ms"]) == 2 and r["AvgTime_ms"] > 0
    out = open(tmp_path / "mr_output_0" / "part-00000").read().split("\n")
    assert [int(x.split("\t")[0]) for x in out if x] == sorted(range(20), key=str)


def test_sortvalidator_accepts_sort_and_rejects_tampering(tmp_path):
    inp, out = str(tmp_path / "in"), str(tmp_path / "out")
    JobClient.runJob(randomwriter.make_job(inp, maps=2, bytes_per_map=200_000), verbose=False)
    JobClient.runJob(sort.make_job(inp, out, reduces=3), verbose=False)
    res = sortvalidator.validate(inp, out)
    assert res["ok"], res
    assert res["IN_RECORDS"] == res["OUT_RECORDS"] > 0
    # tamper: swap the first two records of one output file → unsorted (and the
    # records are still the same multiset)
    p = os.path.join(out, "part-00001")
    r = seqf.Reader(p)
    kc, vc = r.key_class, r.value_class
    recs = list(iter(r.next_raw, None))
    r.close()
    recs[0], recs[1] = recs[1], recs[0]
    with seqf.Writer(p, kc, vc) as w:
        for kb, vb in recs:
            w.append_raw(kb, vb)
    res = sortvalidator.validate(inp, out)
    assert not res["ok"] and res["UNSORTED_RECORDS"] >= 1 and res["checksum_match"]
    # drop a record → counts/checksum mismatch
    with seqf.Writer(p, kc, vc) as w:
        for kb, vb in sorted(recs[1:], key=lambda kv: kc.raw_sort_key(kv[0])):
            w.append_raw(kb, vb)
    res = sortvalidator.validate(inp, out)
    assert not res["ok"] and res["IN_RECORDS"] == res["OUT_RECORDS"] + 1


def test_bigmapoutput_spills_and_survives(tmp_path):
    r = bigmapoutput.big_map_output(str(tmp_path), create_mb=3, sort_mb=1)
    assert r["map_output_records"] == r["records_generated"] == r["reduce_output_records"]
    assert r["spilled_records"] >= r["map_output_records"]  # map spills (+ merge passes)


def test_threaded_map_benchmark(tmp_path):
    conf = JobConf()
    r = bigmapoutput.threaded_map_benchmark(str(tmp_path), maps=2, mb_per_map=1, threads=3,
                                            conf=conf)
    assert r["sort_s"] > 0
    res = sortvalidator.validate(str(tmp_path / "tmb-in"), str(tmp_path / "tmb-out"))
    assert res["ok"], res
