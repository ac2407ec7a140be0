"""DistCp, Hadoop archives (har://), Rumen traces and Gridmix replay
(hadoop-1.0.3/src/tools/org/apache/hadoop/tools/{DistCp,HadoopArchives}.java,
tools/rumen, contrib/gridmix; reference tests TestCopyFiles.java,
TestHarFileSystem.java, rumen/TestRumenJobTraces.java, gridmix/TestGridmixSubmission.java)."""
from __future__ import annotations

import json
import os

import pytest

from hbmr import fs as F
from hbmr.mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.models import wordcount
from hbmr.tools import distcp, gridmix, har, rumen


def _tree(root, seed=0):
    import random
    rng = random.Random(seed)
    files = {}
    for rel in ["a/x.txt", "a/b/y.txt", "c.txt", "a/b/d/z.bin"]:
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        data = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 5000))) \
            if rel.endswith(".bin") else \
            (" ".join(rng.choice(["foo", "bar", "baz", "qux"]) for _ in range(300)) + "\n").encode()
        with open(p, "wb") as f:
            f.write(data)
        files[rel] = data
    return files


def _read_tree(root):
    out = {}
    for rel in F.walk_files(root):
        with F.fopen(os.path.join(root, rel)) as f:
            out[rel] = f.read()
    return out


def test_distcp_copy_update_overwrite_delete(tmp_path):
    src, dst = str(tmp_path / "src"), str(tmp_path / "dst")
    files = _tree(src)
    rj = distcp.copy([src], dst, maps=3)
    assert _read_tree(dst) == files
    cs = rj.getCounters()
    assert cs.get("distcp", "COPY") == len(files)
    assert cs.get("distcp", "BYTESCOPIED") == sum(map(len, files.values()))
    # -update: nothing changed → nothing to copy
    assert distcp.copy([src], dst, update=True) is None or \
        distcp.copy([src], dst, update=True).getCounters().get("distcp", "COPY") == 0
    # change one file, add a stray file at the destination
    with open(os.path.join(src, "c.txt"), "wb") as f:
        f.write(b"changed\n")
    with open(os.path.join(dst, "stray"), "wb") as f:
        f.write(b"x")
    rj = distcp.copy([src], dst, update=True, delete=True)
    assert rj.getCounters().get("distcp", "COPY") == 1
    assert not os.path.exists(os.path.join(dst, "stray"))
    assert open(os.path.join(dst, "c.txt"), "rb").read() == b"changed\n"
    # without -update/-overwrite into an existing dir: copied under dst/<basename>
    rj = distcp.copy([src], dst)
    assert os.path.exists(os.path.join(dst, "src", "a", "x.txt"))
    # second plain copy skips existing files
    rj = distcp.copy([src], dst)
    assert rj.getCounters().get("distcp", "SKIP") == len(files)
    with pytest.raises(ValueError):
        distcp.copy([src], dst, delete=True)


def test_distcp_local_to_dfs_and_back(tmp_path):
    from hbmr.dfs.cluster import MiniDFSCluster
    src = str(tmp_path / "src")
    files = _tree(src, seed=3)
    with MiniDFSCluster(num_datanodes=2, base_dir=str(tmp_path / "dfs")) as dfs:
        uri = dfs.uri + "/copied"
        distcp.copy([src], uri, maps=2)
        assert _read_tree(uri) == files
        back = str(tmp_path / "back")
        distcp.copy([uri], back, maps=2)
        assert _read_tree(back) == files


def test_har_archive_list_read_and_mapreduce_input(tmp_path):
    src = str(tmp_path / "data")
    files = _tree(src, seed=1)
    har.create_archive("foo.har", str(tmp_path), ["data"], str(tmp_path / "arch"), maps=2)
    root = f"har://{tmp_path}/arch/foo.har"
    assert sorted(os.listdir(tmp_path / "arch" / "foo.har"))[:2] == ["_index", "_masterindex"]
    fs = F.get_fs(root)
    assert fs.is_dir(root + "/data/a") and not fs.is_dir(root + "/data/c.txt")
    names = sorted(os.path.basename(s.path) for s in fs.list_status(root + "/data/a"))
    assert names == ["b", "x.txt"]
    for rel, data in files.items():
        st = fs.get_file_status(f"{root}/data/{rel}")
        assert st.length == len(data)
        with F.fopen(f"{root}/data/{rel}") as f:
            assert f.read() == data
        with F.fopen(f"{root}/data/{rel}") as f:  # seek inside a member
            f.seek(len(data) // 2)
            assert f.read() == data[len(data) // 2:]
    with pytest.raises(PermissionError):
        fs.delete(root + "/data/c.txt")
    # a job reads its input straight out of the archive
    out = str(tmp_path / "wc")
    job = wordcount.make_job(f"{root}/data/a", out, reduces=1)
    JobClient.runJob(job, verbose=False)
    counts = {}
    for ln in open(os.path.join(out, "part-00000")):
        w, c = ln.split("\t")
        counts[w] = int(c)
    exp = {}
    for rel in ("a/x.txt",):  # FileInputFormat does not recurse into a/b
        for w in files[rel].decode().split():
            exp[w] = exp.get(w, 0) + 1
    assert counts == exp


def test_har_hash_ordered_master_index(tmp_path):
    src = tmp_path / "many"
    src.mkdir()
    for i in range(2500):
        (src / f"f{i}").write_bytes(str(i).encode())
    har.create_archive("m.har", str(tmp_path), ["many"], str(tmp_path / "o"), maps=3)
    lines = (tmp_path / "o" / "m.har" / "_masterindex").read_text().splitlines()
    assert lines[0].split()[0] == str(har.VERSION)
    ranges = [tuple(map(int, ln.split())) for ln in lines[1:]]
    assert len(ranges) == 3  # 2502 index lines / 1000
    assert all(a[1] <= b[0] for a, b in zip(ranges, ranges[1:]))
    fs = F.get_fs(f"har://{tmp_path}/o/m.har")
    with F.fopen(f"har://{tmp_path}/o/m.har/many/f1234") as f:
        assert f.read() == b"1234"
    assert len(fs.listdir(f"har://{tmp_path}/o/m.har/many")) == 2500


def test_java_string_hash():
    assert har.java_string_hash("") == 0
    assert har.java_string_hash("hello") == 99162322
    assert har.java_string_hash("/a/very/long/path/name/for/overflow") == \
        _java_hash_ref("/a/very/long/path/name/for/overflow")


def _java_hash_ref(s):
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def _history_cluster_jobs(tmp_path):
    conf = JobConf()
    hist = str(tmp_path / "history")
    conf.set("hbmr.history.dir", hist)
    src = str(tmp_path / "in")
    _tree(src, seed=2)
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        for i in range(3):
            job = wordcount.make_job(os.path.join(src, "a"), str(tmp_path / f"wc{i}"),
                                     reduces=2, conf=conf)
            JobClient.runJob(job, cluster=cl, verbose=False)
    return hist


def test_rumen_trace_builder_and_zombie_job(tmp_path):
    hist = _history_cluster_jobs(tmp_path)
    trace, topo = str(tmp_path / "trace.json"), str(tmp_path / "topo.json")
    jobs = rumen.trace_builder([hist], trace, topo)
    assert len(jobs) == 3
    j = jobs[0]
    assert j["outcome"] == "SUCCESS" and j["totalReduces"] == 2
    assert len(j["mapTasks"]) == j["totalMaps"] and len(j["reduceTasks"]) == 2
    assert all(t["taskStatus"] == "SUCCESS" for t in j["mapTasks"])
    cdf = j["successfulMapAttemptCDFs"][0]
    assert cdf["numberValues"] == j["totalMaps"]
    assert cdf["minimum"] <= cdf["rankings"][9]["datum"] <= cdf["maximum"]
    assert [r["relativeRanking"] for r in cdf["rankings"]][:2] == [0.05, 0.1]
    t = json.load(open(topo))
    assert {h["name"] for r in t["children"] for h in r["children"]}
    stories = rumen.ZombieJobProducer(trace)
    z = stories.getNextJob()
    assert z.getNumberMaps() == j["totalMaps"]
    info = z.getTaskAttemptInfo("MAP", 0)
    assert info["runtime_ms"] >= 0
    # a task beyond the record draws from the CDF, within [min, max]
    drawn = z.getTaskAttemptInfo("MAP", 10_000)["runtime_ms"]
    assert cdf["minimum"] <= drawn <= cdf["maximum"]


def test_rumen_cdf_sampling_bounds():
    import random
    cdf = rumen.discrete_cdf(range(1, 101))
    assert cdf["minimum"] == 1 and cdf["maximum"] == 100
    rng = random.Random(0)
    xs = [rumen.sample_cdf(cdf, rng) for _ in range(2000)]
    assert min(xs) >= 1 and max(xs) <= 100
    assert 35 < sum(xs) / len(xs) < 65


@pytest.mark.parametrize("kind,policy", [("SLEEPJOB", "SERIAL"), ("LOADJOB", "STRESS"),
                                         ("SLEEPJOB", "REPLAY")])
def test_gridmix_replays_trace(tmp_path, kind, policy):
    hist = _history_cluster_jobs(tmp_path)
    trace = str(tmp_path / "trace.json")
    rumen.trace_builder([hist], trace)
    pool = gridmix.generate_data(str(tmp_path / "pool"), 1 << 20, files=2)
    assert sum(os.path.getsize(p) for p in pool) == 1 << 20
    with LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) as cl:
        st = gridmix.run(trace, kind, policy, pool, time_scale=0.01,
                         out_dir=str(tmp_path / "gm-out"), cluster=cl, max_in_flight=2)
    assert st["succeeded"] == 3 == len(st["jobs"])
    if kind == "LOADJOB":
        outs = F.walk_files(str(tmp_path / "gm-out"))
        assert any(o.endswith("part-00000") for o in outs)
    if policy == "SERIAL":
        js = sorted(st["jobs"], key=lambda r: r["submit_s"])
        assert all(a["finish_s"] <= b["submit_s"] + 1e-6 for a, b in zip(js, js[1:]))
