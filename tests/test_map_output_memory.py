"""In-memory map outputs (hbmr/mapred/mapoutput.py): a small single-spill map
output of an in-process cluster is held in the tracker process instead of
written as file.out + file.out.index, read by the reduce from there, and
purged with the job (KillJobAction, TaskTracker.purgeJob's removeJobFiles)."""
import collections
import os
import time
import types

from hbmr.io.writable import Text
from hbmr.mapred import JobClient, JobConf
from hbmr.mapred import mapoutput
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.task import MapOutputBuffer, MapOutputLocation, TaskReporter
from hbmr.models import wordcount


def _buffer(tmp_path, name, memory, R=3):
    job = JobConf()
    job.set_num_reduce_tasks(R)
    job.set_map_output_key_class(Text)
    job.set_map_output_value_class(Text)
    task = types.SimpleNamespace(check_killed=lambda: None, attempt_id=f"attempt_{name}",
                                 memory_outputs=memory)
    return MapOutputBuffer(task, job, TaskReporter(), str(tmp_path / name / "output"))


def test_memory_output_reads_like_the_file(tmp_path):
    outs = {}
    for name, memory in (("disk", False), ("mem", True)):
        buf = _buffer(tmp_path, name, memory)
        for i in range(500):
            buf.collect(Text(f"k{i % 37}"), Text("v" * (i % 23)))
        path = buf.flush()
        outs[name] = [MapOutputLocation("a", path).read_partition(p) for p in range(3)]
        if memory:
            assert not os.path.exists(path) and not os.path.exists(os.path.dirname(path))
            assert mapoutput.STORE.get(path) is not None
            assert mapoutput.STORE.drop_prefix(str(tmp_path / name)) == 1
        else:
            assert os.path.exists(path) and os.path.exists(path + ".index")
    # the same records; the in-memory output carries no CRC (it is read only
    # as a VerifiedSegment, never checked), the file's CRC is checked
    assert [bytes(x[:-4]) for x in outs["disk"]] == [bytes(x[:-4]) for x in outs["mem"]]
    from hbmr.io.ifile import read_segment
    for d, m in zip(outs["disk"], outs["mem"]):
        assert read_segment(d) == read_segment(m)


def test_memory_output_the_store_turns_away_gets_its_crcs(tmp_path):
    """An output meant for memory (CRC skipped) that the store refuses (its
    total cap) is written to its files with every segment's CRC filled in."""
    from hbmr.io.ifile import read_segment
    buf = _buffer(tmp_path, "full", True)
    buf.mem_total = 1                                   # the store is full
    for i in range(300):
        buf.collect(Text(f"k{i % 31}"), Text("w" * (i % 17)))
    path = buf.flush()
    assert os.path.exists(path) and mapoutput.STORE.get(path) is None
    segs = [MapOutputLocation("a", path).read_partition(p) for p in range(3)]
    assert sum(len(read_segment(x)) for x in segs) == 300     # CRCs verify


def test_memory_output_over_the_cap_goes_to_disk(tmp_path):
    buf = _buffer(tmp_path, "big", True, R=1)
    buf.job.set_long(mapoutput.MAX_KEY, 100)         # the map's output is larger
    buf.mem_max = 100
    for i in range(50):
        buf.collect(Text(f"k{i}"), Text("x" * 10))
    path = buf.flush()
    assert os.path.exists(path) and mapoutput.STORE.get(path) is None


def test_cluster_job_uses_memory_outputs_and_purges_them(tmp_path, monkeypatch):
    held = []
    real_put = mapoutput.STORE.put

    def put(path, data, index, cap=None):
        ok = real_put(path, data, index, cap)
        held.append((path, ok))
        return ok
    monkeypatch.setattr(mapoutput.STORE, "put", put)
    inp = tmp_path / "in"
    inp.mkdir()
    cnt = collections.Counter()
    for i in range(3):
        lines = [" ".join(f"w{(j * 7 + i) % 11}" for _ in range(j % 5)) for j in range(200)]
        (inp / f"f{i}.txt").write_text("\n".join(lines) + "\n")
        for ln in lines:
            cnt.update(ln.split())
    conf = JobConf()
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        wc = JobConf()
        wc.set_boolean("hbmr.wordcount.native", False)
        job = wordcount.make_job(str(inp), str(tmp_path / "out"), reduces=2, conf=wc)
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
        assert rj.isSuccessful()
        jid = str(rj.getID())
        # every map's output was held in memory (3 input files -> 3 maps)
        assert len(held) == 3 and all(ok and jid in p for p, ok in held)
        # the finished job is purged from the trackers (its kill action rides
        # on their next heartbeats)
        end = time.time() + 10
        while time.time() < end and any(jid in p for p in mapoutput.STORE._d):
            time.sleep(0.05)
        assert not any(jid in p for p in mapoutput.STORE._d)
        # (the same job with the store off writes files)
        wc.set_long(mapoutput.MAX_KEY, 0)
        job = wordcount.make_job(str(inp), str(tmp_path / "out2"), reduces=2, conf=wc)
        assert JobClient.runJob(job, cluster=cl, verbose=False).isSuccessful()
        assert len(held) == 3
    got = {}
    for fn in os.listdir(tmp_path / "out"):
        if fn.startswith("part-"):
            for line in open(tmp_path / "out" / fn):
                k, v = line.rstrip("\n").split("\t")
                got[k] = int(v)
    assert got == dict(cnt)


def test_empty_output_without_the_store_is_a_file(tmp_path):
    # an empty map output (0 buffered bytes) of a task that may not use the
    # store (a child-process task) still gets its files: reduces elsewhere
    # open them
    buf = _buffer(tmp_path, "empty", False, R=2)
    path = buf.flush()
    assert os.path.exists(path) and os.path.exists(path + ".index")
    assert mapoutput.STORE.get(path) is None
