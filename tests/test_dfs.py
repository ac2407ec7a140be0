"""hbmr DFS (HDFS redesigned for one node): multi-block files
with replication, checksum failover + re-replication, DataNode death,
NameNode restart from image + edit log with safe mode, MapReduce over hdfs://
paths with data-local placement, and the RPC-served NameNode/DataNodes.
Mirrors TestDFSShell / TestReplication / TestDatanodeDeath / TestCheckpoint /
TestMiniMRWithDFS in the reference's test tree."""
import collections
import os
import random
import time

import pytest

from hbmr import fs as F
from hbmr.dfs import MiniDFSCluster, SafeModeException
from hbmr.mapred import JobClient, JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.models import wordcount


def _conf(block=1 << 20, repl=2):
    c = JobConf()
    c.set_long("dfs.block.size", block)
    c.set_int("dfs.replication", repl)
    c.set_int("dfs.heartbeat.interval.ms", 100)
    c.set_int("dfs.replication.interval.ms", 100)
    c.set_int("dfs.namenode.dead.interval.ms", 1500)
    return c


def _wait(pred, timeout=15):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.05)
    return pred()


def _live_replicas(cl, path):
    return [len(b["dns"]) for b in cl.nn.get_block_locations(path)]


def test_write_read_list_rename_delete():
    with MiniDFSCluster(_conf(), num_datanodes=3) as cl:
        fs = cl.filesystem()
        data = random.Random(1).randbytes(3 * (1 << 20) + 12345)
        with fs.create(f"{cl.uri}/a/b/f.bin") as f:
            f.write(data[:100])
            f.write(data[100:])
        st = fs.get_file_status(f"{cl.uri}/a/b/f.bin")
        assert st.length == len(data) and not st.is_dir
        with fs.open(f"{cl.uri}/a/b/f.bin") as f:
            assert f.read() == data
            f.seek(2 * (1 << 20) - 5)
            assert f.read(10) == data[2 * (1 << 20) - 5:2 * (1 << 20) + 5]
        locs = fs.get_file_block_locations(f"{cl.uri}/a/b/f.bin", 0, len(data))
        assert len(locs) == 4 and all(len(h) == 2 for _, _, h in locs)
        assert [os.path.basename(s.path) for s in fs.list_status(f"{cl.uri}/a/b")] == ["f.bin"]
        assert fs.rename(f"{cl.uri}/a", f"{cl.uri}/c")
        assert fs.exists(f"{cl.uri}/c/b/f.bin") and not fs.exists(f"{cl.uri}/a")
        assert [s.path for s in fs.glob_status(f"{cl.uri}/c/*/f.*")] == [f"{cl.uri}/c/b/f.bin"]
        stored = sum(len(dn.stored_blocks()) for dn in cl.datanodes)
        assert stored == 8
        assert fs.delete(f"{cl.uri}/c", recursive=True)
        assert _wait(lambda: sum(len(dn.stored_blocks()) for dn in cl.datanodes) == 0)
        rep = cl.nn.fsck("/")
        assert rep["files"] == 0 and rep["status"] == "HEALTHY"


def test_corrupt_replica_failover_and_rereplication():
    with MiniDFSCluster(_conf(repl=2), num_datanodes=3) as cl:
        fs = cl.filesystem(host="dnhost0")     # reads prefer the local replica
        data = random.Random(2).randbytes(300_000)
        with fs.create(f"{cl.uri}/f") as f:
            f.write(data)
        (b,) = cl.nn.get_block_locations("/f")
        victim = cl.datanodes[int(b["dns"][0][2:])]
        p = os.path.join(victim.dir, f"blk_{b['block']}")
        raw = bytearray(open(p, "rb").read())
        raw[1000] ^= 0xFF
        open(p, "wb").write(bytes(raw))
        # every replica order: the read must succeed via the good one
        for h in ("dnhost0", "dnhost1", "dnhost2"):
            with cl.filesystem(host=h).open(f"{cl.uri}/f") as f:
                assert f.read() == data
        # the bad replica was reported, deleted and replaced
        assert _wait(lambda: _live_replicas(cl, "/f") == [2] and
                     victim.id not in cl.nn.get_block_locations("/f")[0]["dns"] or
                     victim.block_length(b["block"]) == len(data) and not victim.verify_all())


def test_datanode_death_triggers_rereplication():
    with MiniDFSCluster(_conf(repl=2), num_datanodes=4) as cl:
        fs = cl.filesystem()
        with fs.create(f"{cl.uri}/f") as f:
            f.write(b"x" * (2 * (1 << 20) + 7))
        before = cl.nn.get_block_locations("/f")
        dead = before[0]["dns"][0]
        cl.stop_datanode(int(dead[2:]))
        assert _wait(lambda: all(len(b["dns"]) == 2 and dead not in b["dns"]
                                 for b in cl.nn.get_block_locations("/f")), timeout=20)
        with fs.open(f"{cl.uri}/f") as f:
            assert f.read() == b"x" * (2 * (1 << 20) + 7)
        assert cl.nn.fsck("/")["under_replicated_blocks"] == 0


def test_namenode_restart_replays_edits_and_safemode(tmp_path):
    conf = _conf(repl=1)
    cl = MiniDFSCluster(conf, num_datanodes=2, base_dir=str(tmp_path / "dfs"))
    try:
        fs = cl.filesystem()
        for i in range(3):
            with fs.create(f"{cl.uri}/d/f{i}") as f:
                f.write(bytes([i]) * (1500000 + i))
        cl.nn.save_namespace()                  # checkpoint ...
        with fs.create(f"{cl.uri}/d/after") as f:  # ... then more edits
            f.write(b"tail")
        fs.rename(f"{cl.uri}/d/f0", f"{cl.uri}/d/g0")
        nn = cl.restart_namenode()
        assert nn.safe_mode
        with pytest.raises(SafeModeException):
            nn.mkdirs("/x")
        assert _wait(lambda: not nn.safe_mode)   # block reports arrive on re-register
        fs = cl.filesystem()
        assert sorted(os.path.basename(s.path) for s in fs.list_status(f"{cl.uri}/d")) == \
            ["after", "f1", "f2", "g0"]
        with fs.open(f"{cl.uri}/d/f2") as f:
            assert f.read() == bytes([2]) * 1500002
        with fs.open(f"{cl.uri}/d/after") as f:
            assert f.read() == b"tail"
    finally:
        cl.shutdown()


def test_wordcount_over_hdfs_with_data_local_maps(tmp_path):
    hosts = ["node-a", "node-b"]
    conf = _conf(block=64 << 10, repl=1)
    with MiniDFSCluster(conf, hosts=hosts) as dfs:
        fs = dfs.filesystem(host="node-a")
        cnt = collections.Counter()
        rnd = random.Random(3)
        for i in range(3):
            lines = [" ".join(f"w{rnd.randint(0, 40)}" for _ in range(rnd.randint(1, 9)))
                     for _ in range(4000)]
            with fs.create(f"{dfs.uri}/in/part{i}") as f:
                f.write(("\n".join(lines) + "\n").encode())
            for ln in lines:
                cnt.update(ln.split())
        cc = JobConf()
        # delay scheduling long enough that a loaded host (pytest -n 8) does
        # not hand a tracker the other node's blocks before that one asks
        cc.set_int("hbmr.locality.wait.ms", 3000)
        with LocalCluster(cc, num_trackers=2, cpu_slots=2, hosts=hosts) as cl:
            # the per-record mapper: maps long enough that each tracker is
            # offered its own blocks before the other could take them
            wc = JobConf()
            wc.set_boolean("hbmr.wordcount.native", False)
            job = wordcount.make_job(f"{dfs.uri}/in", f"{dfs.uri}/out", reduces=2, conf=wc)
            rj = JobClient.runJob(job, cluster=cl, verbose=False)
            cs = rj.getCounters()
        got = {}
        for name in F.listdir(f"{dfs.uri}/out"):
            if name.startswith("part-"):
                with F.fopen(f"{dfs.uri}/out/{name}") as f:
                    for line in f.read().decode().splitlines():
                        k, v = line.split("\t")
                        got[k] = int(v)
        assert got == dict(cnt)
        assert F.exists(f"{dfs.uri}/out/_SUCCESS")
        jip = "org.apache.hadoop.mapred.JobInProgress$Counter"
        assert cs.get(jip, "DATA_LOCAL_MAPS") >= cs.get(jip, "TOTAL_LAUNCHED_MAPS") // 2


def test_rpc_served_dfs():
    with MiniDFSCluster(_conf(repl=2), num_datanodes=2, serve_rpc=True) as cl:
        from hbmr.dfs.client import DistributedFileSystem
        fs = DistributedFileSystem(cl.rpc_address)
        # force the DataNode hops over RPC too
        from hbmr.dfs import datanode as D
        saved = dict(D._registry)
        D._registry.clear()
        try:
            with fs.create(f"hdfs://{cl.rpc_address}/r/f") as f:
                f.write(b"hello over rpc" * 1000)
            with fs.open(f"hdfs://{cl.rpc_address}/r/f") as f:
                assert f.read() == b"hello over rpc" * 1000
        finally:
            D._registry.update(saved)
        assert cl.nn.fsck("/")["blocks"] == 1


def test_fs_shell_on_hdfs(tmp_path, capsys):
    from hbmr import cli
    with MiniDFSCluster(_conf(repl=1), num_datanodes=1) as cl:
        src = tmp_path / "local.txt"
        src.write_text("one\ntwo\n")
        assert cli.main(["fs", "-mkdir", f"{cl.uri}/u"]) == 0
        assert cli.main(["fs", "-put", str(src), f"{cl.uri}/u"]) == 0
        assert cli.main(["fs", "-cat", f"{cl.uri}/u/local.txt"]) == 0
        assert capsys.readouterr().out.endswith("one\ntwo\n")
        assert cli.main(["fs", "-ls", f"{cl.uri}/u"]) == 0
        assert "local.txt" in capsys.readouterr().out
        assert cli.main(["fs", "-get", f"{cl.uri}/u/local.txt", str(tmp_path / "back.txt")]) == 0
        assert (tmp_path / "back.txt").read_text() == "one\ntwo\n"
        assert cli.main(["fsck", f"{cl.uri}/"]) == 0
        assert '"HEALTHY"' in capsys.readouterr().out
        assert cli.main(["dfsadmin", "-nn", cl.name, "-report"]) == 0
        assert cli.main(["fs", "-rmr", f"{cl.uri}/u"]) == 0
        assert not F.exists(f"{cl.uri}/u")
