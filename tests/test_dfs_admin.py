"""DFS administration: SecondaryNameNode checkpoints (TestCheckpoint.java),
Balancer (balancer/TestBalancer.java), name/space quotas (TestQuota.java) and
lease hard-limit recovery (TestLeaseRecovery.java) on hbmr.dfs."""
import json
import os
import random

import pytest

from hbmr.dfs import MiniDFSCluster
from hbmr.dfs.balancer import SUCCESS, Balancer, utilisation
from hbmr.dfs.namenode import QuotaExceededException
from hbmr.dfs.secondary import SecondaryNameNode

from test_dfs import _conf, _wait


def _names(fs, d):
    return sorted(os.path.basename(s.path) for s in fs.list_status(d))


def test_secondary_namenode_checkpoint_and_restart(tmp_path):
    cl = MiniDFSCluster(_conf(repl=1), num_datanodes=2, base_dir=str(tmp_path / "dfs"))
    try:
        fs = cl.filesystem()
        for i in range(3):
            with fs.create(f"{cl.uri}/d/f{i}") as f:
                f.write(bytes([i]) * (700000 + i))
        snn = SecondaryNameNode(cl.nn, str(tmp_path / "ckpt"), name_dir=cl.name_dir)
        edits_before = os.path.getsize(os.path.join(cl.name_dir, "edits"))
        assert snn.do_checkpoint()
        img = json.load(open(os.path.join(cl.name_dir, "fsimage.json")))
        assert "/d/f2" in img["inodes"] and img["through_segment"] == 0
        assert not os.path.exists(os.path.join(cl.name_dir, "edits.old"))
        assert os.path.getsize(os.path.join(cl.name_dir, "edits")) < edits_before
        fs.rename(f"{cl.uri}/d/f0", f"{cl.uri}/d/g0")        # edits after the checkpoint
        # a roll whose merge never completes (SNN crash): restart must replay edits.old once
        cl.nn.roll_edit_log()
        with fs.create(f"{cl.uri}/d/late") as f:
            f.write(b"x")
        nn = cl.restart_namenode()
        assert _wait(lambda: not nn.safe_mode)
        fs = cl.filesystem()
        assert _names(fs, f"{cl.uri}/d") == ["f1", "f2", "g0", "late"]
        # the pending roll can still be checkpointed after the restart
        assert SecondaryNameNode(nn, str(tmp_path / "ckpt"), name_dir=cl.name_dir).do_checkpoint()
        nn = cl.restart_namenode()
        assert _wait(lambda: not nn.safe_mode)
        fs = cl.filesystem()
        assert _names(fs, f"{cl.uri}/d") == ["f1", "f2", "g0", "late"]
        with fs.open(f"{cl.uri}/d/f2") as f:
            assert f.read() == bytes([2]) * 700002
    finally:
        cl.shutdown()


def test_secondary_namenode_periodic_thread(tmp_path):
    cl = MiniDFSCluster(_conf(repl=1), num_datanodes=1, base_dir=str(tmp_path / "dfs"))
    try:
        snn = SecondaryNameNode(cl.nn, str(tmp_path / "ckpt"), period_s=0.1,
                                name_dir=cl.name_dir).start()
        fs = cl.filesystem()
        fs.mkdirs(f"{cl.uri}/x/y")
        assert _wait(lambda: snn.checkpoints >= 2, timeout=10)
        snn.shutdown()
    finally:
        cl.shutdown()


def test_balancer_moves_replicas_to_new_datanodes(tmp_path):
    conf = _conf(block=256 << 10, repl=1)
    conf.set_long("dfs.datanode.capacity", 8 << 20)
    cl = MiniDFSCluster(conf, num_datanodes=1, base_dir=str(tmp_path / "dfs"))
    try:
        fs = cl.filesystem()
        data = {i: random.Random(i).randbytes(600_000) for i in range(6)}
        for i, d in data.items():
            with fs.create(f"{cl.uri}/f{i}") as f:
                f.write(d)
        cl.start_datanode(1, "dnhost1")
        cl.start_datanode(2, "dnhost2")
        assert _wait(lambda: len([d for d in cl.nn.datanode_report() if d["alive"]]) == 3)
        before = utilisation(cl.nn)
        assert before["dn1"][0] == 0 and before["dn2"][0] == 0
        b = Balancer(cl.nn, threshold=10.0, max_iterations=10)
        assert b.run() == SUCCESS
        assert b.moved_blocks > 0
        after = utilisation(cl.nn)
        used = [after[d][0] for d in ("dn0", "dn1", "dn2")]
        total = sum(used)
        assert all(abs(u - total / 3) <= 0.25 * total for u in used), used
        # sources deleted their copies; every file still reads back intact
        assert _wait(lambda: sum(len(dn.stored_blocks()) for dn in cl.datanodes) ==
                     sum(len(cl.nn.get_blocks(d)) for d in ("dn0", "dn1", "dn2")))
        for i, d in data.items():
            with fs.open(f"{cl.uri}/f{i}") as f:
                assert f.read() == d
        assert cl.nn.fsck("/")["status"] == "HEALTHY"
    finally:
        cl.shutdown()


def test_quotas_and_content_summary(tmp_path):
    cl = MiniDFSCluster(_conf(block=128 << 10, repl=2), num_datanodes=2,
                        base_dir=str(tmp_path / "dfs"))
    try:
        fs = cl.filesystem()
        fs.mkdirs(f"{cl.uri}/q")
        fs.set_quota(f"{cl.uri}/q", 3, -1)        # the dir itself + 2 names
        fs.mkdirs(f"{cl.uri}/q/a")
        with fs.create(f"{cl.uri}/q/f") as f:
            f.write(b"1234")
        with pytest.raises(QuotaExceededException):
            fs.mkdirs(f"{cl.uri}/q/b")
        with pytest.raises(QuotaExceededException):
            fs.create(f"{cl.uri}/q/a/g")
        cs = fs.get_content_summary(f"{cl.uri}/q")
        assert cs == {"directoryCount": 2, "fileCount": 1, "length": 4, "spaceConsumed": 8,
                      "quota": 3, "spaceQuota": -1}
        fs.set_quota(f"{cl.uri}/q", -1, -1)       # clear
        fs.mkdirs(f"{cl.uri}/q/b")
        # space quota: one 128 KiB block at replication 2 needs 256 KiB
        fs.mkdirs(f"{cl.uri}/s")
        fs.set_quota(f"{cl.uri}/s", -1, 300 << 10)
        with fs.create(f"{cl.uri}/s/ok") as f:
            f.write(b"x" * 1000)
        with pytest.raises(QuotaExceededException):
            with fs.create(f"{cl.uri}/s/big") as f:
                f.write(b"y" * (200 << 10))
        # quotas persist in the edit log
        nn = cl.restart_namenode()
        assert nn.get_content_summary("/s")["spaceQuota"] == 300 << 10
    finally:
        cl.shutdown()


def test_lease_hard_limit_closes_abandoned_file(tmp_path):
    conf = _conf(block=128 << 10, repl=1)
    conf.set_int("dfs.lease.hard.limit.ms", 200)
    cl = MiniDFSCluster(conf, num_datanodes=1, base_dir=str(tmp_path / "dfs"))
    try:
        nn = cl.nn
        nn.create("/open", client="writer-1")
        r = nn.add_block("/open", client="writer-1")
        cl.datanodes[0].write_block(r["block"], b"z" * 5000)
        nn.add_block("/open", client="writer-1", prev_len=5000)   # never written
        assert nn.get_file_info("/open")["under_construction"]
        assert _wait(lambda: not nn.get_file_info("/open")["under_construction"], timeout=10)
        info = nn.get_file_info("/open")
        assert info["length"] == 5000
        fs = cl.filesystem()
        with fs.open(f"{cl.uri}/open") as f:
            assert f.read() == b"z" * 5000
        nn = cl.restart_namenode()
        assert nn.get_file_info("/open")["length"] == 5000
    finally:
        cl.shutdown()


def test_quota_and_balancer_cli(tmp_path, capsys):
    from hbmr import cli
    cl = MiniDFSCluster(_conf(repl=1), num_datanodes=2, base_dir=str(tmp_path / "dfs"))
    try:
        fs = cl.filesystem()
        fs.mkdirs(f"{cl.uri}/q/a")
        assert cli.main(["dfsadmin", "-nn", cl.name, "-setQuota", "10", "/q"]) == 0
        assert cli.main(["dfsadmin", "-nn", cl.name, "-setSpaceQuota", "1000000", "/q"]) == 0
        capsys.readouterr()
        assert cli.main(["fs", "-count", "-q", f"{cl.uri}/q"]) == 0
        out = capsys.readouterr().out.split()
        assert out[:7] == ["10", "8", "1000000", "1000000", "2", "0", "0"]
        assert cli.main(["dfsadmin", "-nn", cl.name, "-clrQuota", "/q"]) == 0
        assert cl.nn.get_content_summary("/q")["quota"] == -1
        assert cl.nn.get_content_summary("/q")["spaceQuota"] == 1000000
        assert cli.main(["balancer", "-nn", cl.name]) == 0
        assert cli.main(["secondarynamenode", "-nn", cl.name, "-dir",
                         str(tmp_path / "ck"), "-checkpoint"]) == 0
    finally:
        cl.shutdown()
