"""The example programs (src/examples/org/apache/hadoop/examples + dancing +
terasort) through ExampleDriver, on the local runner and the mini cluster."""
import collections
import os

import numpy as np
import pytest

from hbmr.examples import dancing, driver, grep, join, pi, secondarysort
from hbmr.io import sequencefile as seqf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import terasort as T


@pytest.fixture(scope="module")
def cluster():
    cl = LocalCluster(JobConf(), num_trackers=2, cpu_slots=2)
    yield cl
    cl.shutdown()


def _text(tmp_path, name="in", files=2, lines=150):
    d = tmp_path / name
    d.mkdir()
    for i in range(files):
        (d / f"f{i}.txt").write_text("\n".join(
            " ".join(f"w{(i * 3 + j + t) % 9}" for t in range(j % 5)) for j in range(lines)) + "\n")
    return d


def _read_kv(out, sep="\t"):
    res = []
    for fn in sorted(os.listdir(out)):
        if fn.startswith("part-"):
            for line in open(os.path.join(out, fn)):
                res.append(line.rstrip("\n").split(sep))
    return res


def test_driver_lists_programs_and_rejects_unknown(capsys):
    assert driver.main(["nope"]) == -1
    assert "terasort" in capsys.readouterr().err


def test_grep_counts_and_sorts_descending(tmp_path, cluster):
    inp = _text(tmp_path)
    words = collections.Counter()
    for f in inp.iterdir():
        for w in f.read_text().split():
            words[w] += 1
    grep.run(str(inp), str(tmp_path / "out"), r"w[1-4]", cluster=cluster)
    rows = _read_kv(tmp_path / "out")
    counts = [int(c) for c, _ in rows]
    assert counts == sorted(counts, reverse=True)
    assert {w: int(c) for c, w in rows} == {w: c for w, c in words.items() if w in
                                             {"w1", "w2", "w3", "w4"}}


def test_randomwriter_then_total_order_sort(tmp_path, cluster):
    assert driver.run("randomwriter", [str(tmp_path / "rw"), "-m", "3", "-b", "20000"],
                      cluster=cluster) == 0
    assert driver.run("sort", [str(tmp_path / "rw"), str(tmp_path / "sorted"), "-r", "3",
                               "-totalOrder", "0.5", "1000", "3"], cluster=cluster) == 0
    keys = []
    n_in = 0
    for d, acc in (("rw", None), ("sorted", keys)):
        for fn in sorted(os.listdir(tmp_path / d)):
            if fn.startswith("part-"):
                with seqf.Reader(tmp_path / d / fn) as r:
                    for k, _v in r:
                        if acc is None:
                            n_in += 1
                        else:
                            acc.append(bytes(k.get()))
    assert len(keys) == n_in > 0
    from hbmr.io.writable import BytesWritable
    sk = [BytesWritable.raw_sort_key(BytesWritable(k).serialize()) for k in keys]
    assert sk == sorted(sk)


def test_pi_estimate():
    est = float(pi.estimate(4, 20000))
    assert abs(est - 3.14159) < 0.01


def test_secondary_sort(tmp_path):
    (tmp_path / "in").mkdir()
    rows = [(a, b) for a in (5, -3, 17) for b in (9, -2, 4, 4, 0)]
    (tmp_path / "in" / "x.txt").write_text("\n".join(f"{a} {b}" for a, b in rows[::-1]) + "\n")
    from hbmr.mapred import JobClient
    JobClient.runJob(secondarysort.make_job(str(tmp_path / "in"), str(tmp_path / "out")),
                     verbose=False)
    lines = [ln.rstrip("\n") for ln in open(tmp_path / "out" / "part-00000")]
    groups, cur = [], None
    for ln in lines:
        if ln.startswith("---"):
            cur = []
            groups.append(cur)
        else:
            a, b = ln.split("\t")
            cur.append((int(a), int(b)))
    assert [g[0][0] for g in groups] == [-3, 5, 17]
    for g in groups:
        assert [b for _, b in g] == sorted(b for _, b in g)


def test_reduce_side_join(tmp_path, cluster):
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    (tmp_path / "a" / "x").write_text("k1\ta1\nk2\ta2\nk3\ta3\n")
    (tmp_path / "b" / "y").write_text("k1\tb1\nk1\tb1x\nk3\tb3\nk4\tb4\n")
    from hbmr.mapred import JobClient
    JobClient.runJob(join.make_reduce_side_job([str(tmp_path / "a"), str(tmp_path / "b")],
                                               str(tmp_path / "out")), cluster=cluster,
                     verbose=False)
    got = sorted(tuple(r) for r in _read_kv(tmp_path / "out"))
    assert got == [("k1", "a1", "b1"), ("k1", "a1", "b1x"), ("k3", "a3", "b3")]


def test_multifile_and_aggregate_wordcount(tmp_path, cluster):
    inp = _text(tmp_path, files=5, lines=40)
    words = collections.Counter()
    for f in inp.iterdir():
        words.update(f.read_text().split())
    assert driver.run("multifilewc", [str(inp), str(tmp_path / "o1")], cluster=cluster) == 0
    assert {k: int(v) for k, v in _read_kv(tmp_path / "o1")} == dict(words)
    assert driver.run("aggregatewordcount", [str(inp), str(tmp_path / "o2"), "2"],
                      cluster=cluster) == 0
    assert {k: int(v) for k, v in _read_kv(tmp_path / "o2")} == dict(words)


def test_sudoku_and_distributed_pentomino(tmp_path, cluster):
    full = [[(r * 3 + r // 3 + c) % 9 + 1 for c in range(9)] for r in range(9)]
    holes = {(r, c) for r in range(9) for c in range(9) if (r * 7 + c * 5) % 3 == 0}
    puzzle = "\n".join(" ".join("?" if (r, c) in holes else str(full[r][c]) for c in range(9))
                       for r in range(9))
    sols = dancing.Sudoku.parse(puzzle).solve(limit=5)
    assert sols
    for s in sols:
        for r in range(9):
            assert sorted(s[r]) == list(range(1, 10))
            assert sorted(s[x][r] for x in range(9)) == list(range(1, 10))
            for c in range(9):
                if (r, c) not in holes:
                    assert s[r][c] == full[r][c]
    n = dancing.distributed_pentomino(str(tmp_path / "pent"), width=20, height=3, depth=2,
                                      cluster=cluster)
    assert n == dancing.Pentomino(20, 3).solve() == 4


def test_teragen_terasort_teravalidate_cli(tmp_path, cluster):
    assert driver.run("teragen", ["5000", str(tmp_path / "gen"), "--split-rows", "2000"],
                      cluster=cluster) == 0
    gen = np.concatenate([np.fromfile(tmp_path / "gen" / f, dtype=np.uint8).reshape(-1, 100)
                          for f in sorted(os.listdir(tmp_path / "gen"))])
    from hbmr.ops import sort as S
    assert np.array_equal(gen, S.teragen_cpu(0, 5000))
    assert driver.run("terasort", [str(tmp_path / "gen"), str(tmp_path / "sorted"),
                                   "--split-rows", "1500"], cluster=cluster) == 0
    v = T.teravalidate(str(tmp_path / "sorted"))
    assert v["misordered"] == 0 and v["records"] == 5000 and v["files"] == 2
    assert T.teravalidate(str(tmp_path / "gen"))["misordered"] > 0


def test_dbcount_pageview(tmp_path):
    """DBCountPageView over sqlite3: page views per URL add up to the log."""
    import sqlite3
    from hbmr.examples import dbcount
    url = str(tmp_path / "URLAccess.db")
    assert dbcount.main(["sqlite3", url]) == 0
    con = sqlite3.connect(url)
    want = dict(con.execute("SELECT url, COUNT(*) FROM Access GROUP BY url"))
    got = dict(con.execute("SELECT url, pageview FROM Pageview"))
    con.close()
    assert got == want and sum(got.values()) >= 50
