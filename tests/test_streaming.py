"""Hadoop Streaming equivalent (contrib/streaming): external commands as
mapper/combiner/reducer over text stdin/stdout."""
import collections
import os
import sys

import pytest

from hbmr import streaming
from hbmr.mapred import JobClient
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf

PY = sys.executable
MAPPER = f"{PY} -c \"import sys\nfor l in sys.stdin:\n  [print(w + chr(9) + '1') for w in l.split()]\""
REDUCER = (f"{PY} -c \"import sys\nc={{}}\nfor l in sys.stdin:\n  k,v=l.rstrip(chr(10)).split(chr(9))\n"
           f"  c[k]=c.get(k,0)+int(v)\nfor k in c: print(k+chr(9)+str(c[k]))\n"
           f"sys.stderr.write('reporter:counter:Stream,Keys,%d' % len(c) + chr(10))\"")


def _input(tmp_path):
    d = tmp_path / "in"
    d.mkdir()
    cnt = collections.Counter()
    for i in range(2):
        lines = [" ".join(f"s{(i + j + t) % 7}" for t in range(j % 4)) for j in range(120)]
        (d / f"f{i}").write_text("\n".join(lines) + "\n")
        for ln in lines:
            cnt.update(ln.split())
    return d, cnt


def _read(out):
    res = {}
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            for line in open(os.path.join(out, fn)):
                k, v = line.rstrip("\n").split("\t")
                res[k] = int(v)
    return res


@pytest.mark.parametrize("use_cluster", [False, True])
def test_streaming_wordcount(tmp_path, use_cluster):
    inp, cnt = _input(tmp_path)
    args = ["-input", str(inp), "-output", str(tmp_path / "out"), "-mapper", MAPPER,
            "-combiner", REDUCER, "-reducer", REDUCER, "-numReduceTasks", "2"]
    job = streaming.stream_job_conf(args)
    cl = LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) if use_cluster else None
    try:
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
    finally:
        if cl:
            cl.shutdown()
    assert _read(tmp_path / "out") == dict(cnt)
    assert rj.getCounters().get("Stream", "Keys") >= len(cnt)


def test_streaming_map_only_cat_and_failure(tmp_path):
    inp, _ = _input(tmp_path)
    job = streaming.stream_job_conf(["-input", str(inp), "-output", str(tmp_path / "o"),
                                     "-mapper", "cat", "-reducer", "NONE"])
    JobClient.runJob(job, verbose=False)
    lines = []
    for fn in sorted(os.listdir(tmp_path / "o")):
        if fn.startswith("part-"):
            lines += open(tmp_path / "o" / fn).read().splitlines()
    src = (inp / "f0").read_text().splitlines() + (inp / "f1").read_text().splitlines()
    assert sorted(ln.rstrip("\t") for ln in lines) == sorted(src)
    bad = streaming.stream_job_conf(["-input", str(inp), "-output", str(tmp_path / "o2"),
                                     "-mapper", "false", "-reducer", "NONE"])
    with pytest.raises(RuntimeError):
        JobClient.runJob(bad, verbose=False)
