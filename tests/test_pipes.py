"""Pipes: the C++ child runtime (libhbmr_pipes) + Python parent side, end to end.

Mirrors the reference's TestPipes (src/test/org/apache/hadoop/mapred/pipes/
TestPipes.java:84-217): wordcount-simple with Java record reader/writer,
wordcount-part with a C++ partitioner, wordcount-nopipe with C++ reader/writer.
"""
import collections
import os

import pytest

from hbmr.mapred import FileInputFormat, FileOutputFormat, JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.pipes import submitter
from hbmr.pipes.protocol import create_digest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hbmr", "bin")


@pytest.fixture(scope="module", autouse=True)
def _built():
    import importlib.util
    spec = importlib.util.spec_from_file_location("nb", os.path.join(ROOT, "native", "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.build()


def _input(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    cnt = collections.Counter()
    for i in range(2):
        lines = [" ".join(f"w{(j * 7 + t * 3 + i) % 13}" for t in range(j % 6)) for j in range(300)]
        (inp / f"f{i}.txt").write_text("\n".join(lines) + "\n")
        for line in lines:
            cnt.update(line.split())
    return inp, cnt


def _read(out, sep="\t"):
    res = {}
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            for line in open(os.path.join(out, fn)):
                k, v = line.rstrip("\n").split(sep)
                res[k] = int(v)
    return res


def test_hmac_digest_matches_reference_algorithm():
    # base64(HMAC-SHA1(key, msg)) — RFC 2202 test case 2
    import base64
    d = create_digest(b"Jefe", "what do ya want for nothing?")
    assert base64.b64decode(d).hex() == "effcdf6ae5eb2fa2d27416d5f184df9c259a7c79"


def _job(tmp_path, exe, reduces=2, java_rr=True, java_rw=True):
    inp, cnt = _input(tmp_path)
    out = tmp_path / "out"
    conf = JobConf()
    FileInputFormat.setInputPaths(conf, str(inp))
    FileOutputFormat.setOutputPath(conf, str(out))
    conf.set_boolean("hadoop.pipes.java.recordreader", java_rr)
    conf.set_boolean("hadoop.pipes.java.recordwriter", java_rw)
    conf.set_num_reduce_tasks(reduces)
    conf.set_num_map_tasks(3)
    submitter.set_executable(conf, os.path.join(BIN, exe))
    return conf, out, cnt


def test_pipes_wordcount_simple_local(tmp_path):
    conf, out, cnt = _job(tmp_path, "wordcount-simple")
    rj = submitter.run_job(conf, verbose=False)
    assert rj.isSuccessful(), rj.getFailureInfo()
    assert _read(out) == dict(cnt)
    cs = rj.getCounters()
    assert cs.get("WORDCOUNT", "INPUT_WORDS") == sum(cnt.values())
    # the reducer class doubles as the combiner, so map-side combines count too
    assert cs.get("WORDCOUNT", "OUTPUT_WORDS") >= len(cnt)


def test_pipes_wordcount_part_partitioner(tmp_path):
    conf, out, cnt = _job(tmp_path, "wordcount-part", reduces=3)
    rj = submitter.run_job(conf, verbose=False)
    assert rj.isSuccessful(), rj.getFailureInfo()
    assert _read(out) == dict(cnt)
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            r = int(fn[5:])
            for line in open(out / fn):
                assert ord(line[0]) % 3 == r


def test_pipes_wordcount_nopipe_cpp_reader_writer(tmp_path):
    conf, out, cnt = _job(tmp_path, "wordcount-nopipe", reduces=1, java_rr=False, java_rw=False)
    rj = submitter.run_job(conf, verbose=False)
    assert rj.isSuccessful(), rj.getFailureInfo()
    res = {}
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            for line in open(out / fn):
                k, v = line.rstrip("\n").split(" -> ")
                res[k] = int(v)
    assert res == dict(cnt)


def test_pipes_on_cluster_two_trackers(tmp_path):
    conf, out, cnt = _job(tmp_path, "wordcount-simple", reduces=2)
    with LocalCluster(JobConf(), num_trackers=2) as cl:
        rj = submitter.run_job(conf, cluster=cl, verbose=False)
        assert rj.isSuccessful(), rj.getFailureInfo()
    assert _read(out) == dict(cnt)


def test_gpu_only_job_is_accepted_and_not_placed_on_cpu(tmp_path):
    conf, out, cnt = _job(tmp_path, "wordcount-simple")
    conf.unset("hadoop.pipes.executable")
    submitter.set_gpu_executable(conf, os.path.join(BIN, "wordcount-simple"))
    submitter.setup_pipes_job(conf)   # the fork crashed here (B3)
    assert conf.get_boolean("hbmr.job.cpu.capable", True) is False
    assert conf.is_gpu_capable()


def test_text_protocol_debug_mode():
    """No command port/file in the environment: the C++ child speaks the text
    protocol on stdin/stdout (HadoopPipes.cc TextProtocol), map and reduce."""
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parent.parent / "hbmr" / "bin" / "wordcount-simple"
    env = {k: v for k, v in os.environ.items() if not k.startswith("hadoop.pipes.")}
    m = subprocess.run([str(exe)], input="start\t0\nsetJobConf\tx\ty\nrunMap\ts\t1\t1\n"
                       "mapItem\t0\ta b\\ta\nclose\n", capture_output=True, text=True,
                       env=env, timeout=30)
    assert m.returncode == 0, m.stderr
    lines = m.stdout.splitlines()
    assert lines[-1] == "done"
    # one reduce → the in-child combiner folds the map output (escaped \t = a tab)
    assert sorted(ln for ln in lines if ln.startswith("output")) == \
        ["output\ta\t2", "output\tb\t1"]
    r = subprocess.run([str(exe)], input="start\t0\nrunReduce\t0\t1\nreduceKey\ta\n"
                       "reduceValue\t1\nreduceValue\t2\nreduceKey\tb\nreduceValue\t5\nclose\n",
                       capture_output=True, text=True, env=env, timeout=30)
    assert r.returncode == 0, r.stderr
    assert [ln for ln in r.stdout.splitlines() if ln.startswith("output")] == \
        ["output\ta\t3", "output\tb\t5"]


def test_pipes_default_debug_script_reports_core(tmp_path):
    """Executables given as <path>#<name> get the default gdb-style debug
    script (Submitter.java:341-347): a failed attempt's diagnostics carry the
    core file found in the Pipes child's working directory."""
    crash = tmp_path / "crasher"
    crash.write_text("#!/bin/sh\necho dying >&2\necho fake > core.4242\nexit 3\n")
    crash.chmod(0o755)
    conf, out, _ = _job(tmp_path, "wordcount-simple", reduces=1)
    conf.unset("hadoop.pipes.executable")
    submitter.set_executable(conf, f"{crash}#crasher")
    conf.set("hbmr.local.scratch", str(tmp_path / "scratch"))
    conf.set_int("mapred.map.max.attempts", 1)
    conf.set_num_map_tasks(1)
    submitter.setup_pipes_job(conf)
    assert conf.get("hadoop.pipes.executable") == str(crash)
    assert conf.get("mapred.map.task.debug.script") == submitter.DEFAULT_DEBUG_SCRIPT
    with LocalCluster(JobConf(), num_trackers=1) as cl:
        rj = submitter.submit_job(conf, cluster=cl)
        rj.waitForCompletion(60)
        assert not rj.isSuccessful()
        jip = rj._impl.jip
        diags = [a.diagnostic for t in jip.maps for a in t.attempts.values() if a.diagnostic]
    text = "\n".join(diags)
    assert "Debug script output" in text and "core file:" in text and "core.4242" in text
    assert "dying" in text          # the child's stderr tail
