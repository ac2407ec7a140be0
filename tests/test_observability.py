"""Observability: web UI (cluster/job pages, GPU-coloured task graph, Perfetto
timeline, Prometheus metrics), job history files + summary/diagnosis, CLI."""
import json
import os
import urllib.request

import pytest

from hbmr import cli
from hbmr.examples.sleepjob import split_sleep_conf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.webui.history import summarize_history
from hbmr.webui.server import CPU_COLOR, GPU_COLOR, WebUI


def _get(url):
    with urllib.request.urlopen(url, timeout=10) as r:
        return r.read().decode()


def test_webui_history_and_metrics(tmp_path):
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 1)
    conf.set_float("hbmr.gpu.simulate.task.ms", 2)
    conf.set("hbmr.history.dir", str(tmp_path / "hist"))
    conf.set("hbmr.scheduler.policy", "stock")
    conf.set_int("hbmr.gpu.queue.depth", 1)
    with LocalCluster(conf, num_trackers=2, gpus=[[0], [1]], cpu_slots=1) as cl:
        ui = WebUI(cl.jt, port=0).start()
        try:
            rj = cl.submit_job(split_sleep_conf(24, map_ms=3, base=conf))
            rj.waitForCompletion(60)
            assert rj.isSuccessful()
            jid = str(rj.getID())
            page = _get(ui.url)
            assert "tracker_0" in page and jid in page
            assert "Map tasks" in _get(ui.url + f"jobdetails?jobid={jid}")
            svg = _get(ui.url + f"taskgraph?jobid={jid}&type=map")
            assert GPU_COLOR in svg and CPU_COLOR in svg
            trace = json.loads(_get(ui.url + f"timeline?jobid={jid}"))
            names = {e["args"]["name"] for e in trace["traceEvents"] if e["ph"] == "M"}
            assert any("gpu" in n for n in names)
            metrics = _get(ui.url + "metrics")
            assert 'hbmr_tasks_launched_total{type="map",where="gpu"}' in metrics
            assert "hbmr_trackers 2.0" in metrics
            api = json.loads(_get(ui.url + f"api/job?jobid={jid}"))
            assert api["cpu_maps"] + api["gpu_maps"] == 24
        finally:
            ui.stop()
    files = os.listdir(tmp_path / "hist")
    assert files == [f"{jid}.jsonl"]
    s = summarize_history(str(tmp_path / "hist" / files[0]))
    assert s["maps"] == 24 and s["state"] == "SUCCEEDED"
    assert s["gpu_map_time"]["n"] + s["cpu_map_time"]["n"] == 24
    assert any(d["rule"] == "acceleration" for d in s["diagnosis"])
    # CLI: hbmr job -history
    assert cli.main(["job", "-history", str(tmp_path / "hist" / files[0])]) == 0


def test_cli_fs_and_version(tmp_path, capsys):
    (tmp_path / "a.txt").write_text("hello\n")
    assert cli.main(["version"]) == 0
    assert cli.main(["fs", "-mkdir", str(tmp_path / "d")]) == 0
    assert cli.main(["fs", "-put", str(tmp_path / "a.txt"), str(tmp_path / "d")]) == 0
    assert cli.main(["fs", "-cat", str(tmp_path / "d" / "a.txt")]) == 0
    assert cli.main(["fs", "-ls", str(tmp_path / "d")]) == 0
    out = capsys.readouterr().out
    assert "hello" in out and "Found 1 items" in out
    assert cli.main(["fs", "-rmr", str(tmp_path / "d")]) == 0
    assert not (tmp_path / "d").exists()


def test_roctx_markers_when_requested():
    """HBMR_ROCTX=1 turns tracer events into roctx marks / ranges (libroctx64)
    for rocprofv3 --marker-trace timelines; without it the tracer stays off."""
    import subprocess
    import sys
    code = ("from hbmr.utils.trace import TRACE\n"
            "TRACE.instant('job.submit', job='j1')\n"
            "with TRACE.span('reduce', n=3):\n    pass\n"
            "print(TRACE.on, TRACE.roctx.lib is not None, len(TRACE.events))\n")
    env = dict(os.environ, HBMR_ROCTX="1", PYTHONPATH=os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    on, lib, n = out.stdout.split()
    assert on == "True" and n == "2"
    if lib != "True":
        pytest.skip("libroctx64 not installed")
    env.pop("HBMR_ROCTX")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.stdout.split()[:2] == ["False", "False"]
