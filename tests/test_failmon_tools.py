"""Failmon parsers (contrib/failmon) with a synthetic amdgpu sysfs, Logalyzer
and DistCh (src/tools)."""
from __future__ import annotations

import os
import stat

from hbmr.tools import distch, logalyzer
from hbmr.utils import failmon


def _fake_card(root, n, temp_mc=45000, umc="ue: 0\nce: 0\n", xgmi="ue: 0\nce: 3\n"):
    dev = root / f"card{n}" / "device"
    (dev / "hwmon" / "hwmon9").mkdir(parents=True)
    (dev / "ras").mkdir()
    (dev / "vendor").write_text("0x1002\n")
    (dev / "gpu_busy_percent").write_text("87\n")
    (dev / "mem_info_vram_used").write_text(str(100 << 30))
    (dev / "mem_info_vram_total").write_text(str(288 << 30))
    hw = dev / "hwmon" / "hwmon9"
    (hw / "temp1_input").write_text(str(temp_mc))
    (hw / "temp1_label").write_text("junction")
    (hw / "power1_average").write_text(str(650 * 10**6))
    (dev / "ras" / "umc_err_count").write_text(umc)
    (dev / "ras" / "xgmi_wafl_err_count").write_text(xgmi)


def test_gpu_parser_levels(tmp_path):
    drm = tmp_path / "drm"
    _fake_card(drm, 0)
    _fake_card(drm, 1, temp_mc=101000)
    _fake_card(drm, 2, umc="ue: 2\nce: 7\n")
    (drm / "renderD128").mkdir(parents=True)
    recs = failmon.GPUParser(str(drm)).query()
    by = {r["properties"]["card"]: r for r in recs}
    assert by["card0"]["logLevel"] == "WARN" and "xgmi_wafl" in by["card0"]["message"]
    assert by["card0"]["properties"]["temp_junction"] == 45.0
    assert by["card0"]["properties"]["power_w"] == 650.0
    assert by["card1"]["logLevel"] == "WARN" and "junction 101C" in by["card1"]["message"]
    assert by["card2"]["logLevel"] == "ERROR" and by["card2"]["properties"]["ras_umc_ue"] == 2


def test_run_once_store_logs_and_anonymizer(tmp_path):
    log = tmp_path / "hbmr-tasktracker.log"
    log.write_text("2026 INFO ok\n2026 WARN slow heartbeat from 10.1.2.3\n2026 ERROR boom\n")
    store = failmon.LocalStore(str(tmp_path / "ev.jsonl"), anonymize_records=True)
    lp = failmon.LogParser([str(tmp_path / "*.log")])
    recs = failmon.run_once(store, [failmon.CPUParser(), failmon.NICParser(), lp])
    levels = [r["logLevel"] for r in recs if r["type"] == "LOG"]
    assert levels == ["WARN", "ERROR"]
    stored = store.read()
    assert len(stored) == len(recs)
    warn = [r for r in stored if r["type"] == "LOG"][0]
    assert "10.1.2.3" not in warn["message"] and warn["hostname"] != failmon.HOST
    assert lp.query() == []          # offsets remembered: nothing new
    with open(log, "a") as f:
        f.write("2026 FATAL gone\n")
    assert [r["logLevel"] for r in lp.query()] == ["FATAL"]
    c = failmon.Continuous(store, [failmon.CPUParser()], interval=0.05).start()
    import time
    time.sleep(0.3)
    c.stop()
    assert c.rounds >= 2


def test_logalyzer_archive_and_analyze(tmp_path):
    logs = tmp_path / "logs"
    logs.mkdir()
    (logs / "a.log").write_text("2026-10-16 INFO JobTracker started\n"
                                "2026-10-16 WARN TaskTracker lost\n"
                                "2026-10-17 WARN TaskTracker lost\n")
    (logs / "b.log").write_text("2026-10-16 WARN DataNode slow\n")
    arch = str(tmp_path / "archive")
    logalyzer.archive([str(logs)], arch)
    out = str(tmp_path / "out")
    logalyzer.analyze(arch, out, grep="WARN", sort_columns="1,2", separator=" ")
    rows = dict(ln.rstrip("\n").split("\t") for ln in open(os.path.join(out, "part-00000")))
    assert rows == {"WARN TaskTracker": "2", "WARN DataNode": "1"}


def test_distch_permissions(tmp_path):
    d = tmp_path / "tree"
    (d / "sub").mkdir(parents=True)
    for p in (d / "f", d / "sub" / "g"):
        p.write_text("x")
    rj = distch.change([f"{d}:::750"])
    assert rj.getCounters().get("distch", "SUCCEED") == 4
    for p in (d, d / "sub", d / "f", d / "sub" / "g"):
        assert stat.S_IMODE(os.stat(p).st_mode) == 0o750
    import pytest
    with pytest.raises(ValueError):
        distch.parse_op("hdfs://nn/x:::700")
    with pytest.raises(ValueError):
        distch.parse_op(f"{d}:::79")


import pytest  # noqa: E402


@pytest.mark.gpu
def test_gpu_parser_on_real_node():
    """On the MI355X box: the amdgpu sysfs is read (skipped where the container
    does not expose /sys/class/drm)."""
    p = failmon.GPUParser()
    if not p.cards():
        pytest.skip("no amdgpu sysfs visible in this container")
    recs = p.query()
    assert recs and all(r["type"] == "GPU" for r in recs)
    print([(r["properties"].get("card"), r["properties"].get("vram_total"),
            r["logLevel"]) for r in recs])
