"""PiEstimator: classic record job vs the split-level job (CPU slots here; the
GPU Halton kernel bit-exact against the numpy map on the MI355X)."""
from __future__ import annotations

import pytest
import torch

from hbmr.examples import pi
from hbmr.mapred import JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.ops import pi as P


def _run_split(cl, maps, samples):
    rj = cl.submit_job(pi.split_job_conf(maps, samples))
    rj.waitForCompletion(timeout=120)
    assert rj.isSuccessful(), rj.getFailureInfo()
    return rj._impl.jip.result[0]


def test_split_job_matches_classic_job_on_cpu_slots():
    conf = JobConf()
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        res = _run_split(cl, maps=4, samples=20000)
    classic = pi.estimate(4, 20000)
    assert res["total"] == 80000
    assert str(classic) == res["pi"]
    assert abs(float(res["pi"]) - 3.14159) < 1e-3


@pytest.mark.gpu
def test_gpu_halton_count_bit_exact():
    for off, n in [(0, 1), (0, 100_000), (123_456_789, 250_000), ((1 << 40) + 7, 65_537)]:
        g = P.count_inside_gpu(off, n)
        torch.cuda.synchronize()
        assert int(g.item()) == P.count_inside_cpu(off, n), (off, n)


@pytest.mark.gpu
def test_gpu_pi_split_job():
    conf = JobConf()
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        res = _run_split(cl, maps=8, samples=2_000_000)
    exp = sum(P.count_inside_cpu(i * 2_000_000, 2_000_000) for i in range(8))
    assert res["inside"] == exp and res["total"] == 16_000_000
