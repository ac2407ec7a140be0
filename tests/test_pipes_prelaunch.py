"""Bulk-launched GPU Pipes maps are sent to the device's shared child ahead
of their task threads (TaskTracker._prelaunch_pipes, mux.MuxChild.prelaunch):
the threads take over their maps' messages and the job's answer is the one
the ordinary per-thread submit gives.  Simulated GPU slots on CPU, the CPU
K-Means binary standing in for the GPU executable (same protocol)."""
import os

import pytest

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K
from hbmr.models import kmeans_pipes as KP

CPUBIN = os.path.join(KP.BIN, "kmeans_cpu")


def _run(tmp_path, name, prelaunch):
    pts = str(tmp_path / "pts")
    if not os.path.exists(pts):
        KP.write_points(pts, 4000, 128, seed=5, centers=16, files=8)
    init = K.initial_centroids(pts, 16, 128)
    conf = JobConf()
    conf.set_int("hbmr.gpu.queue.depth", 16)
    conf.set("hbmr.gpu.simulate", "true")
    conf.set_boolean("hbmr.pipes.gpu.prelaunch", prelaunch)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0,
                      gpu_slots_per_device=1) as cl:
        drv = KP.KMeansPipesDriver(str(tmp_path / name), pts, 16, 128, init, base=conf,
                                   cluster=cl, gpubin=CPUBIN, maps=8, exact=True)
        for _ in range(3):
            drv.step()
        gpu_maps = drv.history[-1]["counters"].get(
            "org.apache.hadoop.mapred.JobInProgress$Counter", "GPU_MAP_TASKS")
        return drv.centroids, gpu_maps


@pytest.mark.skipif(not os.path.exists(CPUBIN), reason="native apps not built")
def test_prelaunched_maps_give_the_ordinary_answer(tmp_path, monkeypatch):
    import torch

    from hbmr.pipes import mux
    sent = []
    real = mux.MuxChild.prelaunch

    def counting(self, *a, **kw):
        t = real(self, *a, **kw)
        sent.append(t is not None)
        return t
    monkeypatch.setattr(mux.MuxChild, "prelaunch", counting)
    a, ga = _run(tmp_path, "pre", True)
    assert sum(sent) >= 16                # most of the 3 x 8 maps went ahead
    assert not mux.PRELAUNCHED            # every prelaunched map was taken over
    sent.clear()
    b, gb = _run(tmp_path, "plain", False)
    assert ga == gb == 8
    assert torch.equal(a, b)
