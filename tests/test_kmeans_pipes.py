"""K-Means through the Pipes task binaries (native/apps/kmeans_{cpu,gpu}) —
BASELINE config 2.  The C++ side reads SequenceFile splits itself
(native/io/sequencefile.cc, incl. RECORD/BLOCK zlib compression) and emits
int64 fixed-point partials, so its centroids equal the in-process split job's
bit for bit."""
import os

import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K
from hbmr.models import kmeans_pipes as KP

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _built():
    import importlib.util
    spec = importlib.util.spec_from_file_location("nb", os.path.join(ROOT, "native", "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.build()


N, D, KC = 12000, 16, 6


def _split_job_centroids(iters):
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=KC,
                             d=D, inp=f"synthetic:{N}:3", split_points=4000)
        for _ in range(iters):
            drv.step()
        return drv.centroids()


@pytest.mark.parametrize("compression", ["NONE", "RECORD", "BLOCK"])
def test_pipes_kmeans_cpu_binary_matches_split_job(tmp_path, compression):
    KP.write_points(str(tmp_path / "pts"), N, D, seed=3, centers=KC, files=2,
                    compression=compression)
    init = K.initial_centroids(f"synthetic:{N}:3", KC, D)
    with LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) as cl:
        drv = KP.KMeansPipesDriver(str(tmp_path / "work"), str(tmp_path / "pts"), KC, D, init,
                                   cluster=cl, gpubin=None, reduces=2)
        cen = drv.run(3)
    cs = drv.history[-1]["counters"]
    assert cs.get("KMEANS", "POINTS") == N
    assert torch.equal(cen, _split_job_centroids(3))


@pytest.mark.gpu
def test_pipes_kmeans_gpu_binary_on_gpu_slots(tmp_path):
    KP.write_points(str(tmp_path / "pts"), N, D, seed=3, centers=KC, files=3)
    init = K.initial_centroids(f"synthetic:{N}:3", KC, D)
    with LocalCluster(JobConf(), num_trackers=1, gpus=[[0]], cpu_slots=0,
                      gpu_slots_per_device=1) as cl:
        drv = KP.KMeansPipesDriver(str(tmp_path / "work"), str(tmp_path / "pts"), KC, D, init,
                                   cluster=cl, reduces=1)
        cen = drv.run(3)
    cs = drv.history[-1]["counters"]
    assert cs.get("org.apache.hadoop.mapred.JobInProgress$Counter", "GPU_MAP_TASKS") == 3
    assert cs.get("KMEANS", "GPU_MAPS") == 3
    ref = _split_job_centroids(3)
    # bf16 MFMA distances may flip exact near-ties; centroids agree closely
    assert (cen - ref).abs().max() < 1e-2
