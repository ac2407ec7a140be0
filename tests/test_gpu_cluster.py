"""K-Means jobs through the full runtime on a GPU tracker (MI355X)."""
import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K

JOB = "org.apache.hadoop.mapred.JobInProgress$Counter"


@pytest.mark.gpu
def test_gpu_kmeans_job_matches_cpu_job():
    n, k, d, sp = 60000, 16, 128, 15000
    inp = f"synthetic:{n}:5"

    conf = JobConf()
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=k,
                             d=d, inp=inp, split_points=sp)
        for _ in range(3):
            r = drv.step()
        assert r["points"] == n
        assert r["counters"].get(JOB, "GPU_MAP_TASKS") == 4
        gpu_cen = drv.centroids().clone()

    conf2 = JobConf()
    with LocalCluster(conf2, num_trackers=1, cpu_slots=2) as cl:
        drv2 = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf2,
                              k=k, d=d, inp=inp, split_points=sp)
        for _ in range(3):
            drv2.step()
        cpu_cen = drv2.centroids()
    # same bf16 data, same fixed-point partials; only near-tie assignments may
    # differ (MFMA fp32 accumulation order vs the CPU's dot products), moving a
    # centroid by ~|x|/count per flipped point
    # (the GPU also scores against bf16-rounded centroids, the CPU against fp32)
    diff = (gpu_cen - cpu_cen).abs()
    assert diff.mean().item() < 2e-2 and diff.max().item() < 1.0, (diff.mean(), diff.max())


@pytest.mark.gpu
def test_hybrid_scheduler_profiles_then_prefers_gpu():
    conf = JobConf()
    conf.set("hbmr.scheduler.policy", "hybrid")
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=2) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=256,
                             d=128, inp="synthetic:2000000:9", split_points=100000)
        first = drv.step()
        for _ in range(3):
            last = drv.step()
        # after profiling, the min-makespan rule leaves CPU slots idle for this job
        assert last["counters"].get(JOB, "CPU_MAP_TASKS") == 0
        assert last["counters"].get(JOB, "GPU_MAP_TASKS") == 20
        cm = cl.jt.cost_model.snapshot()
        sig = next(iter(cm))
        assert cm[sig]["gpu"]["n"] >= 20
        _ = first


@pytest.mark.gpu
def test_split_cache_hits_after_first_iteration():
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=64,
                             d=128, inp="synthetic:400000:2", split_points=100000)
        r1 = drv.step()
        r2 = drv.step()
        g = "hbmr.GpuCounters"
        assert r1["counters"].get(g, "GPU_SPLIT_CACHE_MISSES") == 4
        assert r2["counters"].get(g, "GPU_SPLIT_CACHE_HITS") == 4
        assert r2["counters"].get(g, "GPU_SPLIT_CACHE_MISSES") == 0
        assert torch.cuda.is_available()
