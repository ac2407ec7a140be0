"""K-Means jobs through the full runtime on a GPU tracker (MI355X)."""
import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K

JOB = "org.apache.hadoop.mapred.JobInProgress$Counter"


def _one_step(conf, gpu, inp, k, d, sp, iters=1):
    kw = dict(num_trackers=1, gpus=[[0]], cpu_slots=0) if gpu else dict(num_trackers=1,
                                                                        cpu_slots=2)
    with LocalCluster(conf, **kw) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=k,
                             d=d, inp=inp, split_points=sp)
        for _ in range(iters):
            r = drv.step()
        return drv.centroids().clone(), r


@pytest.mark.gpu
def test_gpu_kmeans_job_matches_cpu_job():
    """bf16 GPU map vs fp32 CPU map from the same centroids: they may only
    differ by the points whose assignment flips (the GPU scores bf16-rounded
    centroids); the centroid difference is bounded by what those flips can
    move, counted directly with both kernels."""
    from hbmr.ops import kmeans as km
    n, k, d, sp = 60000, 16, 128, 15000
    inp = f"synthetic:{n}:5"
    gpu_cen, r = _one_step(JobConf(), True, inp, k, d, sp)
    assert r["points"] == n
    assert r["counters"].get(JOB, "GPU_MAP_TASKS") == 4
    cpu_cen, _ = _one_step(JobConf(), False, inp, k, d, sp)
    # the points as stored (bf16) and the two kernels' labels from the initial centroids
    x = K.synthetic_points(5, 0, n, d, k, "cuda").to(torch.bfloat16)
    c0 = K.initial_centroids(inp, k, d)
    lab_g = km.assign(x.contiguous(), km.CentroidImage(c0, "cuda")).cpu()
    lab_c = torch.empty(n, dtype=torch.int32)
    xs, cs = torch.zeros(k, d, dtype=torch.int64), torch.zeros(k, dtype=torch.int64)
    km.map_split_cpu(x.float().cpu(), c0, xs, cs, labels=lab_c)
    flips = int((lab_g != lab_c).sum())
    xf = x.float().cpu()
    reach = float(xf.norm(dim=1).max()) + float(torch.maximum(gpu_cen.norm(dim=1).max(),
                                                              cpu_cen.norm(dim=1).max()))
    cnt = torch.bincount(lab_c.long(), minlength=k).clamp(min=1).float()
    # a flip moves its old and its new centroid by at most reach / (count - flips)
    bound = flips * reach / max(1.0, float(cnt.min()) - flips) + 1e-5
    diff = (gpu_cen - cpu_cen).abs().max().item()
    assert diff <= bound, (diff, bound, flips)
    if flips == 0:
        assert diff < 1e-5


@pytest.mark.gpu
def test_gpu_exact_kmeans_job_equals_cpu_exact_job():
    """Exact mode on both slot types is the fp64 assignment of the fp32 data:
    GPU and CPU jobs give the same centroids (to the 2^-24 fixed-point grid)."""
    n, k, d, sp = 60000, 16, 128, 15000
    inp = f"synthetic:{n}:5"
    confs = []
    for _ in range(2):
        c = JobConf()
        c.set_boolean(K.EXACT_KEY, True)
        confs.append(c)
    g, r = _one_step(confs[0], True, inp, k, d, sp, iters=3)
    c, _ = _one_step(confs[1], False, inp, k, d, sp, iters=3)
    assert (g - c).abs().max().item() < 1e-5
    assert r["counters"].get(JOB, "GPU_MAP_TASKS") == 4


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


@pytest.mark.gpu
def test_gpu_first_chunk_handoff_gives_same_result():
    """hbmr.gpu.first.chunk.handoff.ms > 0 (the submitter of an idle device's
    first chunk waits until it is launched) changes only launch timing: the
    iteration's centroids equal those of the default launch path."""
    n, k, d, sp = 120000, 16, 128, 5000      # 24 maps: a first chunk of 4 + the rest
    inp = f"synthetic:{n}:9"
    base, r0 = _one_step(JobConf(), True, inp, k, d, sp, iters=2)
    conf = JobConf()
    conf.set("hbmr.gpu.first.chunk.handoff.ms", "2.0")
    got, r1 = _one_step(conf, True, inp, k, d, sp, iters=2)
    assert r1["counters"].get(JOB, "GPU_MAP_TASKS") == n // sp
    assert torch.equal(base, got)


@pytest.mark.gpu
def test_gpu_device_time_does_not_double_count_overlapping_slots():
    """Two GPU slots (streams) run a job's batches concurrently; the tasks'
    device time (GPU_KERNEL_US, the cost model's t_gpu) sums to the device's
    busy time, which cannot exceed the job's wall time."""
    import time
    n, k, d, sp = 1_600_000, 256, 128, 50_000      # 32 maps over 2 slots
    inp = f"synthetic:{n}:4"
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0,
                      gpu_slots_per_device=2) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=k,
                             d=d, inp=inp, split_points=sp)
        drv.step()                                  # splits materialised in HBM
        t0 = time.perf_counter()
        r = drv.step()
        wall_us = (time.perf_counter() - t0) * 1e6
    assert r["counters"].get(JOB, "GPU_MAP_TASKS") == n // sp
    busy_us = r["counters"].get("hbmr.GpuCounters", "GPU_KERNEL_US")
    assert 0 < busy_us <= wall_us * 1.02, (busy_us, wall_us)
