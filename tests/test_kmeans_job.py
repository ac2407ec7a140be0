"""K-Means as chained MapReduce jobs on the in-process cluster (CPU slots here;
the GPU variant is in test_gpu_cluster.py)."""
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K


def _reference_lloyd(x, c, iters):
    for _ in range(iters):
        lab = torch.cdist(x.double(), c.double()).argmin(1)
        s = torch.zeros_like(c, dtype=torch.float64).index_add_(0, lab, x.double())
        n = torch.bincount(lab, minlength=c.shape[0]).double()[:, None]
        c = torch.where(n > 0, s / n.clamp(min=1), c.double()).float()
    return c


def test_synthetic_generator_deterministic_and_split_invariant():
    a = K.synthetic_points(5, 0, 1000, 16, 4, "cpu")
    b = torch.cat([K.synthetic_points(5, 0, 400, 16, 4, "cpu"),
                   K.synthetic_points(5, 400, 600, 16, 4, "cpu")])
    assert torch.equal(a, b)
    assert a.std() > 3  # a mixture, not plain noise


def _run(num_trackers, iters=4, split_points=2500, n=10000, k=6, d=16, policy="hybrid"):
    conf = JobConf()
    conf.set("hbmr.scheduler.policy", policy)
    with LocalCluster(conf, num_trackers=num_trackers, cpu_slots=2) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf,
                             k=k, d=d, inp=f"synthetic:{n}:3", split_points=split_points)
        for _ in range(iters):
            r = drv.step()
            assert r["points"] == n
        return drv, drv.centroids()


def test_kmeans_cpu_matches_reference():
    n, k, d, iters = 10000, 6, 16, 4
    drv, cen = _run(1, iters=iters, n=n, k=k, d=d)
    x = K.synthetic_points(3, 0, n, d, k, "cpu").to(torch.bfloat16).float()
    c0 = K.initial_centroids(f"synthetic:{n}:3", k, d)
    ref = _reference_lloyd(x, c0, iters)
    assert torch.allclose(cen, ref, atol=1e-4), (cen - ref).abs().max()
    assert len(drv.history) == iters
    # every map ran on a CPU slot (no GPUs here)
    cs = drv.history[-1]["counters"]
    assert cs.get("org.apache.hadoop.mapred.JobInProgress$Counter", "CPU_MAP_TASKS") == 4


def test_kmeans_two_trackers_collective_reduce_is_exact():
    _, c1 = _run(1, iters=3)
    _, c2 = _run(2, iters=3)
    # fixed-point partials: identical bits regardless of tracker count/placement
    assert torch.equal(c1, c2)
