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


def _exact_split_job_centroids(iters):
    conf = JobConf()
    conf.set_boolean(K.EXACT_KEY, True)
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=KC,
                             d=D, inp=f"synthetic:{N}:3", split_points=4000)
        for _ in range(iters):
            drv.step()
        return drv.centroids()


def _pipes_exact(tmp_path, name, conf, gpus, cpu_slots, files=6, block=True, binary=True):
    pts = tmp_path / "pts"
    if not pts.exists():
        KP.write_points(str(pts), N, D, seed=3, centers=KC, files=files, bf16_exact=False)
    init = K.initial_centroids(f"synthetic:{N}:3", KC, D, exact=True)
    with LocalCluster(conf, num_trackers=1, gpus=gpus, cpu_slots=cpu_slots,
                      gpu_slots_per_device=1) as cl:
        drv = KP.KMeansPipesDriver(str(tmp_path / name), str(pts), KC, D, init, cluster=cl,
                                   reduces=1, gpubin=None if not gpus else KP.os.path.join(
                                       KP.BIN, "kmeans_gpu"), exact=True, block=block,
                                   binary=binary)
        cen = drv.run(3)
    return cen, drv.history


def test_pipes_kmeans_exact_cpu_binary_matches_exact_split_job(tmp_path):
    """Exact mode (hbmr.kmeans.exact) through the CPU Pipes binary: the fp64
    arg-min of the fp32 points and fixed-point sums of the fp32 rows — the
    exact split job's centroids, bit for bit."""
    cen, hist = _pipes_exact(tmp_path, "cpu", JobConf(), None, 2)
    assert hist[-1]["counters"].get("KMEANS", "POINTS") == N
    assert torch.equal(cen, _exact_split_job_centroids(3))


def test_pipes_kmeans_block_mode_matches_per_cluster_records(tmp_path):
    """hbmr.kmeans.pipes.block: one partials record per map (in-mapper
    combining) gives the per-cluster records' centroids, bit for bit, with a
    k-th of the map output records; the binary centroid output
    (hbmr.kmeans.pipes.binary.output) reads back the text output's floats."""
    blk, hb = _pipes_exact(tmp_path, "blk", JobConf(), None, 2, block=True, binary=True)
    per, hp = _pipes_exact(tmp_path, "per", JobConf(), None, 2, block=False, binary=False)
    assert torch.equal(blk, per)
    tc = "org.apache.hadoop.mapred.Task$Counter"
    assert hb[-1]["counters"].get(tc, "MAP_OUTPUT_RECORDS") == 6
    assert hp[-1]["counters"].get(tc, "MAP_OUTPUT_RECORDS") > 6


@pytest.mark.gpu
def test_pipes_kmeans_exact_gpu_and_hybrid_are_placement_independent(tmp_path):
    """The GPU binary's exact mode (fp16 MFMA top-3 + certification + fp64
    re-score, fp32 fixed-point sums) emits the CPU binary's partials: an
    all-GPU job, a hybrid job whose maps ran on both kinds of slots, and the
    exact split job give identical centroids.  The GPU maps of a device run
    in one shared child with several maps in flight (hbmr/pipes/mux.py)."""
    from hbmr.pipes import mux
    ref = _exact_split_job_centroids(3)
    mux.REGISTRY.close_all()
    gpu, hg = _pipes_exact(tmp_path, "gpu", JobConf(), [[0]], 0)
    assert torch.equal(gpu, ref)
    assert all(h["counters"].get("KMEANS", "GPU_MAPS") == 6 for h in hg)
    # the shared child kept every split resident after the first iteration
    assert [h["counters"].get("KMEANS", "GPU_SPLIT_CACHE_HITS") for h in hg] == [0, 6, 6]
    children = list(mux.REGISTRY._children.values())
    assert len(children) == 1 and children[0].maps == 18
    conf = JobConf()
    conf.set("hbmr.scheduler.policy", "stock")     # CPU slots take maps too
    hyb, hh = _pipes_exact(tmp_path, "hyb", conf, [[0]], 2)
    cpu_maps = sum(h["counters"].get("KMEANS", "CPU_MAPS") for h in hh)
    gpu_maps = sum(h["counters"].get("KMEANS", "GPU_MAPS") for h in hh)
    assert cpu_maps > 0 and gpu_maps > 0 and cpu_maps + gpu_maps == 18
    assert torch.equal(hyb, ref)
    mux.REGISTRY.close_all()


@pytest.mark.parametrize("compression", ["NONE", "RECORD", "BLOCK"])
def test_pipes_kmeans_cpu_binary_matches_split_job(tmp_path, compression):
    KP.write_points(str(tmp_path / "pts"), N, D, seed=3, centers=KC, files=2,
                    compression=compression)
    init = K.initial_centroids(f"synthetic:{N}:3", KC, D)
    with LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) as cl:
        drv = KP.KMeansPipesDriver(str(tmp_path / "work"), str(tmp_path / "pts"), KC, D, init,
                                   cluster=cl, gpubin=None, reduces=2, exact=False)
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
                                   cluster=cl, reduces=1, exact=False)
        cen = drv.run(3)
    cs = drv.history[-1]["counters"]
    assert cs.get("org.apache.hadoop.mapred.JobInProgress$Counter", "GPU_MAP_TASKS") == 3
    assert cs.get("KMEANS", "GPU_MAPS") == 3
    ref = _split_job_centroids(3)
    # bf16 MFMA distances may flip exact near-ties; centroids agree closely
    assert (cen - ref).abs().max() < 1e-2


def test_native_point_writer_and_reader_match_python_sequencefile(tmp_path):
    from hbmr.io import nativeio
    from hbmr.io import sequencefile as seqf
    x = K.synthetic_points(9, 0, 3000, 12, 4, "cpu").numpy()
    nativeio.write_points(tmp_path / "p.seq", x, first_id=100)
    rows = []
    with seqf.Reader(str(tmp_path / "p.seq")) as r:      # the Python reader reads it
        while True:
            raw = r.next_raw()
            if raw is None:
                break
            rows.append((int.from_bytes(raw[0], "big"), raw[1]))
    assert [k for k, _ in rows] == list(range(100, 3100))
    import numpy as np
    got = np.stack([np.frombuffer(v[4:], dtype=">f4") for _, v in rows]).astype(np.float32)
    assert np.array_equal(got, x)
    size = os.path.getsize(tmp_path / "p.seq")
    # splits by byte range: every record exactly once (SequenceFileRecordReader rule)
    parts = [nativeio.read_points(tmp_path / "p.seq", a, b - a, 12)
             for a, b in [(0, size // 3), (size // 3, 2 * size // 3), (2 * size // 3, size)]]
    assert np.array_equal(np.concatenate(parts), x)


def _file_job_centroids(inp, iters, gpus=None):
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1, gpus=gpus, cpu_slots=0 if gpus else 2) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=KC,
                             d=D, inp=inp, split_points=4000)
        for _ in range(iters):
            assert drv.step()["points"] == N
        return drv.centroids()


def test_kmeans_split_job_on_sequencefile_input_matches_synthetic(tmp_path):
    # the file path (native reader → pinned host → device) sees the same bf16
    # points as the synthetic generator, so the exact partials give equal centroids
    KP.write_points(str(tmp_path / "pts"), N, D, seed=3, centers=KC, files=3)
    assert torch.equal(_file_job_centroids(str(tmp_path / "pts"), 3), _split_job_centroids(3))


def test_kmeans_file_splits_follow_map_count_not_local_blocks(tmp_path):
    """Local SequenceFile input is split about input / mapred.map.tasks (splits
    sized to stay HBM-resident), not once per local-FS block."""
    from hbmr.utils.reflection import new_instance
    KP.write_points(str(tmp_path / "pts"), N, D, seed=3, centers=KC, files=2)
    conf = K.make_iteration_conf(JobConf(), KC, D, str(tmp_path / "pts"), 1000, "c0", "c1")
    conf.set_long("fs.local.block.size", 4096)            # many blocks per file
    conf.set_int("mapred.map.tasks", 2)
    sj = new_instance(conf.get("hbmr.splitjob.class"), conf)
    assert len(sj.get_splits(conf, ["t0"])) == 2
    conf.set_long("mapred.min.split.size", 1 << 40)      # an explicit choice wins
    assert len(sj.get_splits(conf, ["t0"])) == 2
    conf.set_long("mapred.min.split.size", 4096)
    assert len(sj.get_splits(conf, ["t0"])) > 2


@pytest.mark.gpu
def test_gpu_kmeans_split_job_on_sequencefile_input(tmp_path):
    KP.write_points(str(tmp_path / "pts"), N, D, seed=3, centers=KC, files=3)
    got = _file_job_centroids(str(tmp_path / "pts"), 3, gpus=[[0]])
    ref = _file_job_centroids(str(tmp_path / "pts"), 3)
    assert (got - ref).abs().max() < 1e-2      # bf16 MFMA distances on the GPU


@pytest.mark.gpu
def test_gpu_pipes_binary_is_reused_and_keeps_splits_in_hbm(tmp_path):
    from hbmr.pipes.application import POOL
    KP.write_points(str(tmp_path / "pts"), N, D, seed=3, centers=KC, files=3)
    init = K.initial_centroids(f"synthetic:{N}:3", KC, D)
    # one child per slot: with hbmr.gpu.pipes.concurrency > 1 a split finds the
    # child that holds it only when that child is idle (ChildPool prefers it),
    # so every-split hit counts are exact only here
    conf = JobConf()
    conf.set_int("hbmr.gpu.pipes.concurrency", 1)
    conf.set_boolean("hbmr.pipes.gpu.mux", False)       # the per-map child pool path
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0,
                      gpu_slots_per_device=1) as cl:
        drv = KP.KMeansPipesDriver(str(tmp_path / "work"), str(tmp_path / "pts"), KC, D, init,
                                   cluster=cl, reduces=1, exact=False)
        drv.run(3)
        assert POOL.size() >= 1             # the children wait for the next job
    hits = [h["counters"].get("KMEANS", "GPU_SPLIT_CACHE_HITS") for h in drv.history]
    assert hits[0] == 0 and hits[1] == 3 and hits[2] == 3
    POOL.close_all()


def test_native_mapped_reader_matches_stream_reader_on_random_splits(tmp_path, monkeypatch):
    """The mmap fast path of hbmr_seq_read_points keeps the split boundary rule
    of the stdio SequenceFile reader: any cut of the file yields every record
    exactly once, identically on both paths."""
    import numpy as np

    from hbmr.io import nativeio
    x = K.synthetic_points(4, 0, 5000, 16, 4, "cpu").numpy()
    p = tmp_path / "p.seq"
    nativeio.write_points(p, x)
    size = os.path.getsize(p)
    rng = np.random.default_rng(0)
    for trial in range(12):
        cuts = sorted({0, size, *rng.integers(1, size, size=int(rng.integers(1, 9))).tolist()})
        mapped = [nativeio.read_points(p, a, b - a, 16) for a, b in zip(cuts, cuts[1:])]
        monkeypatch.setenv("HBMR_SEQ_NO_MMAP", "1")
        stream = [nativeio.read_points(p, a, b - a, 16) for a, b in zip(cuts, cuts[1:])]
        monkeypatch.delenv("HBMR_SEQ_NO_MMAP")
        assert [m.shape[0] for m in mapped] == [s.shape[0] for s in stream], cuts
        assert np.array_equal(np.concatenate(mapped), x), trial
