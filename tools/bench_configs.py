"""Benchmarks of the BASELINE.json configs other than the headline one.

  python tools/bench_configs.py wordcount    [--mb 64]                   # config 1
  python tools/bench_configs.py kmeans-pipes [--points 1000000 --k 64]   # config 2
  python tools/bench_configs.py mrbench      [--jobs 20]                 # job-launch latency
  python tools/bench_configs.py wordcount-gpu [--mb 1024 --files 16]      # GPU WordCount

config 1: WordCount through the LocalJobRunner (mapred.job.tracker=local,
CPU-only mappers), synthetic RandomTextWriter-style text.
config 2: K-Means 1M points × 128-d, k=64, one GPU map slot: the Pipes GPU
binary (native/apps/kmeans_gpu.hip, -gpubin, told its device as argv[1]) reads
its SequenceFile split itself; reduce = Pipes C++ reducer.  For comparison the
same iteration runs as the in-process split-level job (HBM-resident splits).
mrbench: MRBench (src/test/org/apache/hadoop/mapred/MRBench.java) — many
tiny jobs back to back through the JobTracker/TaskTracker; the per-job
latency is the framework's map-task invocation + scheduling overhead, the
quantity Shirahata et al. found dominant (the reference's floor is a 3 s
heartbeat, MRConstants.java:28).

Each prints one JSON line.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _text(path, mb, seed=3, files=8):
    """RandomTextWriter-style text: words from a 2,000-word vocabulary (Zipf-ish
    draw), space separated, ~10 words per line.  numpy-generated so GBs are quick."""
    import numpy as np
    rng = np.random.default_rng(seed)
    vocab = np.array([list(f"w{i:04d}".encode()) for i in range(2000)], dtype=np.uint8)
    os.makedirs(path, exist_ok=True)
    per_words = mb * (1 << 20) // 6 // files
    total = 0
    for f in range(files):
        idx = np.minimum(rng.zipf(1.3, per_words) - 1, 1999)
        rec = np.empty((per_words, 6), dtype=np.uint8)
        rec[:, :5] = vocab[idx]
        rec[:, 5] = ord(" ")
        rec[9::10, 5] = ord("\n")
        rec[-1, 5] = ord("\n")
        rec.tofile(os.path.join(path, f"part-{f:05d}"))
        total += per_words
    return total


def wordcount(a):
    from hbmr.mapred import JobClient, JobConf
    from hbmr.models import wordcount as W
    tmp = tempfile.mkdtemp(prefix="hbmr-wc-")
    try:
        inp = os.path.join(tmp, "in")
        words = _text(inp, a.mb)
        conf = JobConf()
        conf.set("mapred.job.tracker", "local")
        if a.procs > 1:
            # LocalJobRunner maps on child processes (the reference's runner is serial)
            conf.set_int("mapred.local.map.tasks.maximum", a.procs)
            conf.set("mapred.task.isolation", "process")
        elif a.threads > 1:
            # ... or on threads of this process (the native map runner releases the GIL)
            conf.set_int("mapred.local.map.tasks.maximum", a.threads)
        times = []
        for i in range(a.steps):
            job = W.make_job(inp, os.path.join(tmp, f"out{i}"), reduces=1, conf=conf)
            t = time.perf_counter()
            rj = JobClient.runJob(job, verbose=False)
            times.append(time.perf_counter() - t)
        cs = rj.getCounters()
        best = min(times)
        print(json.dumps({
            "config": "WordCount on LocalJobRunner, CPU-only mappers (BASELINE config 1)",
            "input_mb": a.mb, "words": words, "map_processes": a.procs,
            "map_threads": a.threads if a.procs <= 1 else 1,
            "job_seconds": [round(t, 3) for t in times],
            "mb_per_s": round(a.mb / best, 2), "words_per_s": round(words / best, 1),
            "map_input_records": cs.get("org.apache.hadoop.mapred.Task$Counter",
                                        "MAP_INPUT_RECORDS"),
            "combine_output_records": cs.get("org.apache.hadoop.mapred.Task$Counter",
                                             "COMBINE_OUTPUT_RECORDS")}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def wordcount_gpu(a):
    """WordCount as a split-level GPU job (text.hip): cold job (file → HBM) and
    warm jobs (splits resident in HBM), output checked against a CPU count."""
    import collections

    import torch

    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.models import wordcount as W
    tmp = tempfile.mkdtemp(prefix="hbmr-wcg-")
    try:
        inp = os.path.join(tmp, "in")
        words = _text(inp, a.mb, files=a.files)
        conf = JobConf()
        conf.set_int("hbmr.gpu.queue.depth", 16)
        with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=a.cpu_slots) as cl:
            times = []
            for i in range(a.steps + 1):
                job = W.gpu_job(inp, os.path.join(tmp, f"out{i}"), base=conf, maps=a.files)
                t = time.perf_counter()
                rj = cl.submit_job(job)
                rj.waitForCompletion()
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t)
                if not rj.isSuccessful():
                    raise RuntimeError(rj.getFailureInfo())
            cs = rj.getCounters()
        got = {}
        with open(os.path.join(tmp, f"out{a.steps}", "part-00000"), "rb") as f:
            for line in f:
                w, n = line.rstrip(b"\n").split(b"\t")
                got[w] = int(n)
        ref = collections.Counter()
        for fn in os.listdir(inp):
            with open(os.path.join(inp, fn), "rb") as f:
                ref.update(f.read().split())
        best = min(times[1:]) if len(times) > 1 else times[0]
        print(json.dumps({
            "config": "WordCount as a split-level GPU job (1 MI355X, text.hip kernels)",
            "input_mb": a.mb, "words": words, "map_tasks": a.files, "cpu_slots": a.cpu_slots,
            "cold_job_s": round(times[0], 3), "warm_job_ms": [round(1e3 * t, 2) for t in times[1:]],
            "warm_gb_per_s": round(a.mb / 1024 / best, 2), "words_per_s": round(words / best, 1),
            "gpu_maps": cs.get("org.apache.hadoop.mapred.JobInProgress$Counter", "GPU_MAP_TASKS"),
            "output_matches_cpu_count": got == dict(ref)}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def kmeans_pipes(a):
    import torch

    from hbmr.utils.sampler import dump_profiles, maybe_profile_threads
    cprof = maybe_profile_threads()   # HBMR_CPROFILE=path: cProfile of every thread
    try:
        _kmeans_pipes(a, torch)
    finally:
        if cprof:
            dump_profiles(cprof)


def _kmeans_pipes(a, torch):

    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.models import kmeans as K
    from hbmr.models import kmeans_pipes as KP
    tmp = tempfile.mkdtemp(prefix="hbmr-kmp-")
    try:
        t = time.perf_counter()
        KP.write_points(os.path.join(tmp, "pts"), a.points, a.dims, seed=5, centers=a.k,
                        files=a.files)
        t_write = time.perf_counter() - t
        init = K.initial_centroids(os.path.join(tmp, "pts"), a.k, a.dims)
        res = {"config": f"K-Means {a.points} pts x {a.dims}-d, k={a.k}, 1 GPU map slot via "
                         f"HIP Pipes (BASELINE config 2)", "points": a.points, "dims": a.dims,
               "k": a.k, "map_tasks": a.files, "write_input_s": round(t_write, 2),
               "exact": a.exact}
        gpu = torch.cuda.is_available()
        conf = JobConf()
        # every map of an iteration in flight on the GPU slot (the Pipes child
        # runs them back to back; 4 = the default left half for a second round)
        conf.set_int("hbmr.gpu.queue.depth", max(16, a.files))
        for kv in a.defines:
            kk, _, vv = kv.partition("=")
            conf.set(kk, vv)
        with LocalCluster(conf, num_trackers=1, gpus=[[0]] if gpu else None,
                          cpu_slots=0 if gpu else 2, gpu_slots_per_device=1) as cl:
            drv = KP.KMeansPipesDriver(os.path.join(tmp, "work"), os.path.join(tmp, "pts"),
                                       a.k, a.dims, init, base=conf, cluster=cl,
                                       gpubin=KP.os.path.join(KP.BIN, "kmeans_gpu") if gpu
                                       else None, maps=a.files, exact=a.exact)
            times = []
            for _ in range(a.steps):
                t = time.perf_counter()
                drv.step()
                times.append(time.perf_counter() - t)
            cs = drv.history[-1]["counters"]
            res["pipes_iteration_s"] = [round(x, 4) for x in times]
            res["pipes_gpu_maps"] = cs.get("org.apache.hadoop.mapred.JobInProgress$Counter",
                                           "GPU_MAP_TASKS")
            res["pipes_points_per_s"] = round(a.points / min(times), 1)
            pipes_cen = drv.centroids
        # the same iteration as the split-level in-process GPU job
        if gpu:
            conf = JobConf()
            conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
            with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
                d2 = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf,
                                    k=a.k, d=a.dims, inp=os.path.join(tmp, "pts"),
                                    split_points=-(-a.points // a.files))
                t = time.perf_counter()
                d2.step()   # materialise splits in HBM: native reader → pinned → H2D
                torch.cuda.synchronize()
                cold = time.perf_counter() - t
                times = []
                for _ in range(a.steps):
                    t = time.perf_counter()
                    d2.step()
                    torch.cuda.synchronize()
                    times.append(time.perf_counter() - t)
                res["splitjob_iteration_ms"] = [round(1e3 * x, 3) for x in times]
                res["splitjob_cold_first_iteration_ms"] = round(1e3 * cold, 2)
                nbytes = sum(os.path.getsize(os.path.join(tmp, "pts", f))
                             for f in os.listdir(os.path.join(tmp, "pts")))
                res["input_file_bytes"] = nbytes
                res["cold_load_gb_per_s"] = round(nbytes / max(1e-9, cold - min(times)) / 1e9,
                                                  2)
                res["splitjob_points_per_s"] = round(a.points / min(times), 1)
        res["pipes_final_centroid_norm"] = round(float(pipes_cen.norm()), 4)
        print(json.dumps(res), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def mrbench(a):
    """MRBench: small text input, 1 map + 1 reduce per job, many jobs."""
    from hbmr.mapred import JobClient, JobConf
    from hbmr.mapred.cluster import LocalCluster
    from hbmr.models import wordcount as W
    tmp = tempfile.mkdtemp(prefix="hbmr-mrb-")
    try:
        inp = os.path.join(tmp, "in")
        os.makedirs(inp)
        with open(os.path.join(inp, "f"), "w") as f:
            for i in range(a.lines):
                f.write(f"{i:08d} line of mrbench input\n")
        out = {}
        for mode in ("inproc", "child"):
            conf = JobConf()
            with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
                times = []
                for i in range(a.jobs):
                    job = W.make_job(inp, os.path.join(tmp, f"{mode}-{i}"), reduces=1)
                    job.set_num_map_tasks(a.maps)
                    if mode == "child":
                        job.set("mapred.task.isolation", "process")
                    t = time.perf_counter()
                    JobClient.runJob(job, cluster=cl, verbose=False)
                    times.append(time.perf_counter() - t)
            times.sort()
            out[mode] = {"median_job_ms": round(1e3 * times[len(times) // 2], 2),
                         "min_job_ms": round(1e3 * times[0], 2)}
        print(json.dumps({"benchmark": "MRBench (tiny jobs through JobTracker/TaskTracker)",
                          "jobs": a.jobs, "maps_per_job": a.maps, "reduces_per_job": 1,
                          "reference_floor_note": "Hadoop 1.0.3 heartbeat floor 3000 ms per "
                                                  "assignment round (MRConstants.java:28)",
                          **out}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["wordcount", "wordcount-gpu", "kmeans-pipes", "mrbench"])
    ap.add_argument("--mb", type=int, default=64)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--jobs", type=int, default=20)
    ap.add_argument("--maps", type=int, default=1)
    ap.add_argument("--lines", type=int, default=100)
    ap.add_argument("--procs", type=int, default=1, help="wordcount: parallel map processes")
    ap.add_argument("--threads", type=int, default=1, help="wordcount: parallel map threads")
    ap.add_argument("--cpu-slots", type=int, default=0)
    ap.add_argument("-D", dest="defines", action="append", default=[], metavar="KEY=VALUE",
                    help="kmeans-pipes: extra cluster/job conf")
    ap.add_argument("--exact", action=argparse.BooleanOptionalAction, default=True,
                    help="kmeans-pipes: fp64-exact labels on both binaries (hbmr.kmeans.exact)")
    a = ap.parse_args()
    {"wordcount": wordcount, "wordcount-gpu": wordcount_gpu, "kmeans-pipes": kmeans_pipes,
     "mrbench": mrbench}[a.which](a)


if __name__ == "__main__":
    main()
