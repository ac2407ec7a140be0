"""File -> HBM split loading throughput of the K-Means split job (SURVEY §2.6
NativeIO row): N points x D fp32 written as F SequenceFiles (native writer,
parallel), then one GPU tracker runs K-Means iterations over the files.  The
first iteration loads every split (native mmap decode into pinned host memory
by the loader threads, H2D on the slot streams, bf16 conversion); later ones
hit the HBM split cache.  Load throughput = input bytes / (cold - warm).

    python tools/bench_file_load.py --points 100000000 --files 32 --out profiles/file_load.json
"""
import argparse
import concurrent.futures as cf
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def write_inputs(d, n, dims, files, threads):
    from hbmr.io import nativeio
    os.makedirs(d, exist_ok=True)
    per = -(-n // files)

    def one(i):
        a = i * per
        m = min(per, n - a)
        x = np.random.default_rng(i).standard_normal((m, dims), dtype=np.float32)
        x += (np.random.default_rng(1000 + i).integers(0, 16, (m, 1)) * 8).astype(np.float32)
        nativeio.write_points(os.path.join(d, f"part-{i:05d}"), x, first_id=a)
        return m
    with cf.ThreadPoolExecutor(threads) as ex:
        return sum(ex.map(one, range(files)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--files", type=int, default=32)
    ap.add_argument("--maps", type=int, default=128)
    ap.add_argument("--write-threads", type=int, default=16)
    ap.add_argument("--load-threads", type=int, default=16)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.models import kmeans as K
    tmp = a.dir or tempfile.mkdtemp(prefix="hbmr-load-")
    inp = os.path.join(tmp, "pts")
    try:
        t = time.perf_counter()
        n = write_inputs(inp, a.points, a.dims, a.files, a.write_threads)
        t_write = time.perf_counter() - t
        nbytes = sum(os.path.getsize(os.path.join(inp, f)) for f in os.listdir(inp))
        print(json.dumps({"written_points": n, "bytes": nbytes, "write_s": round(t_write, 2)}),
              flush=True)
        conf = JobConf()
        conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
        conf.set_int("mapred.map.tasks", a.maps)
        conf.set_int("hbmr.gpu.load.threads", a.load_threads)
        with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
            drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf,
                                 k=a.k, d=a.dims, inp=inp)
            times = []
            for _ in range(3):
                t = time.perf_counter()
                r = drv.step()
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t)
                print(json.dumps({"iteration_s": round(times[-1], 4), "points": r["points"]}),
                      flush=True)
        cold, warm = times[0], min(times[1:])
        res = {"what": "K-Means split job: SequenceFile splits -> HBM (cold first iteration) "
                       "vs HBM-resident (warm)",
               "points": n, "dims": a.dims, "files": a.files, "map_tasks": a.maps,
               "input_bytes": nbytes, "load_threads": a.load_threads,
               "cold_iteration_s": round(cold, 3), "warm_iteration_s": round(warm, 4),
               "load_gb_per_s": round(nbytes / max(1e-9, cold - warm) / 1e9, 2),
               "write_gb_per_s": round(nbytes / t_write / 1e9, 2)}
        print(json.dumps(res), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
    finally:
        if a.dir is None:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
