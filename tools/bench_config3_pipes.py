"""BASELINE config 3 (K-Means 100M x 128, k = 1024, exact fp32) through the
Pipes bridge — the reference's own shape of the GPU map (PipesGPUMapRunner ->
Application -> the GPU binary) — against the in-framework split job on the
same SequenceFile input.

Input: 100M points of the bench distribution (hbmr.models.kmeans.synthetic_points,
seed 7, 1024 centres), generated on the GPU and written by the native writer as
``--files`` SequenceFiles.  Both jobs run exact mode from the same initial
centroids (the first k points), so their centroids must match bit for bit.

    python tools/bench_config3_pipes.py --points 100000000 --files 128 --iters 4
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


def write_inputs(d, n, dims, k, files, threads, seed=7):
    import torch

    from hbmr.io import nativeio
    from hbmr.models import kmeans as K
    os.makedirs(d, exist_ok=True)
    per = -(-n // files)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        futs = []
        for i in range(files):
            a = i * per
            m = min(per, n - a)
            if m <= 0:
                break
            x = K.synthetic_points(seed, a, m, dims, k, dev).cpu().numpy()
            futs.append(ex.submit(nativeio.write_points, os.path.join(d, f"part-{i:05d}"), x, a))
            if i % 16 == 15:
                print(json.dumps({"written_files": i + 1, "s": round(time.perf_counter() - t0, 1)}),
                      flush=True)
            while len([f for f in futs if not f.done()]) > threads:
                time.sleep(0.01)
        for f in futs:
            f.result()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--files", type=int, default=128)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--write-threads", type=int, default=8)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--skip-split-job", action="store_true")
    ap.add_argument("--trace", default=None, help="event timeline of the last Pipes iteration")
    ap.add_argument("-D", dest="defines", action="append", default=[], metavar="KEY=VALUE",
                    help="extra conf for the Pipes job's cluster")
    a = ap.parse_args()
    import torch

    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.models import kmeans as K
    from hbmr.models import kmeans_pipes as KP
    from hbmr.pipes import mux
    tmp = a.dir or tempfile.mkdtemp(prefix="hbmr-c3-")
    inp = os.path.join(tmp, "pts")
    res = {"config": f"K-Means {a.points} x {a.dims}, k={a.k}, exact, 1 GPU: Pipes GPU binary "
                     f"vs split job (BASELINE config 3)", "points": a.points, "files": a.files}
    try:
        t = time.perf_counter()
        write_inputs(inp, a.points, a.dims, a.k, a.files, a.write_threads)
        res["write_s"] = round(time.perf_counter() - t, 1)
        res["input_bytes"] = sum(os.path.getsize(os.path.join(inp, f)) for f in os.listdir(inp))
        print(json.dumps({"write_s": res["write_s"], "bytes": res["input_bytes"]}), flush=True)
        init = K.initial_centroids(inp, a.k, a.dims, exact=True)
        if not a.skip_split_job:
            conf = JobConf()
            conf.set_boolean(K.EXACT_KEY, True)
            conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
            conf.set_int("mapred.map.tasks", a.files)
            with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
                drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf,
                                     k=a.k, d=a.dims, inp=inp)
                times = []
                for _ in range(a.iters):
                    t = time.perf_counter()
                    drv.step()
                    torch.cuda.synchronize()
                    times.append(time.perf_counter() - t)
                    print(json.dumps({"split_job_iteration_s": round(times[-1], 4)}), flush=True)
                res["split_job_iteration_ms"] = [round(1e3 * x, 2) for x in times]
                split_cen = drv.centroids().clone()
            torch.cuda.empty_cache()
        conf = JobConf()
        conf.set_int("hbmr.gpu.queue.depth", max(16, a.files))
        for kv in a.defines:
            kk, _, vv = kv.partition("=")
            conf.set(kk, vv)
        # one map per file, as the split job's 128 splits (FileInputFormat
        # would cut each 420 MB file into 64 MB blocks: 7x the map tasks)
        conf.set_long("mapred.min.split.size", 1 << 40)
        # every split resident in the GPU child's HBM cache (exact mode holds
        # the fp32 rows, their fp16 copy and per-point norms: ~78 GB here)
        os.environ["HBMR_PIPES_SPLIT_CACHE_MB"] = "200000"
        with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0,
                          gpu_slots_per_device=1) as cl:
            drv = KP.KMeansPipesDriver(os.path.join(tmp, "work"), inp, a.k, a.dims, init,
                                       base=conf, cluster=cl,
                                       gpubin=os.path.join(KP.BIN, "kmeans_gpu"),
                                       maps=a.files, exact=True)
            times = []
            from hbmr.utils.trace import TRACE
            for it in range(a.iters):
                if a.trace and it == a.iters - 1:
                    TRACE.enable()
                    TRACE.clear()
                t = time.perf_counter()
                drv.step()
                times.append(time.perf_counter() - t)
                print(json.dumps({"pipes_iteration_s": round(times[-1], 4)}), flush=True)
            if a.trace:
                TRACE.disable()
                ev = [e for e in TRACE.events if e[3] not in ("jt.heartbeat",)]
                t0 = ev[0][0]
                with open(a.trace, "w") as f:
                    for ts, th, _ph, name, _dur, args in ev:
                        f.write(f"{(ts - t0) / 1e6:9.3f} ms {th[:24]:>24} {name:<24} "
                                f"{ {k: v for k, v in args.items() if k != 'attempt'} }\n")
            res["pipes_iteration_ms"] = [round(1e3 * x, 2) for x in times]
            cs = drv.history[-1]["counters"]
            res["pipes_gpu_maps"] = cs.get("KMEANS", "GPU_MAPS")
            res["pipes_split_cache_hits"] = cs.get("KMEANS", "GPU_SPLIT_CACHE_HITS")
            pipes_cen = drv.centroids.clone()
        mux.REGISTRY.close_all()
        if not a.skip_split_job:
            # both started from the first k fp32 points and run the exact
            # assignment with fixed-point sums: the same centroids, bit for bit
            res["centroids_equal"] = bool(torch.equal(split_cen, pipes_cen))
            warm_s = min(res["split_job_iteration_ms"][1:])
            warm_p = min(res["pipes_iteration_ms"][1:])
            res["pipes_over_split_job"] = round(warm_p / warm_s, 2)
        print(json.dumps(res), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
    finally:
        if a.dir is None:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
