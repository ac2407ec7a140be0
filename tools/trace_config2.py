"""Event timeline of one Pipes K-Means iteration (BASELINE config 2) after
warm-up: where the per-iteration time goes (task launch, Pipes child, reduce).

usage: python tools/trace_config2.py [--points 1000000] [--files 8] [--gpu]
"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("-D", dest="defines", action="append", default=[], metavar="KEY=VALUE")
    a = ap.parse_args()
    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.models import kmeans as K
    from hbmr.models import kmeans_pipes as KP
    from hbmr.utils.trace import TRACE
    tmp = tempfile.mkdtemp(prefix="hbmr-trace2-")
    child_trace = os.path.join(tmp, "child.trace")
    os.environ["HBMR_PIPES_TRACE"] = child_trace      # the GPU child's phase marks
    KP.write_points(os.path.join(tmp, "pts"), a.points, 128, seed=5, centers=a.k, files=a.files)
    init = K.initial_centroids(os.path.join(tmp, "pts"), a.k, 128)
    conf = JobConf()
    conf.set_int("hbmr.gpu.queue.depth", max(16, a.files))
    for kv in a.defines:
        k, _, v = kv.partition("=")
        conf.set(k, v)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]] if a.gpu else None,
                      cpu_slots=0 if a.gpu else 2, gpu_slots_per_device=1) as cl:
        drv = KP.KMeansPipesDriver(os.path.join(tmp, "work"), os.path.join(tmp, "pts"), a.k, 128,
                                   init, cluster=cl, gpubin=os.path.join(KP.BIN, "kmeans_gpu")
                                   if a.gpu else None, maps=a.files)
        for _ in range(3):
            t = time.perf_counter()
            drv.step()
            print("warm-up iteration", round(time.perf_counter() - t, 4), flush=True)
        TRACE.enable()
        TRACE.clear()
        skip = os.path.getsize(child_trace) if os.path.exists(child_trace) else 0
        t = time.perf_counter()
        drv.step()
        print("traced iteration", round(time.perf_counter() - t, 4), flush=True)
        TRACE.disable()
    from hbmr.utils.trace import wall_ns
    events = list(TRACE.events)
    if os.path.exists(child_trace):
        off = wall_ns(0)                  # child wall clock -> this process's perf clock
        with open(child_trace) as f:
            f.seek(skip)
            for line in f:
                w, _, name = line.strip().partition(" ")
                events.append((int(float(w) * 1e9) - off, "pipes-child", "i", name, 0, {}))
    events.sort(key=lambda e: e[0])
    t0 = TRACE.events[0][0]
    for ts, th, ph, name, dur, args in events:
        if name in ("jt.heartbeat",):
            continue
        print(f"{(ts - t0) / 1e6:9.3f} ms {dur / 1e6:7.3f} {th[:24]:>24} {name:<22} "
              f"{ {k: v for k, v in args.items() if k not in ('attempt',)} }")


if __name__ == "__main__":
    main()
