"""cProfile of every thread of a Pipes K-Means cluster (BASELINE config 2)
over N warm iterations: where the parent-side Python time of an iteration
goes (the GPU child's time is outside Python).  Each thread started after this
module patches threading.Thread.run gets its own profiler; the stats are
merged at exit.

usage: python tools/profile_config2.py [--gpu] [--iters 20] [--points 1000000]
"""
import argparse
import cProfile
import os
import pstats
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PROFS = []
_run = threading.Thread.run


def _profiled(run):
    def wrapped(self):
        pr = cProfile.Profile()
        # registered up front: pool workers outlive the cluster (their stats are
        # read while they idle)
        PROFS.append(pr)
        pr.enable()
        try:
            run(self)
        finally:
            pr.disable()
    return wrapped


_profiled_run = _profiled(_run)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.models import kmeans as K
    from hbmr.models import kmeans_pipes as KP
    tmp = tempfile.mkdtemp(prefix="hbmr-prof2-")
    KP.write_points(os.path.join(tmp, "pts"), a.points, 128, seed=5, centers=64, files=a.files)
    init = K.initial_centroids(os.path.join(tmp, "pts"), 64, 128)
    conf = JobConf()
    conf.set_int("hbmr.gpu.queue.depth", max(16, a.files))
    threading.Thread.run = _profiled_run
    from hbmr.pipes.protocol import UplinkReader
    UplinkReader.run = _profiled(UplinkReader.run)     # overrides Thread.run
    main_pr = cProfile.Profile()
    with LocalCluster(conf, num_trackers=1, gpus=[[0]] if a.gpu else None,
                      cpu_slots=0 if a.gpu else 2, gpu_slots_per_device=1) as cl:
        drv = KP.KMeansPipesDriver(os.path.join(tmp, "work"), os.path.join(tmp, "pts"), 64, 128,
                                   init, cluster=cl, gpubin=os.path.join(KP.BIN, "kmeans_gpu")
                                   if a.gpu else None, maps=a.files)
        for _ in range(3):
            drv.step()
        # only the measured iterations: every thread's profile restarts here
        main_pr.enable()
        t = time.perf_counter()
        for _ in range(a.iters):
            drv.step()
        dt = (time.perf_counter() - t) / a.iters
        main_pr.disable()
    time.sleep(0.3)
    print(f"ms/iteration {dt * 1e3:.2f} over {a.iters} (profiled: slower than unprofiled)")
    st = pstats.Stats(main_pr)
    for p in PROFS:
        st.add(p)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumtime").print_stats("hbmr", a.top)


if __name__ == "__main__":
    main()
