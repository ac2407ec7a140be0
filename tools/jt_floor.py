"""Control-plane floor of the headline K-Means chain, all in one process:
a LocalCluster of N trackers with simulated GPU slots (no data, T ms of device
time per split), the same pre-staged K-Means driver as bench.py.  Reports
ms/job and, with --cprofile, the CPU per job by component (JobTracker +
scheduler, TaskTracker, GPU runtime/split executor, model, RPC/other), which is
what a JobTracker process of its own would have to sustain per job.
The profiles measure per-thread CPU time (time.thread_time), so threads
waiting for the interpreter lock or a Python lock are not charged.

usage: python tools/jt_floor.py [--trackers 8] [--jobs 40] [--ms 0.01] [--cprofile]
"""
import argparse
import collections
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hbmr.mapred.cluster import LocalCluster  # noqa: E402
from hbmr.mapred.jobconf import JobConf  # noqa: E402
from hbmr.models import kmeans as K  # noqa: E402

_PROFILES = []


def _install_thread_profiler():
    import cProfile
    orig = threading.Thread.run

    def run(self):
        pr = cProfile.Profile(time.thread_time)
        _PROFILES.append(pr)
        pr.enable()
        try:
            orig(self)
        finally:
            pr.disable()
    threading.Thread.run = run
    main_pr = cProfile.Profile(time.thread_time)
    _PROFILES.append(main_pr)
    return main_pr


def component(fn):
    if "mapred/jobtracker" in fn or "mapred/scheduler" in fn or "mapred/ids" in fn:
        return "jobtracker"
    if "mapred/tasktracker" in fn or "mapred/protocol" in fn:
        return "tasktracker"
    if "/gpu/" in fn:
        return "gpu runtime"
    if "/models/" in fn:
        return "model"
    if "hbmr/" in fn:
        return "hbmr other"
    return "python/libs"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trackers", type=int, default=8)
    ap.add_argument("--jobs", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ms", type=float, default=0.01)
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--split-points", type=int, default=781_250)
    ap.add_argument("--cprofile", action="store_true")
    ap.add_argument("--filter", default="", help="regex: print only matching functions")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--sort", default="tottime")
    a = ap.parse_args()
    main_pr = _install_thread_profiler() if a.cprofile else None
    conf = JobConf()
    conf.set("hbmr.scheduler.policy", "hybrid")
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
    conf.set_int("hbmr.gpu.queue.depth", 64)          # bench.py's defaults
    conf.set_int("hbmr.job.prestage.depth", 2)
    conf.set_int("hbmr.heartbeat.interval.ms", 200)
    conf.set_int("mapred.task.timeout", 0)
    conf.set_int("hbmr.locality.wait.ms", 5000)
    conf.set_boolean("hbmr.job.prestage", True)
    conf.set("hbmr.gpu.simulate", "true")
    conf.set("hbmr.gpu.simulate.nodata", "true")
    conf.set("hbmr.gpu.simulate.task.ms", str(a.ms))
    conf.set_boolean("hbmr.gpu.worker.process", False)
    with LocalCluster(conf, num_trackers=a.trackers, gpus=[[0]] * a.trackers,
                      cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result, conf=conf,
                             k=1024, d=128, inp=f"synthetic:{a.points}:7",
                             split_points=a.split_points)
        for w in range(a.warmup):
            drv.step(prefetch=min(2, a.warmup - 1 - w))
        if main_pr:
            for pr in _PROFILES:
                pr.clear() if hasattr(pr, "clear") else None
            main_pr.enable()
        cpu0 = time.process_time()
        t0 = time.perf_counter()
        for s in range(a.jobs):
            drv.step(prefetch=min(2, a.jobs - 1 - s))
        dt = time.perf_counter() - t0
        cpu = time.process_time() - cpu0
    print(f"trackers={a.trackers} jobs={a.jobs} ms/job={1e3 * dt / a.jobs:.2f} "
          f"process cpu ms/job={1e3 * cpu / a.jobs:.2f}")
    if main_pr:
        import pstats
        for pr in _PROFILES:
            pr.disable()
        st = None
        for pr in _PROFILES:
            try:
                st = pstats.Stats(pr) if st is None else (st.add(pr) or st)
            except TypeError:
                pass
        by = collections.Counter()
        for (fn, _line, _name), (_cc, _nc, tt, _ct, _callers) in st.stats.items():
            by[component(fn)] += tt
        idle = sum(tt for (fn, _l, name), (_c, _n, tt, _ct, _cl) in st.stats.items()
                   if name in ("<method 'acquire' of '_thread.lock' objects>",
                               "<method 'wait' of '_thread.lock' objects>",
                               "<built-in method time.sleep>"))
        print(f"cProfile self time per job by component (ms; lock waits/sleeps "
              f"{1e3 * idle / a.jobs:.2f} ms/job are in python/libs):")
        for k, v in by.most_common():
            print(f"  {k:14s} {1e3 * v / a.jobs:8.2f}")
        st.sort_stats(a.sort).print_stats(*([a.filter] if a.filter else []), a.top)


if __name__ == "__main__":
    main()
