"""Profile the control plane (JobTracker + TaskTracker + GPU runtime bookkeeping)
without a GPU: split-level SleepJobs with zero-length maps on a simulated GPU
slot, timed per job, with a wall-clock sampling profiler over all threads.

usage: python tools/profile_control_plane.py [--maps 128] [--jobs 20] [--sample]
"""
import argparse
import collections
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hbmr.examples.sleepjob import split_sleep_conf  # noqa: E402
from hbmr.mapred.cluster import LocalCluster  # noqa: E402
from hbmr.mapred.jobconf import JobConf  # noqa: E402


class Sampler(threading.Thread):
    """Samples every thread's stack each ``interval`` s; counts self and
    inclusive hits per (file:function) for threads that are not idle-waiting."""

    IDLE = {"wait", "_wait_for_tstate_lock", "get", "select", "sleep", "accept", "poll",
            "_worker", "recv_into", "readinto"}

    def __init__(self, interval=0.0005):
        super().__init__(daemon=True)
        self.interval = interval
        self.self_hits = collections.Counter()
        self.incl_hits = collections.Counter()
        self.samples = 0
        self._stop = threading.Event()

    def run(self):
        me = threading.get_ident()
        while not self._stop.is_set():
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                top = fr.f_code.co_name
                if top in self.IDLE:
                    continue
                self.samples += 1
                seen = set()
                f = fr
                first = True
                while f is not None:
                    key = f"{os.path.basename(f.f_code.co_filename)}:{f.f_code.co_name}"
                    if first:
                        self.self_hits[key] += 1
                        first = False
                    if key not in seen:
                        self.incl_hits[key] += 1
                        seen.add(key)
                    f = f.f_back
            time.sleep(self.interval)

    def stop(self):
        self._stop.set()

    def report(self, top=30):
        print(f"samples (busy threads): {self.samples}")
        print("-- self --")
        for k, v in self.self_hits.most_common(top):
            print(f"{v:7d} {100.0 * v / max(1, self.samples):5.1f}%  {k}")
        print("-- inclusive --")
        for k, v in self.incl_hits.most_common(top):
            print(f"{v:7d} {100.0 * v / max(1, self.samples):5.1f}%  {k}")


_PROFILES = []


def _install_thread_profiler():
    """Run every thread started from now on under its own cProfile.Profile."""
    import cProfile
    orig = threading.Thread.run

    def run(self):
        pr = cProfile.Profile()
        _PROFILES.append(pr)
        pr.enable()
        try:
            orig(self)
        finally:
            pr.disable()
    threading.Thread.run = run
    main_pr = cProfile.Profile()
    _PROFILES.append(main_pr)
    return main_pr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--maps", type=int, default=128)
    ap.add_argument("--jobs", type=int, default=20)
    ap.add_argument("--slots", type=int, default=1)
    ap.add_argument("--queue-depth", type=int, default=128)
    ap.add_argument("--sample", action="store_true")
    ap.add_argument("--cpu-slots", type=int, default=0)
    ap.add_argument("--cprofile", action="store_true", help="cProfile all threads")
    ap.add_argument("--trace", action="store_true", help="print the event timeline of the last job")
    a = ap.parse_args()
    main_pr = _install_thread_profiler() if a.cprofile else None
    conf = JobConf()
    conf.set_boolean("hbmr.gpu.simulate", True)
    conf.set("hbmr.scheduler.policy", "hybrid")
    conf.set_int("hbmr.gpu.queue.depth", a.queue_depth)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", a.slots)
    conf.set_int("mapred.task.timeout", 0)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=a.cpu_slots) as cl:
        for _ in range(3):
            cl.submit_job(split_sleep_conf(a.maps, base=conf)).waitForCompletion()
        sampler = Sampler() if a.sample else None
        if sampler:
            sampler.start()
        if main_pr:
            for pr in _PROFILES:
                pr.disable() if pr is not main_pr else None
            import cProfile  # noqa: F401
            for pr in _PROFILES:
                pr.enable() if pr is not main_pr else None
            main_pr.enable()
        lat = []
        phases = collections.defaultdict(list)
        for _ in range(a.jobs):
            t0 = time.perf_counter()
            rj = cl.submit_job(split_sleep_conf(a.maps, base=conf))
            rj.waitForCompletion()
            lat.append(time.perf_counter() - t0)
            assert rj.isSuccessful(), rj.getFailureInfo()
            tl = rj._impl.jip.timeline()
            for k, v in tl.items():
                if isinstance(v, (int, float)) and v is not None:
                    phases[k].append(v)
        if sampler:
            sampler.stop()
        if main_pr:
            import pstats
            main_pr.disable()
            for pr in _PROFILES:
                pr.disable()
            st = pstats.Stats(_PROFILES[0])
            for pr in _PROFILES[1:]:
                try:
                    st.add(pr)
                except TypeError:
                    pass
            st.sort_stats("tottime").print_stats(35)
        lat.sort()
        print(f"maps/job={a.maps} jobs={a.jobs}: median {1e3 * lat[len(lat) // 2]:.2f} ms, "
              f"min {1e3 * lat[0]:.2f} ms, per-map {1e6 * lat[len(lat) // 2] / a.maps:.1f} us")
        for k, v in phases.items():
            v.sort()
            print(f"  {k:>16}: median {1e3 * v[len(v) // 2]:.2f} ms")
        if sampler:
            sampler.report()
        if a.trace:
            from hbmr.utils.trace import TRACE
            TRACE.enable()
            TRACE.clear()
            cl.submit_job(split_sleep_conf(a.maps, base=conf)).waitForCompletion()
            TRACE.disable()
            t0 = TRACE.events[0][0]
            last = None
            for ts, th, ph, name, dur, args in TRACE.events:
                if name == "tt.finish" and last == "tt.finish":
                    continue
                last = name
                print(f"{(ts - t0) / 1e6:9.3f} ms {dur / 1e6:7.3f} {th[:22]:>22} {name:<20} "
                      f"{ {k: v for k, v in args.items() if k != 'attempt'} }")


if __name__ == "__main__":
    main()
