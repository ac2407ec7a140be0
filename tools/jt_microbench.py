"""JobTracker control-plane cost per job, in one process and without threads.

Drives a real :class:`hbmr.mapred.jobtracker.JobTracker` through the headline
job's steady state — a chain of staged K-Means iteration jobs (128 splits of
the 100M x 128 input, k = 1024) on N simulated one-GPU trackers — with the
calls a tracker makes (initial heartbeat, ``report(assign=True)`` carrying its
batched map completions and its collective reduce's completion) and measures
the JobTracker's CPU per job as N grows: the thread CPU time spent inside the
JobTracker's entry points plus the msgpack decode of each request and encode of
each reply (what its RPC server does per call).  No sockets, no tracker
threads, no GPU: the number isolates the JobTracker's own work, the quantity
that bounds multi-rank scaling (VERDICT r4 Next #1).

    python tools/jt_microbench.py --trackers 1 2 4 8 --jobs 60
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import msgpack  # noqa: E402

from hbmr.mapred import protocol as P  # noqa: E402
from hbmr.mapred.jobconf import JobConf  # noqa: E402
from hbmr.mapred.jobtracker import DEPENDS_KEY, JobTracker  # noqa: E402
from hbmr.models import kmeans as K  # noqa: E402

COUNTERS = {"hbmr.GpuCounters": {"GPU_KERNEL_US": 3300, "GPU_MAP_BATCHES": 1},
            "org.apache.hadoop.mapred.Task$Counter": {"MAP_INPUT_RECORDS": 12_500_000}}


def _status(name, rank, world, reports=(), bulk=(), cached=()):
    return P.TaskTrackerStatus(
        tracker_name=name, host="node0", max_cpu_map_slots=0, max_reduce_slots=1,
        gpus=[{"device": rank, "max_slots": 2, "running": 0, "queued": 0,
               "hbm_total": 288 << 30, "hbm_free": 200 << 30, "name": "sim"}],
        task_reports=list(reports), bulk_reports=list(bulk),
        cached_splits_added=list(cached), rank=rank, world_size=world).to_dict()


class Harness:
    def __init__(self, n, points=100_000_000, split_points=781_250, k=1024, d=128, ahead=3,
                 conf_overrides=None):
        conf = JobConf()
        conf.set("hbmr.scheduler.policy", "hybrid")
        conf.set_int("mapred.task.timeout", 0)
        conf.set_int("hbmr.locality.wait.ms", 5000)
        conf.set_int("hbmr.job.prestage.depth", ahead)
        conf.set_int("hbmr.gpu.queue.depth", 64)           # bench.py's defaults
        conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", 2)
        for kk, v in (conf_overrides or {}).items():
            conf.set(kk, v)
        self.base = conf
        self.jt = JobTracker(conf)
        self.n = n
        self.k, self.d, self.split_points = k, d, split_points
        self.inp = f"synthetic:{points}:7"
        self.ahead = ahead
        self.names = [f"tracker_sim_r{r}" for r in range(n)]
        self.pend = {nm: {} for nm in self.names}    # tracker -> job -> launched work
        self.cached = {nm: [] for nm in self.names}
        self.cpu = 0.0
        self.calls = 0
        self.park = False
        self.parked_steps = 0
        self.rng = None                 # random.Random: trackers step at self.speed[r]
        self.speed = [1.0] * n
        self.submitted: list[str] = []
        self.finished = 0
        for r, nm in enumerate(self.names):
            self._call(self.jt.heartbeat, _status(nm, r, n), initial=True)

    # every JobTracker entry point is timed with the msgpack decode of its
    # request and the encode of its reply
    def _call(self, fn, payload, *a, **kw):
        t0 = time.thread_time()
        req = msgpack.unpackb(msgpack.packb(payload), raw=False, strict_map_key=False) \
            if isinstance(payload, dict) else payload
        res = fn(req, *a, **kw)
        out = msgpack.unpackb(msgpack.packb(res), raw=False, strict_map_key=False) \
            if isinstance(res, dict) else res
        self.cpu += time.thread_time() - t0
        self.calls += 1
        return out

    def submit(self):
        i = len(self.submitted)
        job = K.make_iteration_conf(self.base, self.k, self.d, self.inp, self.split_points,
                                    f"mb:{i}", f"mb:{i + 1}")
        if self.submitted:
            job.set(DEPENDS_KEY, self.submitted[-1])
        wire = msgpack.packb(job.to_dict())        # the driver's side
        t0 = time.thread_time()
        d = msgpack.unpackb(wire, raw=False)
        jid = self.jt.rpc_submit_job(d)
        self.cpu += time.thread_time() - t0
        self.calls += 1
        self.submitted.append(jid)

    def _apply(self, nm, resp):
        for a in resp.get("actions") or ():
            t = a["type"]
            if t == "launch_batch":
                w = self.pend[nm].setdefault(a["job_id"], {"maps": [], "reduce": None})
                w["maps"] += [x[0] for x in a["tasks"]]
                self.cached[nm] += [[x[2].get("key"), a["device"]] for x in a["tasks"]
                                    if isinstance(x[2], dict) and x[2].get("key")]
            elif t == "launch":
                spec = a["task"]
                w = self.pend[nm].setdefault(spec["job_id"], {"maps": [], "reduce": None})
                if spec["is_map"]:
                    w["maps"].append(spec["attempt_id"])
                else:
                    w["reduce"] = spec["attempt_id"]
            elif t == "commit":
                pass

    def _oldest(self, nm):
        for jid in self.submitted:
            if jid in self.pend[nm]:
                return jid, self.pend[nm][jid]
        return None, None

    def step(self, r):
        """Tracker ``r`` finishes the oldest job it holds work of (its maps'
        batch and its reduce) and reports it; with nothing held it polls —
        or, with ``park`` (a long-poll modelled), it waits for its bell and
        only then heartbeats: work left in a parked tracker's queues with its
        bell unrung is a lost wake-up (the real long-poll would sit it out)."""
        nm = self.names[r]
        jid, w = self._oldest(nm)
        now = time.time()
        if w is None or (not w["maps"] and w["reduce"] is None):
            tr = self.jt.trackers[nm]
            if self.park:
                if not tr.bell.is_set():
                    self.parked_steps += 1
                    return
                tr.bell.clear()
            resp = self._call(self.jt.heartbeat, _status(nm, r, self.n), block=0.0)
            self._apply(nm, resp)
            return
        bulk = []
        if w["maps"]:
            bulk = [{"attempts": w["maps"], "device_time": 0.00026 * len(w["maps"]),
                     "finish_time": now, "counters": COUNTERS, "output": {"where": "gpu"}}]
            w["maps"] = []
        reps = []
        if w["reduce"] is not None:
            reps = [P.TaskStatus(attempt_id=w["reduce"], is_map=False, state=P.SUCCEEDED,
                                 progress=1.0, run_on_gpu=True, gpu_device_id=r,
                                 finish_time=now, counters=COUNTERS,
                                 output={"result": {"shift": 0.0}}).to_dict()]
            del self.pend[nm][jid]
        cached, self.cached[nm] = self.cached[nm], []
        resp = self._call(self.jt.report, _status(nm, r, self.n, reps, bulk, cached), True)
        self._apply(nm, resp)

    def run(self, jobs, warmup=8):
        for _ in range(self.ahead + 1):
            self.submit()
        for r in range(self.n):
            self._apply(self.names[r], self._call(self.jt.heartbeat,
                                                  _status(self.names[r], r, self.n)))
        done = 0
        cpu0 = calls0 = None
        guard = 0
        while done < jobs + warmup:
            guard += 1
            if guard > 200 * (jobs + warmup) * self.n:
                raise RuntimeError("no progress")
            for r in range(self.n):
                if self.rng is None or self.rng.random() < self.speed[r]:
                    self.step(r)
            while done < len(self.submitted) and self.jt.jobs[self.submitted[done]].done.is_set():
                st = self.jt.jobs[self.submitted[done]].status.state
                if st != "SUCCEEDED":
                    raise RuntimeError(f"job {self.submitted[done]} {st}")
                done += 1
                if done == warmup:
                    cpu0, calls0 = self.cpu, self.calls
                if len(self.submitted) < jobs + warmup:
                    self.submit()
        return {"trackers": self.n, "jobs": jobs,
                "jt_cpu_ms_per_job": round((self.cpu - cpu0) / jobs * 1e3, 3),
                "calls_per_job": round((self.calls - calls0) / jobs, 2)}


def measure(n, jobs=40, **kw):
    h = Harness(n, **kw)
    try:
        return h.run(jobs)
    finally:
        h.jt.shutdown() if hasattr(h.jt, "shutdown") else None


def main():
    from hbmr.utils.gctune import tune
    tune()                  # the JobTracker process's collector settings
    ap = argparse.ArgumentParser()
    ap.add_argument("--trackers", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--jobs", type=int, default=40)
    ap.add_argument("--splits", type=int, default=128)
    ap.add_argument("--ahead", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3, help="best of this many runs per N")
    ap.add_argument("--one", action="store_true", help="one run in this process")
    ap.add_argument("--profile", default=None, help="cProfile one run into this file")
    a = ap.parse_args()
    kw = dict(ahead=a.ahead, split_points=-(-100_000_000 // a.splits))
    if a.one or a.profile:
        pr = None
        if a.profile:
            import cProfile
            pr = cProfile.Profile(time.thread_time)
            pr.enable()
        r = measure(a.trackers[0], a.jobs, **kw)
        if pr is not None:
            pr.disable()
            pr.dump_stats(a.profile)
        print(json.dumps(r), flush=True)
        return
    import subprocess
    for n in a.trackers:
        # every run in a fresh interpreter: a JobTracker's state (and what the
        # collector has to walk) must not carry over into the next measurement
        runs = []
        for _ in range(a.reps):
            out = subprocess.run([sys.executable, __file__, "--one", "--trackers", str(n),
                                  "--jobs", str(a.jobs), "--splits", str(a.splits),
                                  "--ahead", str(a.ahead)], check=True, capture_output=True,
                                 text=True).stdout
            runs.append(json.loads(out.strip().splitlines()[-1]))
        r = min(runs, key=lambda x: x["jt_cpu_ms_per_job"])
        r["runs_ms"] = [x["jt_cpu_ms_per_job"] for x in runs]
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
