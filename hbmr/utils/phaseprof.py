"""Per-method thread-CPU accounting for a live process: ``HBMR_PHASE_PROF=
/path/prefix`` wraps a fixed list of control-plane methods (JobTracker entry
points, scheduling and bookkeeping phases) with ``time.thread_time`` deltas
and writes calls / CPU per method to ``<prefix>_<pid>.txt`` at exit.  Unlike
cProfile it costs two clock reads per wrapped call, so the numbers stay close
to an unprofiled run's (nested phases are included in their callers)."""
from __future__ import annotations

import atexit
import collections
import os
import time

_TARGETS = (
    ("hbmr.mapred.jobtracker", "JobTracker", ("rpc_submit_job", "_heartbeat", "heartbeat",
                                              "report", "_maybe_stage", "_bulk_succeeded",
                                              "_update_task_status", "launch_gpu_batch",
                                              "launch", "reduce_inputs", "_finish_job",
                                              "rpc_wait_job_info", "wakeup")),
    ("hbmr.mapred.jobtracker", "JobInProgress", ("__init__", "init_tasks", "obtain_maps")),
    ("hbmr.mapred.scheduler.hybrid", "HybridTaskScheduler", ("assign_tasks", "plan_staged",
                                                             "_assign_reduces")),
    ("hbmr.mapred.protocol", "TaskTrackerStatus", ("from_dict",)),
)


def maybe_install():
    prefix = os.environ.get("HBMR_PHASE_PROF")
    if not prefix:
        return None
    import importlib
    acc = collections.defaultdict(lambda: [0, 0.0, []])

    def wrap(owner, name, label):
        f = owner.__dict__.get(name)
        if f is None:
            return
        static = isinstance(f, (staticmethod, classmethod))
        fn = f.__func__ if static else f

        def g(*a, **k):
            t0 = time.thread_time()
            try:
                return fn(*a, **k)
            finally:
                st = acc[label]
                st[0] += 1
                dt = time.thread_time() - t0
                st[1] += dt
                if len(st[2]) < 100000:
                    st[2].append(dt)
        g.__name__ = getattr(fn, "__name__", name)
        setattr(owner, name, type(f)(g) if static else g)

    # who rings the trackers' long-polls (JobTracker._kick, by calling line)
    try:
        import sys
        from ..mapred import jobtracker as _jt
        kick = _jt.JobTracker._kick

        def counted_kick(self):
            f = sys._getframe(1)
            st = acc[f"kick<-{f.f_code.co_name}:{f.f_lineno}"]
            st[0] += 1
            return kick(self)
        _jt.JobTracker._kick = counted_kick
    except ImportError:
        pass
    for mod, cls, names in _TARGETS:
        try:
            owner = getattr(importlib.import_module(mod), cls)
        except (ImportError, AttributeError):
            continue
        for n in names:
            wrap(owner, n, f"{cls}.{n}")

    def dump():
        with open(f"{prefix}_{os.getpid()}.txt", "w") as f:
            f.write("method calls cpu_s us_per_call median_us\n")
            for k, (n, t, ds) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
                med = sorted(ds)[len(ds) // 2] if ds else 0.0
                f.write(f"{k} {n} {t:.4f} {t / max(1, n) * 1e6:.1f} {med * 1e6:.1f}\n")
    atexit.register(dump)
    return acc
