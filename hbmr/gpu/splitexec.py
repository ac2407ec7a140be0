"""Execution of split-level tasks that do not go through a GPU slot's stream:
CPU-slot maps (and sampled CPU profiling probes) and the collective reduce.

Shared by the TaskTracker (device work in-process) and the per-GPU worker
process (:mod:`hbmr.gpu.worker`, device work isolated from the tracker), so
both run exactly the same task code.  ``host`` is the tracker, or the worker's
tracker facade: it provides ``split_cache``, ``comm``, ``cpu_threads``,
``_finish`` and ``_maybe_inject_fault``.

Reference: MapTask.run / ReduceTask.run (hadoop-1.0.3/src/mapred/org/apache/
hadoop/mapred/MapTask.java:340, ReduceTask.java:348) — here a split is handed
to the job's map function whole and the reduce is a collective over the
trackers' combined map outputs.
"""
from __future__ import annotations

import time
import traceback

from ..mapred import counters as C
from ..mapred import protocol as P
from ..mapred.task import TaskReporter
from ..utils.trace import TRACE
from .splitjob import SplitSpec


class SplitTaskShim:
    """What a running split task exposes to its tracker (reporter + kill flag)."""

    def __init__(self, reporter, kill_event=None):
        self.reporter = reporter
        self.kill_event = kill_event


def run_split_cpu_map(host, run):
    """A split job's map on a CPU slot (``profile_fraction`` > 0: a sampled
    profiling probe whose output is dropped).  Finishes ``run`` on ``host``."""
    from ..mapred.tasktracker import TaskContext
    spec, js = run.spec, run.job
    run.status.start_time = time.time()
    try:
        if run.kill.is_set():
            host._finish(run, P.KILLED, "killed before start")
            return
        host._maybe_inject_fault(run)
        rep = TaskReporter()
        run.task = SplitTaskShim(rep, run.kill)
        ctx = TaskContext(host, js, spec, rep, device="cpu")
        ctx.kill_event = run.kill          # cooperative kill (preemption, speculation)
        sspec = SplitSpec.from_dict(spec.split)
        if spec.profile_fraction:
            # sampled profiling probe: time the CPU map on a slice; the output is
            # dropped (the GPUs run the real task)
            sample = js.split_job.load_split_sample(sspec, "cpu", spec.profile_fraction)
            run.status.start_time = time.time()
            t0 = time.perf_counter()
            js.split_job.map_cpu(ctx, sample)
            compute = time.perf_counter() - t0
            rep.counters = C.Counters()
            # the probe's own compute time rides in device_time: the JobTracker
            # scales it by 1/fraction, and launch/report latency must not be
            host._finish(run, P.SUCCEEDED, output={"tracker": host.name, "where": "cpu",
                                                   "profile": True}, device_time=compute)
            return
        data, _hit = host.split_cache.get_or_load(
            sspec.key, "cpu", lambda: js.split_job.load_split(sspec, "cpu"),
            js.split_job.split_nbytes)
        out = js.split_job.map_cpu(ctx, data)
        with js.lock:
            js.map_outputs[spec.attempt_id] = out
        rep.incrCounter(C.JOB_GROUP, C.CPU_MAP_TASKS, 0)
        host._finish(run, P.SUCCEEDED, output={"tracker": host.name, "where": "cpu"})
    except BaseException as e:  # noqa: BLE001
        state = P.KILLED if run.kill.is_set() else P.FAILED
        host._finish(run, state, f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")


def run_split_reduce(host, run, device=None):
    """The collective reduce of a split job on this tracker: combine the
    committed map outputs held here, then ``reduce`` (collectives over
    ``host.comm``).  ``device``: the tracker's GPU (combine + reduce on it)."""
    from ..mapred.tasktracker import TaskContext
    spec, js = run.spec, run.job
    run.status.start_time = time.time()
    if TRACE.on:
        TRACE.instant("tt.reduce.start", attempt=spec.attempt_id)
    try:
        crash = getattr(host, "_maybe_inject_crash", None)
        if crash is not None:
            crash(run)          # GPU worker crash injection (tests of crash isolation)
        fail_on = js.conf.get("hbmr.faultinject.reduce.fail.attempt")
        if fail_on and fail_on in spec.attempt_id:
            # an ordinary task failure (not a crash): the attempt FAILS and the
            # JobTracker re-runs the collective gang on the same worker
            raise RuntimeError(f"injected reduce failure ({spec.attempt_id})")
        rep = TaskReporter()
        run.task = SplitTaskShim(rep, run.kill)
        ctx = TaskContext(host, js, spec, rep)
        comm = getattr(host, "comm", None)
        before = dict(getattr(comm, "stats", None) or {})
        with js.lock:
            outs = [js.map_outputs[a] for _tid, a, _o in spec.map_outputs if a in js.map_outputs]
        missing = [a for _tid, a, _o in spec.map_outputs if a not in js.map_outputs]
        if missing:
            raise RuntimeError(f"map outputs lost on {host.name}: {missing[:4]}")
        if device is not None and device.type == "cuda":
            import torch
            ctx.device = device
            with torch.cuda.device(device):
                combined = js.split_job.combine(ctx, outs)
                if TRACE.on:
                    TRACE.instant("tt.reduce.combined", attempt=spec.attempt_id)
                js.result = js.split_job.reduce(ctx, combined)
        else:
            ctx.device = None
            combined = js.split_job.combine(ctx, outs)
            if TRACE.on:
                TRACE.instant("tt.reduce.combined", attempt=spec.attempt_id)
            js.result = js.split_job.reduce(ctx, combined)
        if TRACE.on:
            TRACE.instant("tt.reduce.done", attempt=spec.attempt_id)
        with js.lock:
            js.map_outputs.clear()       # consumed
        from ..parallel.collectives import COLLECTIVE_GROUP
        for k, v in (getattr(comm, "stats", None) or {}).items():
            if v != before.get(k, 0):
                rep.incrCounter(COLLECTIVE_GROUP, k, v - before.get(k, 0))
        small = js.result if isinstance(js.result, dict) else None
        host._finish(run, P.SUCCEEDED, output={"tracker": host.name, "result": small})
    except BaseException as e:  # noqa: BLE001
        state = P.KILLED if run.kill.is_set() else P.FAILED
        host._finish(run, state, f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")
