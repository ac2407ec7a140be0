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
        # a failure AFTER the gates opened (tests of staged-job restarts): the
        # attempt publishes a poisoned result (split_job.poison_result), lets
        # the staged maps run on it, then fails
        late = js.conf.get("hbmr.faultinject.reduce.fail.after.release.attempt")
        late = bool(late) and late in spec.attempt_id
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
            js.split_job.split_nbytes, cache=getattr(js.split_job, "cache_inputs", True))
        out = js.split_job.map_cpu(ctx, data)
        with js.lock:
            js.map_outputs[spec.attempt_id] = out
        rep.incrCounter(C.JOB_GROUP, C.CPU_MAP_TASKS, 0)
        host._finish(run, P.SUCCEEDED, output={"tracker": host.name, "where": "cpu"})
    except BaseException as e:  # noqa: BLE001
        state = P.KILLED if run.kill.is_set() else P.FAILED
        host._finish(run, state, f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")


def _gather_outputs(js, spec, run):
    """The map outputs this collective reduce combines, and their readiness
    markers.  A reduce launched early (``spec.expect``) waits until every
    expected attempt's kernels are ENQUEUED (JobState.note_launched): each
    output comes with its batch's end event (device) or simulated ready time,
    so the reduce orders itself behind the maps on the device instead of
    waiting on the host for them to finish."""
    want = [a for _tid, a, _o in spec.map_outputs]
    if not spec.expect:
        with js.lock:
            outs = [js.map_outputs[a] for a in want if a in js.map_outputs]
            missing = [a for a in want if a not in js.map_outputs]
        if missing:
            raise RuntimeError(f"map outputs lost: {missing[:4]}")
        return outs, [None] * len(outs)
    with js.cond:
        while True:
            if run.kill.is_set():
                raise RuntimeError("killed while waiting for its expected map outputs")
            bad = [a for a in want if a in js.failed]
            if bad:
                raise RuntimeError(f"expected map attempts failed: {bad[:4]}")
            if all(a in js.map_outputs or a in js.launched for a in want):
                break
            js.cond.wait(0.5)
        outs, marks = [], []
        for a in want:
            if a in js.map_outputs:
                outs.append(js.map_outputs[a])
                marks.append(None)
            else:
                o, m = js.launched[a]
                outs.append(o)
                marks.append(m)
    return outs, marks


def _reduce_stream(host, device):
    """The tracker's reduce stream, shared by its reduce attempts.  (A pool of
    streams, one per attempt, measured worse: with 4 hardware queues per
    process the streams share queues, and an early reduce's wait on maps not
    yet finished blocks whatever follows it in its queue — consecutive jobs
    then completed in threes instead of pairs.  What must not queue behind a
    later job's waits is enqueued before them instead: see the KMeans reduce's
    centroid read-back.)"""
    import torch
    st = host.__dict__.get("_reduce_stream")
    if st is None:
        st = host.__dict__.setdefault("_reduce_stream", torch.cuda.Stream(device=device))
    return st


def run_split_reduce(host, run, device=None):
    """The collective reduce of a split job on this tracker: combine the
    committed map outputs held here, then ``reduce`` (collectives over
    ``host.comm``).  ``device``: the tracker's GPU (combine + reduce on it, on
    a reduce stream of its own).  As soon as the reduce has *enqueued* its
    result (the split job calls ``ctx.release_dependents()``, else when
    ``reduce`` returns) the maps of jobs staged behind this one are released
    on this tracker's GPU runtime, behind a device event (hbmr/gpu/gates.py)."""
    from ..mapred.tasktracker import TaskContext
    spec, js = run.spec, run.job
    run.status.start_time = time.time()
    if TRACE.on:
        TRACE.instant("tt.reduce.start", attempt=spec.attempt_id, expect=spec.expect)
    try:
        crash = getattr(host, "_maybe_inject_crash", None)
        if crash is not None:
            crash(run)          # GPU worker crash injection (tests of crash isolation)
        fail_on = js.conf.get("hbmr.faultinject.reduce.fail.attempt")
        if fail_on and fail_on in spec.attempt_id:
            # an ordinary task failure (not a crash): the attempt FAILS and the
            # JobTracker re-runs the collective gang on the same worker
            raise RuntimeError(f"injected reduce failure ({spec.attempt_id})")
        # a failure AFTER the gates opened (tests of staged-job restarts): the
        # attempt publishes a poisoned result (split_job.poison_result), lets
        # the staged maps run on it, then fails
        late = js.conf.get("hbmr.faultinject.reduce.fail.after.release.attempt")
        late = bool(late) and late in spec.attempt_id
        rep = TaskReporter()
        run.task = SplitTaskShim(rep, run.kill)
        ctx = TaskContext(host, js, spec, rep)
        # a reduce killed by a gang restart must not publish its result (the
        # restarted gang's attempt publishes the same key): the split job
        # checks this right before it does
        ctx.killed = run.kill.is_set
        hconf = getattr(host, "conf", None)
        if hconf is not None and hconf.get_boolean("hbmr.gpu.simulate.nodata", False) and \
                (hconf.get("hbmr.gpu.simulate.collective") or "device") == "device":
            # control-plane rehearsal without data: the device collective (RCCL
            # all-reduce over xGMI) is modelled as device time like the maps are,
            # instead of moving zeros through gloo on the host
            ctx.simulated_collective_s = hconf.get_float(
                "hbmr.gpu.simulate.collective.ms", 0.1) / 1e3
        comm = getattr(host, "comm", None)
        before = dict(getattr(comm, "stats", None) or {})
        try:
            outs, marks = _gather_outputs(js, spec, run)
        except RuntimeError as e:
            raise RuntimeError(f"{e} on {host.name}") from None
        if TRACE.on:
            TRACE.instant("tt.reduce.gathered", attempt=spec.attempt_id, n=len(outs))
        cuda = device is not None and device.type == "cuda"
        rt = getattr(host, "gpu_runtime", None)
        released = [False]
        gates = getattr(rt, "gates", None)
        gate_epoch = gates.epoch(spec.job_id) if gates is not None else None

        def release_dependents():
            if released[0]:
                return
            released[0] = True
            if late and hasattr(js.split_job, "poison_result"):
                js.split_job.poison_result(ctx)
            if rt is None or not hasattr(rt, "open_gate"):
                return
            ev = getattr(ctx, "sim_ready", None)   # simulated device: a ready time
            if cuda:
                import torch
                # timed: a staged batch's device time starts when this fires
                # (hbmr/gpu/busy.py batch_interval), not at its stream's wait
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
            rt.open_gate(spec.job_id, ev, gate_epoch)
            if TRACE.on:
                TRACE.instant("tt.reduce.gate_open", job=spec.job_id)
        ctx.release_dependents = release_dependents
        if cuda:
            import torch
            ctx.device = device
            with torch.cuda.device(device), torch.cuda.stream(_reduce_stream(host, device)):
                cur = torch.cuda.current_stream()
                if getattr(js.split_job, "orders_own_outputs", False):
                    # the split job waits on each output's event itself (e.g.
                    # TeraSort's shuffle waves: early outputs move while later
                    # maps still run)
                    ctx.output_marks = marks
                else:
                    for ev in {id(m): m for m in marks if m is not None}.values():
                        cur.wait_event(ev)
                    if TRACE.on:
                        TRACE.instant("tt.reduce.waited", attempt=spec.attempt_id)
                combined = js.split_job.combine(ctx, outs)
                if TRACE.on:
                    TRACE.instant("tt.reduce.combined", attempt=spec.attempt_id)
                js.result = js.split_job.reduce(ctx, combined)
                release_dependents()
        else:
            real = [m for m in marks if m is not None]
            if real and getattr(ctx, "simulated_collective_s", None) is not None:
                # no-data rehearsal: the reduce's device work queues behind the
                # maps (as the real reduce stream waits on their events) — the
                # split job orders its simulated result after this time
                ctx.sim_base = max(real)
            elif real:
                # simulated device: the outputs are "ready" at these times
                delay = max(real) - time.time()
                if delay > 0:
                    time.sleep(delay)
            ctx.device = None
            combined = js.split_job.combine(ctx, outs)
            if TRACE.on:
                TRACE.instant("tt.reduce.combined", attempt=spec.attempt_id)
            js.result = js.split_job.reduce(ctx, combined)
            release_dependents()
        if late:
            raise RuntimeError(f"injected reduce failure after release ({spec.attempt_id})")
        if TRACE.on:
            TRACE.instant("tt.reduce.done", attempt=spec.attempt_id)
        with js.lock:
            js.map_outputs.clear()       # consumed
            js.launched.clear()
        from ..parallel.collectives import COLLECTIVE_GROUP
        for k, v in (getattr(comm, "stats", None) or {}).items():
            if v != before.get(k, 0):
                rep.incrCounter(COLLECTIVE_GROUP, k, v - before.get(k, 0))
        small = js.result if isinstance(js.result, dict) else None
        host._finish(run, P.SUCCEEDED, output={"tracker": host.name, "result": small})
    except BaseException as e:  # noqa: BLE001
        state = P.KILLED if run.kill.is_set() else P.FAILED
        host._finish(run, state, f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")
