"""Per-tracker GPU execution: one worker per device, one HIP stream per GPU slot.

A GPU map attempt is: look up (or materialise) its split in HBM, enqueue the
job's map kernels on the slot's stream between two HIP events, and hand the
end event to the slot's completion thread.  The launching thread never waits
for the device, so a slot keeps ``hbmr.gpu.queue.depth`` tasks in flight and
the GPU never idles between tasks while the tracker reports completions
(contrast: the reference's TaskLauncher blocks a GPU slot for the lifetime of
a forked child JVM + Pipes binary, TaskTracker.java:2502-2628).

The event pair's elapsed time is the attempt's *device time*; the JobTracker's
cost model uses it as the GPU task time (queueing on the stream excluded).
"""
from __future__ import annotations

import logging
import queue
import threading
import time
import traceback

import torch

from ..mapred import protocol as P
from .busy import BusyTimeline, batch_interval
from ..mapred.task import TaskReporter
from ..utils.trace import TRACE

log = logging.getLogger("hbmr.gpu")


class _Slot:
    def __init__(self, device, index):
        self.device = device
        self.index = index
        self.stream = torch.cuda.Stream(device=device)
        self.inflight = 0
        self.done_q: "queue.Queue" = queue.Queue()
        self.thread = None


class _Device:
    def __init__(self, index, slots):
        self.index = index
        self.torch_device = torch.device("cuda", index)
        self.q: "queue.Queue" = queue.Queue()
        self.slots = [_Slot(self.torch_device, i) for i in range(slots)]
        self.rr = 0
        self.thread = None
        self.queued = 0
        props = torch.cuda.get_device_properties(index)
        self.name = props.name
        self.total_mem = props.total_memory
        # maps of jobs with a cap on maps in flight (a split job's
        # max_inflight_maps: TeraSort's out-of-core mode, whose inputs are not
        # cached and whose per-map working set must stay inside its HBM budget)
        self.cap_cond = threading.Condition()
        self.capped = 0
        self.device_errors = 0      # consecutive failed batches with a device-level error
        self.last_error = ""
        # device-time accounting: batch intervals are placed on one timeline
        # (offsets from ``ref``) and a batch is charged only the busy time it
        # adds beyond the frontier, so overlapping slot streams are not
        # double-counted in the tasks' device time (the cost model's t_gpu)
        self.ref = None
        self.busy = BusyTimeline()      # union of this device's charged batch intervals


class _Batch(list):
    """A queued list of runs whose submitter waits (``picked``) until the
    launcher has put it on the device."""
    picked = None


class _NoPrefetch:
    @staticmethod
    def take(key):
        return None


class _Prefetch:
    """Host buffers of cold splits decoded ahead of their tasks (in task order,
    at most ``window`` decoded or in flight)."""

    def __init__(self, pool, sj, cold, window):
        self.pool, self.sj = pool, sj
        self.todo = list(cold)
        self.futs: dict = {}
        self.window = max(1, window)
        self._fill()

    def _fill(self):
        while self.todo and len(self.futs) < self.window:
            s = self.todo.pop(0)
            self.futs[s.key] = self.pool.submit(self.sj.load_split_host, s)

    def take(self, key):
        f = self.futs.pop(key, None)
        if f is None:
            return None
        try:
            h = f.result()
        except Exception:  # noqa: BLE001 — the per-task load reports it
            h = None
        self._fill()
        return h


class GpuRuntime:
    def __init__(self, tracker, devices, slots_per_device):
        self.tracker = tracker
        self.devices = {d: _Device(d, max(1, slots_per_device)) for d in devices}
        self.slots_per_device = max(1, slots_per_device)
        self.max_batch = max(1, tracker.conf.get_int("hbmr.gpu.batch.max", 64))
        self.first_chunk = max(1, tracker.conf.get_int("hbmr.gpu.first.chunk", 4))
        # tasks per launch after the first chunk: smaller batches reach the
        # device sooner (each costs ~10-20 µs of host work per task to prepare),
        # larger ones amortise the per-launch kernels
        self.batch_target = max(1, tracker.conf.get_int("hbmr.gpu.batch.target", 16))
        # a job whose maps were not pre-staged (nothing to wait for: the
        # device idles until they are launched) goes out in larger batches
        # after its first chunk, so the launcher's ~1 ms of host work per batch
        # stays ahead of the device (traced: a 16-task batch takes the launcher
        # about as long as the device, and the first job of a chain ran ~30 %
        # slower than the pre-staged ones behind it)
        self.batch_target_unstaged = max(1, tracker.conf.get_int(
            "hbmr.gpu.batch.target.unstaged", 32))
        # a job's last batches halve in size (see _chunks)
        self.taper = tracker.conf.get_boolean("hbmr.gpu.batch.taper", True)
        # > 0: the submitter of an idle device's first chunk waits (up to this
        # long) until it is launched.  In-process traces show the device
        # starting ~1 ms earlier, but same-box A/Bs of the bench measured no
        # end-to-end gain (worker process: 33.7 vs 35.5 ms median), so off
        self.handoff_s = tracker.conf.get_float("hbmr.gpu.first.chunk.handoff.ms", 0.0) / 1e3
        # > 0: a slot's completer polls its batch's end event at this period
        # instead of blocking in hipEventSynchronize, which (traced on the box)
        # held up other threads' operations on the same stream — an early
        # reduce's wait on the batch, the launcher's next batch — until the
        # batch finished
        self.poll_s = tracker.conf.get_float("hbmr.gpu.completion.poll.us", 100.0) / 1e6
        self._stop = threading.Event()
        reserve = tracker.conf.get_float("hbmr.gpu.hbm.reserve.gb", 16.0) * (1 << 30)
        for d, dev in self.devices.items():
            tracker.split_cache.capacity[d] = max(0, int(dev.total_mem - reserve))
        from .split_cache import configure as _configure_split_cache
        _configure_split_cache(tracker)
        from .gates import Gates
        self.gates = Gates()

    def torch_device(self, d):
        return self.devices[d].torch_device

    # -- staged maps (hbmr/gpu/gates.py) ---------------------------------------------------
    def open_gate(self, job_id, event=None, epoch=None):
        """Job ``job_id``'s reduce result is enqueued on the device (``event``):
        its staged dependents' held maps go to the slots, behind the event."""
        held = self.gates.open(job_id, event, epoch)
        if held:
            self.submit_many(held)

    def drop_held(self, job_id):
        return self.gates.drop(job_id)

    def close_gate(self, job_id):
        self.gates.close(job_id)

    def device_status(self):
        out = []
        for d, dev in self.devices.items():
            out.append(P.GpuDeviceStatus(device=d, max_slots=len(dev.slots),
                                         running=sum(s.inflight for s in dev.slots),
                                         queued=dev.q.qsize(), hbm_total=dev.total_mem,
                                         name=dev.name))
        return out

    def has_capacity(self):
        return True

    def start(self):
        for dev in self.devices.values():
            dev.thread = threading.Thread(target=self._worker, args=(dev,), daemon=True,
                                          name=f"gpu{dev.index}-launcher")
            dev.thread.start()
            for s in dev.slots:
                s.thread = threading.Thread(target=self._completer, args=(s,), daemon=True,
                                            name=f"gpu{dev.index}-slot{s.index}-done")
                s.thread.start()

    def stop(self):
        self._stop.set()
        for dev in self.devices.values():
            dev.q.put(None)
            for s in dev.slots:
                s.done_q.put(None)

    def submit(self, run):
        self.submit_many([run])

    def submit_many(self, runs):
        """Queue attempts; a job's bulk launch arrives as one list, so the
        launcher plans the whole batch at once (first_chunk).  Staged attempts
        of an unopened gate are held (open_gate)."""
        runs = self.gates.admit(runs)
        by_dev: dict = {}
        for run in runs:
            d = run.spec.gpu_device_id
            if d not in self.devices:
                # placement bug guard: never silently run on another device (B1)
                self.tracker._finish(run, P.FAILED,
                                     f"device {d} not on tracker {self.tracker.name}")
                continue
            by_dev.setdefault(d, []).append(run)
        for d, rs in by_dev.items():
            dev = self.devices[d]
            if len(rs) <= self.first_chunk and self.handoff_s > 0 and dev.q.empty() and \
                    not any(s.inflight for s in dev.slots):
                # an idle device's first chunk of a bulk launch: the caller goes
                # on to build the rest of the batch and, holding the interpreter,
                # kept the launcher from starting the device for ~0.7 ms (traced
                # on the box); wait until the chunk is on its streams
                b = _Batch(rs)
                b.picked = threading.Event()
                dev.q.put(b)
                b.picked.wait(self.handoff_s)
            else:
                dev.q.put(rs)

    # -- launcher -----------------------------------------------------------------------
    def _drain(self, dev: _Device, first, picked):
        """first + whatever else is queued right now (queue items are lists of
        runs; at least everything of ``first``, then up to max_batch); the
        submitters waiting on them are collected in ``picked``."""
        runs = list(first)
        while len(runs) < self.max_batch:
            try:
                r = dev.q.get_nowait()
            except queue.Empty:
                break
            if r is None:
                dev.q.put(None)
                break
            runs.extend(r)
            if getattr(r, "picked", None) is not None:
                picked.append(r.picked)
        return runs

    def _worker(self, dev: _Device):
        torch.cuda.set_device(dev.index)
        ref = torch.cuda.Event(enable_timing=True)
        ref.record()
        ref.synchronize()
        dev.ref = ref
        tracker = self.tracker
        from ..gpu.splitjob import SplitSpec
        from ..mapred.tasktracker import TaskContext
        while not self._stop.is_set():
            run = dev.q.get()
            if run is None:
                break
            if TRACE.on:
                TRACE.instant("gpu.wake", n=len(run) if isinstance(run, list) else 1)
            groups: dict = {}
            picked = [run.picked] if getattr(run, "picked", None) is not None else []
            for r in self._drain(dev, run, picked):
                if r.kill.is_set():
                    tracker._finish(r, P.KILLED, "killed before start")
                    continue
                groups.setdefault(id(r.job), []).append(r)
            for runs in groups.values():
                js = runs[0].job
                sj = js.split_job
                i = 0
                if hasattr(sj, "map_gpu_batch") and len(runs) > 2 * self.first_chunk and \
                        not getattr(sj, "max_inflight_maps", 0) and \
                        not any(s.inflight for s in dev.slots):
                    # idle device: start it on a few tasks while the rest are
                    # prepared (each task costs ~20 µs of host work to launch)
                    self._launch_batch(dev, runs[:self.first_chunk], js, sj, SplitSpec,
                                       TaskContext)
                    i = self.first_chunk
                # split the rest of the job's batch over the slots so streams overlap
                rest = len(runs) - i
                nslot = len(dev.slots) if hasattr(sj, "map_gpu_batch") else rest
                target = self._batch_target(runs, self.batch_target, self.batch_target_unstaged)
                per = min(self.max_batch, target, max(1, -(-rest // max(1, nslot))))
                if rest <= self.first_chunk and hasattr(sj, "map_gpu_batch"):
                    per = max(1, rest)       # a first chunk: one launch, no split
                cap = int(getattr(sj, "max_inflight_maps", 0) or 0)
                if cap > 0:
                    per = min(per, cap)
                for j, n in self._chunks(i, len(runs), per, cap == 0 and self.taper):
                    chunk = runs[j:j + n]
                    if cap > 0:
                        # the launcher waits for capped maps to complete (the
                        # completer releases them): their device memory is
                        # allocated at launch, not when the kernels run
                        with dev.cap_cond:
                            while dev.capped and dev.capped + len(chunk) > cap and \
                                    not self._stop.is_set():
                                dev.cap_cond.wait(0.5)
                            dev.capped += len(chunk)
                    n = self._launch_batch(dev, chunk, js, sj, SplitSpec, TaskContext,
                                           capped=cap > 0)
                    if cap > 0 and n < len(chunk):
                        self._release_capped(dev, len(chunk) - n)
            for ev in picked:
                ev.set()

    @staticmethod
    def _batch_target(runs, staged, unstaged):
        """Tasks per launch: pre-staged maps (released behind a gate event)
        are launched while the job before them runs, so small batches reach
        the device early; a job with nothing to wait for is on the critical
        path of an idle device, where larger batches keep the launcher ahead."""
        return staged if any(r.wait is not None for r in runs) else unstaged

    @staticmethod
    def _chunks(i, n, per, taper):
        """(start, size) of the batches of runs[i:n].  Tapered: the last
        2 x per runs go as halving batches, so the work left after a job's
        last full batch — its certification and combiner kernels, which do
        not fill the GPU — is short (the iteration tail)."""
        out, j = [], i
        while j < n:
            r = n - j
            if not taper or r > 2 * per:
                c = min(per, r)
            elif r > 4:
                c = -(-r // 2)
            else:
                c = r
            out.append((j, c))
            j += c
        return out

    @staticmethod
    def _release_capped(dev, n):
        with dev.cap_cond:
            dev.capped = max(0, dev.capped - n)
            dev.cap_cond.notify_all()

    def _launch_batch(self, dev, runs, js, sj, SplitSpec, TaskContext,  # noqa: N803
                      capped=False):
        """Launch one batch on the next slot; returns how many of its runs
        went to the device (their completion is the completer's)."""
        tracker = self.tracker
        slot = dev.slots[dev.rr % len(dev.slots)]
        dev.rr += 1
        live = []
        try:
            if sj is None:
                raise RuntimeError("GPU map of a non split-level job requires the Pipes GPU "
                                   "runner (hadoop.pipes.gpu.executable)")
            now = time.time()
            if TRACE.on:
                TRACE.instant("gpu.prep", n=len(runs))
            ctxs, datas = [], []
            prefetched = self._prefetch_hosts(dev, runs, sj, SplitSpec)
            with torch.cuda.stream(slot.stream):
                for r in runs:
                    rep = TaskReporter()
                    r.task = _Shim(rep, r.kill)
                    try:
                        tracker._maybe_inject_fault(r)
                        sspec = SplitSpec.from_dict(r.spec.split)
                        host = prefetched.take(sspec.key)
                        if host is not None:
                            loader = (lambda s=sspec, h=host:
                                      sj.load_split_from_host(s, h, dev.torch_device))
                        else:
                            loader = (lambda s=sspec: sj.load_split(s, dev.torch_device))
                        data, hit = tracker.split_cache.get_or_load(
                            sspec.key, dev.index, loader, sj.split_nbytes,
                            cache=getattr(sj, "cache_inputs", True))
                    except BaseException as e:  # noqa: BLE001
                        tracker._finish(r, P.FAILED, f"{type(e).__name__}: {e}\n"
                                                     f"{traceback.format_exc()[-2000:]}")
                        continue
                    rep.incrCounter("hbmr.GpuCounters",
                                    "GPU_SPLIT_CACHE_HITS" if hit else "GPU_SPLIT_CACHE_MISSES")
                    r.status.start_time = now
                    ctxs.append(TaskContext(tracker, js, r.spec, rep, device=dev.torch_device,
                                            stream=slot.stream))
                    datas.append(data)
                    live.append(r)
                if not live:
                    return 0
                # staged attempts: the job they depend on enqueued its reduce
                # result; the kernels wait for it on the device, not the host
                waits = {id(r.wait): r.wait for r in live if r.wait is not None}
                for w in waits.values():
                    slot.stream.wait_event(w)
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                if TRACE.on:
                    TRACE.instant("gpu.native", n=len(live))
                ev0.record(slot.stream)
                if len(live) > 1 and hasattr(sj, "map_gpu_batch"):
                    outs = sj.map_gpu_batch(ctxs, datas)
                else:
                    outs = [sj.map_gpu(c, d) for c, d in zip(ctxs, datas)]
                ev1.record(slot.stream)
                # the marker an early reduce orders itself behind: an event of
                # its own, because HIP serialises operations on one event — a
                # stream wait on ev1 blocked the reduce thread on the host for
                # as long as the completer sat in ev1.synchronize() (traced on
                # the box: the combine was enqueued only after the last map
                # finished, ~1.5 ms of idle before each update and again
                # before the next job's first assign)
                evr = torch.cuda.Event()
                evr.record(slot.stream)
            slot.inflight += len(live)
            if TRACE.on:
                TRACE.instant("gpu.launch", n=len(live), slot=slot.index)
            # an early collective reduce may consume the outputs now, ordered
            # behind evr on its own stream
            by_job: dict = {}
            for r, out in zip(live, outs):
                by_job.setdefault(id(r.job), (r.job, []))[1].append((r.spec.attempt_id, out, evr))
            for js, items in by_job.values():
                js.note_launched(items)
            slot.done_q.put((live, ev0, ev1, outs, capped, list(waits.values())))
            return len(live)
        except BaseException as e:  # noqa: BLE001
            self._note_error(dev.index, e)
            for r in (live or runs):
                if r.status.state not in P.TERMINAL:
                    tracker._finish(r, P.FAILED,
                                    f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")
            return 0

    def _prefetch_hosts(self, dev, runs, sj, SplitSpec):  # noqa: N803
        """Cold splits of a batch whose job can load them on the host
        (``load_split_host``: file decode into pinned memory) are read by a
        thread pool ahead of their tasks, a bounded window at a time; each task
        takes its buffer when it is its turn, so the H2D copies on the slot's
        stream overlap the decoding of the splits behind it."""
        if sj is None or not hasattr(sj, "load_split_host"):
            return _NoPrefetch
        cold = []
        for r in runs:
            sspec = SplitSpec.from_dict(r.spec.split)
            if sspec.kind == "file" and \
                    self.tracker.split_cache.get(sspec.key, dev.index) is None:
                cold.append(sspec)
        if len(cold) < 2:
            return _NoPrefetch
        import concurrent.futures as cf
        n = max(1, self.tracker.conf.get_int("hbmr.gpu.load.threads", 8))
        if getattr(self, "_loader_pool", None) is None:
            self._loader_pool = cf.ThreadPoolExecutor(n, thread_name_prefix="split-loader")
        return _Prefetch(self._loader_pool, sj, cold, window=2 * n)

    def _completer(self, slot: _Slot):
        torch.cuda.set_device(slot.device)
        tracker = self.tracker
        where = f"cuda:{slot.device.index}"
        while True:
            item = slot.done_q.get()
            if item is None:
                break
            runs, ev0, ev1, outs, capped, gates = item
            try:
                if self.poll_s > 0:
                    while not ev1.query():
                        time.sleep(self.poll_s)
                else:
                    ev1.synchronize()
                if TRACE.on:
                    TRACE.instant("gpu.complete", n=len(runs), slot=slot.index)
                # a batch completes together; the busy time it adds to the
                # device (beyond what overlapping batches on the other slots
                # already account for, from when its gates let it start) is
                # shared evenly by its tasks
                dt = self._busy_ms(self.devices[slot.device.index], ev0, ev1, gates) / 1000.0 / \
                    max(1, len(runs))
                for r, out in zip(runs, outs):   # a batch may mix jobs
                    with r.job.lock:
                        r.job.map_outputs[r.spec.attempt_id] = out
                self.devices[slot.device.index].device_errors = 0
                # one compact report for the batch (JobTracker._bulk_succeeded)
                agg = _merge_counters(runs)
                agg.incr("hbmr.GpuCounters", "GPU_KERNEL_US", int(dt * 1e6) * len(runs))
                tracker.finish_bulk(runs, dt, {"tracker": tracker.name, "where": where},
                                    agg.to_dict())
                news = getattr(tracker, "maps_done_news", None)
                if news is not None:
                    news({r.spec.job_id for r in runs})
                else:
                    tracker.notify_jobtracker()
            except BaseException as e:  # noqa: BLE001
                self._note_error(slot.device.index, e)
                for r in runs:
                    tracker._finish(r, P.FAILED,
                                    f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")
            finally:
                slot.inflight -= len(runs)
                if capped:
                    self._release_capped(self.devices[slot.device.index], len(runs))

    @staticmethod
    def _busy_ms(dev, ev0, ev1, gates=()):
        """The device time a batch adds (hbmr/gpu/busy.py): its [start, end)
        on the device clock — start no earlier than the gate events its
        stream waited on — charged against the union of the device's batches."""
        elapsed = ev0.elapsed_time(ev1)
        if dev.ref is None:
            return elapsed
        gate_ms = []
        for g in gates or ():
            try:
                gate_ms.append(dev.ref.elapsed_time(g))
            except RuntimeError:        # an event without timing: start at ev0
                pass
        start, end = batch_interval(dev.ref.elapsed_time(ev0), elapsed, gate_ms)
        return dev.busy.charge(start, end)

    # -- device health (NodeHealthChecker probes) --------------------------------------
    def _note_error(self, d, exc):
        """Count consecutive device-level failures (HIP runtime errors surface as
        RuntimeError/AcceleratorError from torch or 'native error' from ops)."""
        msg = f"{type(exc).__name__}: {exc}"
        if any(s in msg for s in ("HIP", "hip", "CUDA", "Accelerator", "native error",
                                  "device-side")):
            dev = self.devices.get(d)
            if dev is not None:
                dev.device_errors += 1
                dev.last_error = msg[:500]

    def probe(self, d):
        """None if device d looks usable, else a reason (for NodeHealthChecker)."""
        dev = self.devices.get(d)
        if dev is None:
            return "unknown device"
        limit = self.tracker.conf.get_int("hbmr.gpu.max.consecutive.errors", 3)
        if dev.device_errors >= limit:
            return f"{dev.device_errors} consecutive device errors; last: {dev.last_error}"
        try:
            torch.cuda.mem_get_info(d)
        except Exception as e:  # noqa: BLE001
            return f"device query failed: {e}"
        return None


def _merge_counters(runs):
    from ..mapred.counters import Counters
    agg = Counters()
    for r in runs:
        if r.task is not None:
            agg.incr_all(r.task.reporter.counters)
    return agg


class _Shim:
    __slots__ = ("reporter", "kill_event")

    def __init__(self, reporter, kill_event):
        self.reporter = reporter
        self.kill_event = kill_event
