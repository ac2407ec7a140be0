"""GPU slots without a GPU: a TaskTracker runtime that behaves like
:class:`~hbmr.gpu.runtime.GpuRuntime` (per-device launcher, per-slot in-order
"streams", batched launches, asynchronous completion, device time reported to
the cost model) but executes split-level map tasks with the job's CPU map
function and charges a configurable simulated device time per task.

Enabled with ``hbmr.gpu.simulate=true`` on a tracker that has GPU device ids.
It lets the hybrid scheduler, GPU placement, speculative GPU backups, split
caching and the collective reduce be exercised (and the control plane be
profiled) on machines without a GPU — the role the reference's unit tests gave
to fake trackers with ``availableGPUDevices`` set
(src/test/org/apache/hadoop/mapred/TestJobQueueTaskScheduler.java:183-201).

Keys:
  hbmr.gpu.simulate.task.ms   simulated device time per map task (default 0); the
                              device runs one task at a time whatever its slot count
  hbmr.gpu.simulate.hbm.gb    simulated HBM size per device (default 288)
  hbmr.gpu.simulate.nodata    do not materialise splits and skip the map
                              function (the job's ``map_sim`` hook, if any,
                              still runs on a ``None`` split): control-plane
                              and collective timing at full problem size
"""
from __future__ import annotations

import heapq
import logging
import queue
import threading
import time
import traceback

import torch

from ..mapred import protocol as P
from ..mapred.task import TaskReporter
from ..utils.trace import TRACE

log = logging.getLogger("hbmr.gpu.sim")


_NO_DATA = ("simulated split",)   # cache placeholder of an unmaterialised split


class _SimSlot:
    def __init__(self, index):
        self.index = index
        self.busy_until = 0.0
        self.inflight = 0


class _SimDevice:
    def __init__(self, index, slots, hbm):
        self.index = index
        self.q: "queue.Queue" = queue.Queue()
        self.slots = [_SimSlot(i) for i in range(slots)]
        self.rr = 0
        self.thread = None
        self.total_mem = hbm
        self.name = "simulated-gfx950"
        self.busy_until = 0.0     # the slots' streams share one device


class SimulatedGpuRuntime:
    def __init__(self, tracker, devices, slots_per_device):
        conf = tracker.conf
        self.tracker = tracker
        hbm = int(conf.get_float("hbmr.gpu.simulate.hbm.gb", 288.0) * (1 << 30))
        self.devices = {d: _SimDevice(d, max(1, slots_per_device), hbm) for d in devices}
        self.task_s = conf.get_float("hbmr.gpu.simulate.task.ms", 0.0) / 1000.0
        self.max_batch = max(1, conf.get_int("hbmr.gpu.batch.max", 64))
        self.nodata = conf.get_boolean("hbmr.gpu.simulate.nodata", False)
        self._stop = threading.Event()
        self._done: list = []          # heap of (ready_time, seq, item)
        self._done_cv = threading.Condition()
        self._seq = 0
        self._completer = None
        reserve = conf.get_float("hbmr.gpu.hbm.reserve.gb", 16.0) * (1 << 30)
        for d, dev in self.devices.items():
            tracker.split_cache.capacity[d] = max(0, int(dev.total_mem - reserve))
        from .split_cache import configure as _configure_split_cache
        _configure_split_cache(tracker)
        from .gates import Gates
        self.gates = Gates()

    def torch_device(self, d):
        return torch.device("cpu")

    def open_gate(self, job_id, event=None, epoch=None):
        """Staged maps held for ``job_id`` go to the device queue; a simulated
        device runs them after its earlier work (busy_until), as a stream would."""
        held = self.gates.open(job_id, event, epoch)
        if held:
            self.submit_many(held)

    def drop_held(self, job_id):
        return self.gates.drop(job_id)

    def close_gate(self, job_id):
        self.gates.close(job_id)

    def device_status(self):
        return [P.GpuDeviceStatus(device=d, max_slots=len(dev.slots),
                                  running=sum(s.inflight for s in dev.slots),
                                  queued=dev.q.qsize(), hbm_total=dev.total_mem, name=dev.name)
                for d, dev in self.devices.items()]

    def has_capacity(self):
        return True

    def probe(self, d):
        """Device health for NodeHealthChecker: ``hbmr.gpu.simulate.bad.devices``
        lists devices that report a fault (tests the unhealthy-GPU path)."""
        bad = self.tracker.conf.get("hbmr.gpu.simulate.bad.devices", "") or ""
        return "simulated device fault" if str(d) in [x.strip() for x in bad.split(",")] else None

    def start(self):
        for dev in self.devices.values():
            dev.thread = threading.Thread(target=self._worker, args=(dev,), daemon=True,
                                          name=f"simgpu{dev.index}-launcher")
            dev.thread.start()
        self._completer = threading.Thread(target=self._complete_loop, daemon=True,
                                           name="simgpu-done")
        self._completer.start()

    def stop(self):
        self._stop.set()
        for dev in self.devices.values():
            dev.q.put(None)
        with self._done_cv:
            self._done_cv.notify_all()

    def submit(self, run):
        self.submit_many([run])

    def submit_many(self, runs):
        runs = self.gates.admit(runs)
        by_dev: dict = {}
        for run in runs:
            d = run.spec.gpu_device_id
            if d not in self.devices:
                self.tracker._finish(run, P.FAILED,
                                     f"device {d} not on tracker {self.tracker.name}")
                continue
            by_dev.setdefault(d, []).append(run)
        for d, rs in by_dev.items():
            self.devices[d].q.put(rs)

    def _drain(self, dev, first):
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
        return runs

    def _worker(self, dev: _SimDevice):
        from ..gpu.splitjob import SplitSpec
        from ..mapred.tasktracker import TaskContext
        tracker = self.tracker
        while not self._stop.is_set():
            run = dev.q.get()
            if run is None:
                break
            slot = dev.slots[dev.rr % len(dev.slots)]
            dev.rr += 1
            live, outs = [], []
            now = time.time()
            # the real launcher starts an idle device on its first chunk while
            # it prepares the rest (GpuRuntime._worker): the device time of
            # this batch starts once that many tasks are prepared
            first = max(1, self.tracker.conf.get_int("hbmr.gpu.first.chunk", 4))
            t_first = None
            for r in self._drain(dev, run):
                if t_first is None and len(live) >= first:
                    t_first = time.time()
                if r.kill.is_set():
                    tracker._finish(r, P.KILLED, "killed before start")
                    continue
                js, sj = r.job, r.job.split_job
                rep = TaskReporter()
                r.task = _Shim(rep, r.kill)
                try:
                    if sj is None:
                        raise RuntimeError("GPU map of a non split-level job requires the Pipes "
                                           "GPU runner (hadoop.pipes.gpu.executable)")
                    tracker._maybe_inject_fault(r)
                    sspec = SplitSpec.from_dict(r.spec.split)
                    if self.nodata:
                        data, hit = tracker.split_cache.get_or_load(
                            sspec.key, dev.index, lambda: _NO_DATA, lambda _d, n=sspec.length: n)
                        data = None
                    else:
                        data, hit = tracker.split_cache.get_or_load(
                            sspec.key, dev.index, lambda s=sspec: sj.load_split(s, "cpu"),
                            sj.split_nbytes, cache=getattr(sj, "cache_inputs", True))
                    rep.incrCounter("hbmr.GpuCounters",
                                    "GPU_SPLIT_CACHE_HITS" if hit else "GPU_SPLIT_CACHE_MISSES")
                    r.status.start_time = now
                    ctx = TaskContext(tracker, js, r.spec, rep, device="cpu")
                    fn = getattr(sj, "map_sim", None)
                    if fn is None:
                        fn = (lambda _c, _d: None) if self.nodata else sj.map_cpu
                    outs.append(fn(ctx, data))
                    live.append(r)
                except BaseException as e:  # noqa: BLE001
                    tracker._finish(r, P.FAILED, f"{type(e).__name__}: {e}\n"
                                                 f"{traceback.format_exc()[-2000:]}")
            if not live:
                continue
            # the slots are streams of ONE device: work on any slot queues behind
            # the device's earlier work (task.ms is the device's time per task)
            start = max(t_first or time.time(), dev.busy_until)
            # staged runs of an opened gate: not before the reduce's (simulated)
            # device result is ready
            waits = [r.wait for r in live if isinstance(getattr(r, "wait", None), float)]
            if waits:
                start = max(start, max(waits))
            slot.busy_until = dev.busy_until = start + self.task_s * len(live)
            slot.inflight += len(live)
            # outputs for an early collective reduce, "ready" at the simulated end
            by_job: dict = {}
            for r, out in zip(live, outs):
                by_job.setdefault(id(r.job), (r.job, []))[1].append(
                    (r.spec.attempt_id, out, slot.busy_until))
            for js, items in by_job.values():
                js.note_launched(items)
            if TRACE.on:
                TRACE.instant("gpu.launch", n=len(live))
            with self._done_cv:
                self._seq += 1
                heapq.heappush(self._done, (slot.busy_until, self._seq, (slot, live, outs)))
                self._done_cv.notify()

    def _complete_loop(self):
        tracker = self.tracker
        while not self._stop.is_set():
            with self._done_cv:
                while not self._done and not self._stop.is_set():
                    self._done_cv.wait()
                if self._stop.is_set():
                    return
                ready, _, item = self._done[0]
                delay = ready - time.time()
                if delay > 0:
                    self._done_cv.wait(delay)
                    continue
                heapq.heappop(self._done)
            slot, runs, outs = item
            if TRACE.on:
                TRACE.instant("gpu.complete", n=len(runs))
            for r, out in zip(runs, outs):   # a batch may mix jobs
                with r.job.lock:
                    r.job.map_outputs[r.spec.attempt_id] = out
            finish_bulk = getattr(tracker, "finish_bulk", None)
            if finish_bulk is not None:
                finish_bulk(runs, self.task_s, {"tracker": tracker.name, "where": "simgpu"})
            else:
                for r in runs:
                    tracker._finish(r, P.SUCCEEDED, output={"tracker": tracker.name,
                                                            "where": "simgpu"},
                                    device_time=self.task_s, wake=False)
            slot.inflight -= len(runs)
            news = getattr(tracker, "maps_done_news", None)
            if finish_bulk is not None and news is not None:
                news({r.spec.job_id for r in runs})
            else:
                tracker.notify_jobtracker()


class _Shim:
    __slots__ = ("reporter", "kill_event")

    def __init__(self, reporter, kill_event):
        self.reporter = reporter
        self.kill_event = kill_event
