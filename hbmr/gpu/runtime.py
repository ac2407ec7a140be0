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
from ..mapred.task import TaskReporter

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


class GpuRuntime:
    def __init__(self, tracker, devices, slots_per_device):
        self.tracker = tracker
        self.devices = {d: _Device(d, max(1, slots_per_device)) for d in devices}
        self.slots_per_device = max(1, slots_per_device)
        self._stop = threading.Event()
        reserve = tracker.conf.get_float("hbmr.gpu.hbm.reserve.gb", 16.0) * (1 << 30)
        for d, dev in self.devices.items():
            tracker.split_cache.capacity[d] = max(0, int(dev.total_mem - reserve))

    def torch_device(self, d):
        return self.devices[d].torch_device

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
        d = run.spec.gpu_device_id
        if d not in self.devices:
            # placement bug guard: never silently run on another device (B1)
            self.tracker._finish(run, P.FAILED, f"device {d} not on tracker {self.tracker.name}")
            return
        self.devices[d].q.put(run)

    # -- launcher -----------------------------------------------------------------------
    def _worker(self, dev: _Device):
        torch.cuda.set_device(dev.index)
        tracker = self.tracker
        from ..gpu.splitjob import SplitSpec
        from ..mapred.tasktracker import TaskContext
        while not self._stop.is_set():
            run = dev.q.get()
            if run is None:
                break
            if run.kill.is_set():
                tracker._finish(run, P.KILLED, "killed before start")
                continue
            slot = dev.slots[dev.rr % len(dev.slots)]
            dev.rr += 1
            js = run.job
            rep = TaskReporter()

            class _Shim:
                reporter = rep
                kill_event = run.kill
            run.task = _Shim()
            try:
                tracker._maybe_inject_fault(run)
                sj = js.split_job
                if sj is None:
                    raise RuntimeError("GPU map of a non split-level job requires the Pipes GPU "
                                       "runner (hadoop.pipes.gpu.executable)")
                sspec = SplitSpec.from_dict(run.spec.split)
                ctx = TaskContext(tracker, js, run.spec, rep, device=dev.torch_device,
                                  stream=slot.stream)
                run.status.start_time = time.time()
                with torch.cuda.stream(slot.stream):
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev1 = torch.cuda.Event(enable_timing=True)
                    data, hit = tracker.split_cache.get_or_load(
                        sspec.key, dev.index, lambda: sj.load_split(sspec, dev.torch_device),
                        sj.split_nbytes)
                    rep.incrCounter("hbmr.GpuCounters",
                                    "GPU_SPLIT_CACHE_HITS" if hit else "GPU_SPLIT_CACHE_MISSES")
                    ev0.record(slot.stream)
                    out = sj.map_gpu(ctx, data)
                    ev1.record(slot.stream)
                slot.inflight += 1
                slot.done_q.put((run, ev0, ev1, out))
            except BaseException as e:  # noqa: BLE001
                tracker._finish(run, P.FAILED,
                                f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")

    def _completer(self, slot: _Slot):
        torch.cuda.set_device(slot.device)
        tracker = self.tracker
        while True:
            item = slot.done_q.get()
            if item is None:
                break
            run, ev0, ev1, out = item
            try:
                ev1.synchronize()
                dt = ev0.elapsed_time(ev1) / 1000.0
                js = run.job
                with js.lock:
                    js.map_outputs[run.spec.attempt_id] = out
                run.task.reporter.incrCounter("hbmr.GpuCounters", "GPU_KERNEL_MS", int(dt * 1e6))
                tracker._finish(run, P.SUCCEEDED, output={"tracker": tracker.name,
                                                          "where": f"cuda:{slot.device.index}"},
                                device_time=dt)
            except BaseException as e:  # noqa: BLE001
                tracker._finish(run, P.FAILED,
                                f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")
            finally:
                slot.inflight -= 1
