"""TaskTracker side of the per-GPU worker process (:mod:`hbmr.gpu.worker`).

:class:`RemoteGpuRuntime` has the interface of the in-process
:class:`~hbmr.gpu.runtime.GpuRuntime` (``submit``, ``device_status``,
``probe``, ...) plus the routes for a split job's other tasks (``submit_cpu``,
``submit_reduce``: they run where the job's map outputs live).  Batches of
attempts cross the socketpair as one frame each way, so the extra hop costs
one pickle per batch, not per task.

Crash isolation (the reference's "a crashed GPU binary is a failed attempt",
Application.java:274-290, JvmManager.java:413-485):

* the worker's death (EOF on the socket) fails every attempt it was running
  with the exit status in the diagnostics, and reports the map outputs it
  held (succeeded maps whose job has not reduced yet) as lost, so the
  JobTracker re-executes them (JobTracker._outputs_lost);
* world = 1: a fresh worker is started at once (a new child process: never an
  exec of a GPU-initialised process — this process never initialises HIP);
* world > 1: the dead worker's peers may be blocked in a collective with it,
  so the tracker reports ``gpu_worker_lost`` and the JobTracker restarts the
  whole gang with a new communicator generation (restart_gpu_worker action).
"""
from __future__ import annotations

import logging
import os
import socket
import subprocess
import sys
import threading
import time

from ..mapred import protocol as P
from ..mapred.counters import Counters
from ..utils.trace import TRACE
from .worker import recv_msg, send_msg

log = logging.getLogger("hbmr.gpu.remote")

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Reported:
    """run.task of an attempt that ran in the worker: its final counters."""
    __slots__ = ("reporter", "kill_event", "counters")

    def __init__(self, counters):
        self.reporter = self
        self.kill_event = None
        self.counters = counters


class RemoteGpuRuntime:
    remote = True

    def __init__(self, tracker, devices, slots_per_device):
        self.tracker = tracker
        self.devices = list(devices)
        self.slots_per_device = max(1, slots_per_device)
        conf = tracker.conf
        self.simulate = conf.get_boolean("hbmr.gpu.simulate", False)
        self.max_restarts = conf.get_int("hbmr.gpu.worker.max.restarts", 8)
        self.start_timeout = conf.get_int("hbmr.gpu.worker.start.timeout.s", 300)
        self.inflight: dict = {}          # attempt id -> _Running (tracker side)
        self.held: dict = {}              # job id -> succeeded map attempts held by the worker
        self.resident: set = set()        # (split key, device) in the worker's HBM cache
        self.jobs_sent: set = set()
        self.devinfo: list = []
        self.worker_info: dict = {}
        self.generation = 0
        self.restarts = 0
        self.deaths = 0
        self.last_exit = None
        self._lock = threading.Lock()
        self._send_lock = threading.Lock()
        self._stopping = False
        self._expect_death = False
        self._up = False              # a live worker is accepting work
        self._backlog: list = []      # (kind, runs) submitted while no worker was up
        self.proc = None
        self.sock = None
        self._reader = None
        self._probe_replies: dict = {}
        self._probe_ev = threading.Event()

    # -- lifecycle --------------------------------------------------------------------
    def start(self):
        self._spawn()

    def _spawn(self):
        tr = self.tracker
        parent, child = socket.socketpair()
        env = dict(os.environ)
        if "{rank}" in env.get("HBMR_TRACE", ""):
            # the worker's own trace dump beside the tracker's
            env["HBMR_TRACE"] = env["HBMR_TRACE"].replace("{rank}", "{rank}_worker")
        env["PYTHONPATH"] = _ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH")
                                     else "")
        hwq = tr.conf.get_int("hbmr.gpu.hw.queues", 8 if tr.world_size > 1 else 0)
        if hwq > 0 and "GPU_MAX_HW_QUEUES" not in os.environ:
            # a stream per hardware queue: HIP maps streams onto 4 queues by
            # default, and a queue shared by two streams blocks one behind the
            # other's waits on unfinished work (measured: a pool of reduce
            # streams made jobs complete in threes).  One rank uses 4 streams
            # (default, two slots, reduce); several ranks add RCCL's stream
            env["GPU_MAX_HW_QUEUES"] = str(min(hwq, 32))
        self.proc = subprocess.Popen([sys.executable, "-m", "hbmr.gpu.worker",
                                      str(child.fileno())], pass_fds=(child.fileno(),),
                                     env=env, cwd=_ROOT)
        child.close()
        self.sock = parent
        wc = getattr(tr, "worker_comm", None)
        init = {"conf": tr.conf.to_dict(), "name": tr.name, "rank": tr.rank,
                "world": tr.world_size, "cpu_threads": tr.cpu_threads,
                "cpu_slots": max(1, tr.cpu_slots), "devices": self.devices,
                "slots": self.slots_per_device, "simulate": self.simulate,
                "generation": self.generation,
                "comm": dict(wc) if wc else None,
                "log_level": logging.getLogger().level or logging.WARNING}
        send_msg(parent, ("init", init), self._send_lock)
        parent.settimeout(self.start_timeout)
        msg = recv_msg(parent)
        parent.settimeout(None)
        if msg is None or msg[0] != "ready":
            rc = self.proc.wait(timeout=30)
            raise RuntimeError(f"GPU worker of {tr.name} failed to start (exit {rc})")
        self.devinfo = msg[1]
        self.worker_info = msg[3] if len(msg) > 3 else {}   # its devices and HW queues
        self.worker_info["pid"] = msg[2]
        self.jobs_sent = set()
        self._reader = threading.Thread(target=self._read_loop, args=(parent, self.proc),
                                        daemon=True, name=f"{tr.name}-gpuworker-rx")
        self._reader.start()
        log.info("%s: GPU worker pid %d (generation %d) ready", tr.name, msg[2], self.generation)
        with self._lock:
            self._up = True
            backlog, self._backlog = self._backlog, []
        for kind, runs in backlog:      # work that arrived while no worker was up
            self._dispatch(kind, runs)

    def stop(self):
        self._stopping = True
        if self.sock is not None:
            try:
                send_msg(self.sock, ("stop",), self._send_lock)
            except OSError:
                pass
        if self.proc is not None:
            # under a profiler the worker's exit handlers write its trace: wait for them
            profiled = any(k.startswith("ROCPROF") for k in os.environ)
            try:
                self.proc.wait(timeout=180 if profiled else 20)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()

    def restart(self, generation):
        """JobTracker-ordered gang restart (world > 1): kill this worker (it may
        be blocked in a collective with a dead peer) and start generation G."""
        with self._lock:
            if generation <= self.generation and self.proc is not None and \
                    self.proc.poll() is None:
                return
        self.generation = generation
        proc = self.proc
        if proc is not None and proc.poll() is None:
            self._expect_death = True
            proc.kill()
            proc.wait()
            # the reader thread sees EOF and fails the attempts; wait for it
            if self._reader is not None:
                self._reader.join(timeout=30)
        self._spawn()

    # -- tracker-facing interface ------------------------------------------------------
    def torch_device(self, d):
        return None

    def device_status(self):
        with self._lock:
            running = len(self.inflight)
        out = []
        for g in self.devinfo:
            g = dict(g)
            g["running"] = running
            out.append(P.GpuDeviceStatus(**g))
        return out

    def has_capacity(self):
        return True

    def probe(self, d):
        if self.proc is None or self.proc.poll() is not None:
            return f"GPU worker not running (last exit {self.last_exit})"
        self._probe_ev.clear()
        try:
            send_msg(self.sock, ("probe", d), self._send_lock)
        except OSError as e:
            return f"GPU worker unreachable: {e}"
        if not self._probe_ev.wait(10):
            return "GPU worker did not answer a health probe in 10 s"
        return self._probe_replies.get(d)

    def readvertise(self):
        with self._lock:
            res = [list(k) for k in self.resident]
        with self.tracker.split_cache._lock:
            self.tracker.split_cache.added.extend(res)

    def _ensure_job(self, run):
        jid = run.spec.job_id
        if jid not in self.jobs_sent:
            self.jobs_sent.add(jid)
            send_msg(self.sock, ("job", jid, run.job.conf.to_dict()), self._send_lock)

    def submit(self, run):
        self.submit_many([run])

    def submit_many(self, runs):
        if runs:
            self._dispatch("maps", runs)

    def submit_cpu(self, run):
        self._dispatch("cpu", [run])

    def submit_reduce(self, run):
        self._dispatch("reduce", [run])

    def _dispatch(self, kind, runs):
        """Send attempts to the worker, or hold them until one is up (a worker
        is being restarted).  Attempts sent to a worker that then dies are
        failed by _on_death (they are in ``inflight``)."""
        with self._lock:
            if not self._up:
                self._backlog.append((kind, runs))
                return
            for r in runs:
                self.inflight[r.spec.attempt_id] = r
        by_job: dict = {}
        for r in runs:
            by_job.setdefault(r.spec.job_id, []).append(r)
        if TRACE.on:
            TRACE.instant("remote.dispatch", kind=kind, n=len(runs))
        try:
            for jid, rs in by_job.items():
                self._ensure_job(rs[0])
                if kind == "maps":
                    s0 = rs[0].spec
                    common = (s0.is_map, s0.run_on_gpu, s0.gpu_device_id, s0.num_maps,
                              s0.num_reduces, s0.collective, s0.gate)
                    if all((r.spec.is_map, r.spec.run_on_gpu, r.spec.gpu_device_id,
                            r.spec.num_maps, r.spec.num_reduces, r.spec.collective,
                            r.spec.gate) == common
                           and not r.spec.map_outputs and not r.spec.profile_fraction
                           for r in rs):
                        # a bulk launch: shared fields once, (attempt, partition, split) each
                        send_msg(self.sock, ("maps_c", jid, common,
                                             [(r.spec.attempt_id, r.spec.partition, r.spec.split)
                                              for r in rs]), self._send_lock)
                    else:
                        send_msg(self.sock, ("maps", jid, [r.spec.to_dict() for r in rs]),
                                 self._send_lock)
                else:
                    for r in rs:
                        send_msg(self.sock, (kind, r.spec.to_dict()), self._send_lock)
        except OSError:
            pass        # the reader thread fails them when it sees the worker's death

    def kill(self, aid):
        try:
            send_msg(self.sock, ("kill", aid), self._send_lock)
        except OSError:
            pass

    def close_gate(self, jid):
        try:
            send_msg(self.sock, ("close_gate", jid), self._send_lock)
        except OSError:
            pass

    def drop_job(self, jid):
        """The job is finished or killed (KillJobAction): the worker frees its
        state (map outputs held on the device), and its attempts no longer count
        as held outputs should the worker die later."""
        with self._lock:
            self.held.pop(jid, None)
            sent = jid in self.jobs_sent
            self.jobs_sent.discard(jid)
        if sent:
            try:
                send_msg(self.sock, ("drop", jid), self._send_lock)
            except OSError:
                pass

    # -- receiving ---------------------------------------------------------------------
    def _read_loop(self, sock, proc):
        tr = self.tracker
        while True:
            try:
                msg = recv_msg(sock)
            except (OSError, EOFError, ValueError):
                msg = None
            if msg is None:
                break
            typ = msg[0]
            if typ == "batch":
                self._on_batch(msg[1], msg[2], msg[3])
            elif typ == "probe":
                self._probe_replies[msg[1]] = msg[2]
                self._probe_ev.set()
        if self._stopping or tr._stop.is_set():
            return
        self._on_death(proc)

    def _on_batch(self, items, added, removed):
        tr = self.tracker
        if added or removed:
            with self._lock:
                for k in added:
                    self.resident.add(tuple(k))
                for k in removed:
                    self.resident.discard(tuple(k))
            with tr.split_cache._lock:
                tr.split_cache.added.extend(added)
                tr.split_cache.removed.extend(removed)
        urgent = False
        bulk_jobs = set()
        for it in items:
            if it[0] == "bulk":
                _, aids, dt, output, counters = it
                with self._lock:
                    runs = [self.inflight.pop(a) for a in aids if a in self.inflight]
                    if runs:
                        self.held.setdefault(runs[0].spec.job_id, set()).update(aids)
                tr.finish_bulk(runs, dt, output, counters)
                bulk_jobs.update(r.spec.job_id for r in runs)
            else:
                urgent = True
                d = it[1]
                with self._lock:
                    run = self.inflight.pop(d["attempt_id"], None)
                    if run is not None and d["state"] == P.SUCCEEDED:
                        if run.spec.is_map and not run.spec.profile_fraction:
                            self.held.setdefault(run.spec.job_id, set()).add(d["attempt_id"])
                        elif not run.spec.is_map:
                            self.held.pop(run.spec.job_id, None)   # consumed by the reduce
                            self.jobs_sent.discard(run.spec.job_id)
                if run is None:
                    continue
                run.task = _Reported(Counters.from_dict(d.get("counters") or {}))
                out = d.get("output")
                if not run.spec.is_map and isinstance(out, dict) and "result" in out:
                    run.job.result = out["result"]
                run.status.start_time = d.get("start_time") or run.status.start_time
                tr._finish(run, d["state"], d.get("diagnostic", ""), output=d.get("output"),
                           device_time=d.get("device_time", 0.0), wake=False)
        if urgent or added or removed or not bulk_jobs:
            tr.notify_jobtracker()
        else:
            tr.maps_done_news(bulk_jobs)

    def _on_death(self, proc):
        tr = self.tracker
        rc = proc.wait()
        self.last_exit = rc
        self.deaths += 1
        expected = self._expect_death
        self._expect_death = False
        why = ("GPU worker restarted with its collective gang" if expected else
               f"GPU worker process of {tr.name} died (exit status {rc})")
        log.warning("%s", why)
        with self._lock:
            self._up = False
            runs = list(self.inflight.values())
            self.inflight.clear()
            lost = [a for s in self.held.values() for a in s]
            self.held.clear()
            gone = [list(k) for k in self.resident]
            self.resident.clear()
        with tr.split_cache._lock:
            tr.split_cache.removed.extend(gone)
        for r in runs:
            tr._finish(r, P.FAILED, why, wake=False)
        multi = tr.world_size > 1
        tr.outputs_lost(lost, worker_lost=multi and not expected)
        if expected or multi:
            return          # world > 1: the JobTracker restarts the gang
        if self.restarts >= self.max_restarts:
            log.error("%s: GPU worker died %d times; not restarting", tr.name, self.deaths)
            self._fail_backlog("GPU worker restart limit reached")
            return
        self.restarts += 1
        time.sleep(0.05)
        try:
            self._spawn()
        except Exception as e:  # noqa: BLE001
            log.exception("%s: GPU worker restart failed", tr.name)
            self._fail_backlog(f"GPU worker restart failed: {e}")

    def _fail_backlog(self, why):
        with self._lock:
            backlog, self._backlog = self._backlog, []
        for _kind, runs in backlog:
            for r in runs:
                self.tracker._finish(r, P.FAILED, why, wake=False)
        self.tracker.notify_jobtracker()
