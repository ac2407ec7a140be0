"""TaskTracker: per-process worker with CPU map slots, per-GPU map slots and reduce slots.

Redesign of hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/TaskTracker.java:
offerService/transmitHeartBeat (:1600, :1789), the fork's dual CPU/GPU
TaskLauncher (:2434-2629), status with CPU and GPU slots
(:1816-1822, G6), markUnresponsiveTasks (:2049).

MI355X-first differences:
* the worker is persistent: one process per GPU keeps the HIP context, the
  RCCL communicator and the HBM split cache across tasks and jobs (the
  reference forks a JVM and then the Pipes binary per task — the "map-task
  invocation overhead" Shirahata et al. measured, TaskRunner.java:290-299);
* a GPU slot is a HIP stream; tasks are enqueued asynchronously up to a queue
  depth and completed by HIP events, whose elapsed time is the task's device
  time reported to the cost model;
* every GPU attempt runs on the device the JobTracker chose (fixes B1);
* heartbeats long-poll the JobTracker and are cut short by ``wakeup`` as soon
  as a task finishes (no 3 s floor, B13).
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import logging
import os
import queue
import random
import re
import shutil
import socket
import sys
import threading
import time
import traceback

from ..utils.reflection import load_class, new_instance
from . import counters as C
from . import mapoutput
from . import protocol as P
from .ids import TaskAttemptID
from .jobconf import JobConf
from .child import use_child_process
from .profiling import run_profiled
from .task import MapOutputLocation, MapTask, ReduceTask, TaskReporter

from ..utils.trace import TRACE

log = logging.getLogger("hbmr.tasktracker")


class JobState:
    """Per-job state held by a tracker."""

    def __init__(self, job_id, conf: JobConf):
        self.job_id = job_id
        self.conf = conf
        self.split_job = None
        sj = conf.get("hbmr.splitjob.class")
        if sj:
            self.split_job = new_instance(sj, conf)
        self.map_outputs: dict[str, object] = {}
        self.lock = threading.Lock()
        self.result = None
        self.scratch: dict = {}
        # device map outputs as soon as their kernels are ENQUEUED (attempt ->
        # (output, end event / simulated ready time)) and map attempts that
        # failed here: what an early ("expect") collective reduce waits on
        self.launched: dict[str, tuple] = {}
        self.failed: set[str] = set()
        self.cond = threading.Condition(self.lock)

    def note_launched(self, items):
        """items: (attempt id, output, end marker) of maps just enqueued."""
        with self.cond:
            for aid, out, ev in items:
                self.launched[aid] = (out, ev)
            self.cond.notify_all()

    def note_failed(self, aid):
        with self.cond:
            self.failed.add(aid)
            self.cond.notify_all()


class TaskContext:
    """What a split-level map/reduce sees (SplitJob methods)."""

    def __init__(self, tracker, job: JobState, spec: P.TaskSpec, reporter: TaskReporter,
                 device=None, stream=None):
        self.tracker = tracker
        self.job = job
        self.conf = job.conf
        self.spec = spec
        self.attempt_id = spec.attempt_id
        self.partition = spec.partition
        self.reporter = reporter
        self.run_on_gpu = spec.run_on_gpu
        self.device_index = spec.gpu_device_id
        self.device = device
        self.stream = stream
        self.comm = tracker.comm
        self.cpu_threads = tracker.cpu_threads
        self.split_cache = tracker.split_cache

    @property
    def rank(self):
        return self.comm.rank

    @property
    def world_size(self):
        return self.comm.world_size


class _Flag:
    """Kill flag of a batched GPU attempt: nothing ever waits on it, so no
    Event (whose Condition + Lock cost more than the rest of the launch)."""
    __slots__ = ("v",)

    def __init__(self):
        self.v = False

    def set(self):
        self.v = True

    def is_set(self):
        return self.v


class _ReportGroup:
    """The per-attempt GPU maps of one bulk launch (Pipes GPU executables: a
    thread and a MapTask each) report their completions together: each
    success but the batch's last is queued without ringing the JobTracker
    and the last one's report carries them all — one report per device batch
    instead of one per map (a report costs the tracker and the JobTracker a
    few hundred µs of Python each; BASELINE config 2 runs 8 such maps per
    iteration).  A failure reports at once."""
    __slots__ = ("left", "lock")

    def __init__(self, n):
        self.left = n
        self.lock = threading.Lock()

    def done_one(self) -> bool:
        with self.lock:
            self.left -= 1
            return self.left <= 0


class _Running:
    __slots__ = ("spec", "status", "task", "kill", "job", "wait", "group")

    def __init__(self, spec, status, job, kill=None):
        self.spec = spec
        self.status = status
        self.task = None
        self.kill = threading.Event() if kill is None else kill
        self.job = job
        self.wait = None        # device event of an opened gate (staged attempts)
        self.group = None       # _ReportGroup of a bulk-launched per-attempt map


class TaskTracker:
    def __init__(self, conf, jobtracker, name=None, rank=0, world_size=1, gpu_devices=(),
                 cpu_slots=None, reduce_slots=None, gpu_slots_per_device=None, comm=None,
                 local_dir=None, host=None, worker_comm=None):
        self.conf = conf
        self.jt = jobtracker
        # The launcher, completion and heartbeat threads hand work to each
        # other; with CPython's default 5 ms GIL switch interval a woken
        # thread can wait that long for the interpreter while another one
        # runs bookkeeping, idling the GPU.  0.2 ms keeps hand-offs prompt.
        self.defer_map_reports = conf.get_boolean("hbmr.tracker.defer.map.reports", True)
        from ..utils.gctune import tune_malloc
        tune_malloc()                        # MB-sized task buffers from the heap
        # bulk-launched per-attempt GPU maps report once per batch (_ReportGroup)
        self.batch_reports = conf.get_boolean("hbmr.tracker.batch.reports", True)
        self._act_lock = threading.RLock()   # JobTracker actions, applied one at a time
        self._resp_cond = threading.Condition()
        self._next_seq = 1                   # JobTracker response order (resp["seq"])
        self._skipped: set = set()           # numbers passed over by a timed-out wait
        self._deferred: dict = {}            # job id -> launches that came before its conf
        self._early_kills: dict = {}         # attempts killed before their launch arrived
        # JobTracker.report assigns and returns actions (no long-poll wake-up)
        self.report_assign = conf.get_boolean("hbmr.tracker.report.assign", True)
        # news reaches a long-polling JobTracker as one report call
        self.report_news = conf.get_boolean("hbmr.tracker.report.news", True)
        si = conf.get_float("hbmr.python.switchinterval.ms", 0.2)
        if si > 0:
            sys.setswitchinterval(si / 1000.0)
        # slave.host.name: MiniMRCluster's per-tracker fake host (MiniMRCluster.java:151-188)
        self.host = host or conf.get("slave.host.name") or socket.gethostname()
        self.rank = rank
        self.world_size = world_size
        self.name = name or f"tracker_{self.host}_r{rank}"
        self.cpu_slots = conf.get_int("mapred.tasktracker.map.cpu.tasks.maximum", 2) \
            if cpu_slots is None else cpu_slots
        self.reduce_slots = conf.get_int("mapred.tasktracker.reduce.tasks.maximum", 2) \
            if reduce_slots is None else reduce_slots
        self.gpu_devices = list(gpu_devices)
        gs = conf.get_int("mapred.tasktracker.map.gpu.tasks.maximum", 0)
        if gpu_slots_per_device is None:
            # the reference's key counts GPU slots per node; spread them over devices
            per = max(1, gs // max(1, len(self.gpu_devices))) if gs else 1
            gpu_slots_per_device = per if self.gpu_devices else 0
        self.gpu_slots_per_device = gpu_slots_per_device
        self.cpu_threads = max(1, conf.get_int("hbmr.cpu.threads.per.slot", 1))
        self.interval = conf.get_int("hbmr.heartbeat.interval.ms", 100) / 1000.0
        self.task_timeout = conf.get_int("mapred.task.timeout", 600000) / 1000.0
        self.fault_p = conf.get_float("hbmr.faultinject.probability", 0.0)
        self._rng = random.Random(rank * 7919 + 17)
        from ..gpu.split_cache import SplitCache
        self.split_cache = SplitCache()
        from ..filecache import TrackerCacheManager
        self.cache_manager = TrackerCacheManager(
            local_dir or os.path.join(conf.get("mapred.local.dir", "/tmp/hbmr-local"),
                                      self.name))
        if comm is None:
            from ..parallel.collectives import SoloComm
            comm = SoloComm()
        self.comm = comm
        self.local_dir = local_dir or os.path.join(
            conf.get("mapred.local.dir", "/tmp/hbmr-local"), self.name)
        os.makedirs(self.local_dir, exist_ok=True)
        self.jobs: dict[str, JobState] = {}
        self._results: dict = {}             # results of purged (finished) jobs, newest last
        self.running: dict[str, _Running] = {}
        self._lock = threading.Lock()
        self._changed: set[str] = set()
        self._bulk: list[dict] = []          # batched GPU completions not yet reported
        # jobs with an early ("expect") collective reduce running here: their
        # map outputs go to that reduce on the device, so finished map batches
        # ride on the reduce's completion heartbeat instead of one of their own
        # (maps_done_news)
        self._expect_jobs: set = set()
        # jobs whose maps were launched here behind a gate (pre-staged): their
        # collective reduce is coming (the JobTracker sends it once every map
        # of the job is launched), so their finished batches wait for it too —
        # at most defer_max_s, after which they are reported on their own
        # (a reduce that does not come in time, e.g. a map re-run elsewhere)
        self._gated_jobs: set = set()
        self.defer_gated = self.defer_map_reports and conf.get_boolean(
            "hbmr.tracker.defer.gated.map.reports", True)
        self.defer_max_s = conf.get_float("hbmr.tracker.defer.map.reports.max.ms", 25.0) / 1e3
        self._defer_timer = None
        self._polling = False       # the heartbeat thread is in a long-poll
        self._requeued: list = []   # drained statuses whose report failed
        self._notify_seq = 0                 # wakeup() notifications sent (notify_seq)
        # one report in flight at a time: a task finishing meanwhile leaves its
        # news to that reporter's next round (coalesced, not one call each)
        self._reporting = False
        self._report_again = False
        self._lost: list[str] = []           # succeeded attempts whose output was lost
        self._worker_lost = False            # GPU worker died: the gang must restart
        self._news = threading.Event()
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        # CPU map slots run below the control plane's scheduling priority: a
        # compute-bound CPU map must not delay heartbeats and GPU launches
        # (threads it starts inherit the nice value)
        nice = conf.get_int("hbmr.cpu.slot.nice", 10)
        self.cpu_pool = cf.ThreadPoolExecutor(max(1, self.cpu_slots),
                                              thread_name_prefix=f"{self.name}-cpu",
                                              initializer=_lower_priority, initargs=(nice,))
        self.reduce_pool = cf.ThreadPoolExecutor(max(1, self.reduce_slots),
                                                 thread_name_prefix=f"{self.name}-red")
        # GPU Pipes maps: the scheduler queues up to slots x queue depth per
        # device; ``hbmr.gpu.pipes.concurrency`` of them run at once per slot,
        # each in its own reused child, so one map's task setup and socket
        # round trip overlap another's device work (a lone child serialises
        # them: about 1.5 ms per map against ~50 us of GPU time)
        conc = max(1, conf.get_int("hbmr.gpu.pipes.concurrency", 2))
        if conf.get_boolean("hbmr.pipes.gpu.mux", True):
            # one shared child per device takes up to its queue depth of maps
            # (hbmr/pipes/mux.py): a thread per map in flight
            conc = max(conc, conf.get_int("hbmr.pipes.gpu.queue.depth", 8))
        self.gpu_pipes_pool = cf.ThreadPoolExecutor(
            max(1, len(self.gpu_devices) * max(1, self.gpu_slots_per_device) * conc),
            thread_name_prefix=f"{self.name}-gpupipes")
        self.gpu_runtime = None
        self.worker_comm = worker_comm
        if self.gpu_devices:
            if conf.get_boolean("hbmr.gpu.worker.process", False):
                # device work in a persistent child process per tracker: a GPU
                # fault fails attempts, not the tracker (hbmr/gpu/remote.py)
                from ..gpu.remote import RemoteGpuRuntime as _Rt
            elif conf.get_boolean("hbmr.gpu.simulate", False):
                from ..gpu.simulated import SimulatedGpuRuntime as _Rt
            else:
                from ..gpu.runtime import GpuRuntime as _Rt
            self.gpu_runtime = _Rt(self, self.gpu_devices, self.gpu_slots_per_device)
        from .health import NodeHealthChecker
        self.health = NodeHealthChecker(conf, self.gpu_runtime)
        self.child_manager = None     # JvmManager analogue, created on first use
        self.heartbeats = 0
        self.tasks_done = 0
        self._reinit = False

    # -- status -----------------------------------------------------------------------
    def status(self) -> P.TaskTrackerStatus:
        gpus = []
        if self.gpu_runtime is not None:
            gpus = self.health.filter_gpus(
                [g.__dict__ for g in self.gpu_runtime.device_status()])
        healthy, report = self.health.health_report()
        added, removed = self.split_cache.drain_changes()
        with self._lock:
            ids = list(self._changed)
            self._changed.clear()
            reports = []
            bulk, lost, wlost = [], [], False
            for old in self._requeued:
                reports += old.task_reports
                bulk += old.bulk_reports
                lost += old.lost_outputs
                wlost = wlost or old.gpu_worker_lost
                added = list(old.cached_splits_added) + list(added)
                removed = list(old.cached_splits_removed) + list(removed)
            self._requeued = []
            for aid in ids:
                r = self.running.get(aid)
                if r is not None:
                    reports.append(r.status.to_dict())
                    if r.status.state in P.TERMINAL:
                        self.running.pop(aid, None)
            bulk += self._bulk
            self._bulk = []
            lost += self._lost
            self._lost = []
            wlost = wlost or self._worker_lost
            self._worker_lost = False
            seq = self._notify_seq
        return P.TaskTrackerStatus(tracker_name=self.name, host=self.host, bulk_reports=bulk,
                                   notify_seq=seq,
                                   lost_outputs=lost, gpu_worker_lost=wlost,
                                   max_cpu_map_slots=self.cpu_slots,
                                   max_reduce_slots=self.reduce_slots, gpus=gpus,
                                   task_reports=reports, cached_splits_added=added,
                                   cached_splits_removed=removed, rank=self.rank,
                                   world_size=self.world_size, cpu_threads=self.cpu_threads,
                                   healthy=healthy, health_report=report)

    def _has_capacity(self):
        with self._lock:
            n_cpu = sum(1 for r in self.running.values() if r.spec.is_map and not r.spec.run_on_gpu
                        and r.status.state not in P.TERMINAL)
        if n_cpu < self.cpu_slots:
            return True
        if self.gpu_runtime is not None and self.gpu_runtime.has_capacity():
            return True
        return True  # reduces may still be assignable

    def _mark(self, aid):
        with self._lock:
            self._changed.add(aid)
        self._news.set()

    def _run_debug_script(self, run: _Running, diag: str) -> str:
        """Failed attempt + ``mapred.{map,reduce}.task.debug.script``: run the script
        as ``script stdout stderr syslog jobconf [program]`` in the attempt's log dir,
        keep its output as userlogs/<attempt>/debugout and return it for the
        diagnostics (TaskTracker.TaskInProgress.runDebugScript in the reference;
        Pipes jobs default to the gdb-style ``pipes-default-script`` when
        ``hadoop.pipes.executable`` is set and ``mapred.*.task.debug.script`` is)."""
        import shlex
        import subprocess
        js = run.job
        if js is None or run.spec is None:
            return ""
        aid = run.spec.attempt_id
        is_map = "_m_" in aid
        script = js.conf.get("mapred.map.task.debug.script" if is_map
                             else "mapred.reduce.task.debug.script")
        if not script:
            return ""
        logd = os.path.join(self.local_dir, "userlogs", aid)
        os.makedirs(logd, exist_ok=True)
        files = [os.path.join(logd, n) for n in ("stdout", "stderr", "syslog")]
        for f in files:
            if not os.path.exists(f):
                with open(f, "w") as fh:
                    fh.write(diag if f.endswith("stderr") else "")
        confp = os.path.join(logd, "job.xml")
        with open(confp, "w") as fh:
            js.conf.write_xml(fh)
        args = shlex.split(script) + files + [confp]
        # the program the attempt ran (GPU attempts: the GPU binary)
        on_gpu = bool(getattr(run.spec, "run_on_gpu", False))
        prog = (js.conf.get("hadoop.pipes.gpu.executable") if on_gpu else None) or \
            js.conf.get("hadoop.pipes.executable") or js.conf.get("hadoop.pipes.gpu.executable")
        if prog:
            args.append(prog)
        # where a Pipes child of this attempt ran (and would have dumped core)
        import glob
        env = dict(os.environ)
        import tempfile
        base = js.conf.get("hbmr.local.scratch") or tempfile.gettempdir()
        dirs = [d for d in glob.glob(os.path.join(base, f"_pipes_{aid}_*")) if os.path.isdir(d)]
        env["HBMR_DEBUG_DIRS"] = ":".join(dirs)
        try:
            r = subprocess.run(args, cwd=logd, capture_output=True, text=True, env=env,
                               timeout=js.conf.get_int("hbmr.task.debug.script.timeout.s", 60))
            out = r.stdout + r.stderr
        except (OSError, subprocess.TimeoutExpired) as e:
            out = f"debug script failed: {e}"
        with open(os.path.join(logd, "debugout"), "w") as fh:
            fh.write(out)
        return out

    def _finish(self, run: _Running, state, diag="", output=None, device_time=0.0, wake=True):
        if state != P.SUCCEEDED and run.spec is not None and run.spec.is_map and \
                run.job is not None:
            run.job.note_failed(run.spec.attempt_id)
        if run.spec is not None and not run.spec.is_map and (self._expect_jobs or
                                                             self._gated_jobs):
            with self._lock:
                self._expect_jobs.discard(run.spec.job_id)
                self._gated_jobs.discard(run.spec.job_id)
        if state == P.FAILED:
            dbg = self._run_debug_script(run, diag)
            if dbg:
                diag = f"{diag}\nDebug script output:\n{dbg[-4096:]}"
        st = run.status
        if TRACE.on:
            TRACE.instant("tt.finish", attempt=st.attempt_id, state=state,
                          where=(output or {}).get("where") if isinstance(output, dict) else None)
        st.state = state
        st.finish_time = time.time()
        st.diagnostic = diag
        if run.task is not None:
            st.counters = run.task.reporter.counters.to_dict()
        if output is not None:
            st.output = output
        st.device_time = device_time
        st.progress = 1.0 if state == P.SUCCEEDED else st.progress
        self.tasks_done += 1
        self._mark(st.attempt_id)
        if wake:
            self.notify_jobtracker()

    def finish_bulk(self, runs, device_time, output, counters=None):
        """A batch of GPU map attempts completed together: one compact report
        (JobTracker._bulk_succeeded) instead of one status per attempt.
        ``counters`` is the batch's merged counters dict (else each run's
        reporter counters are merged here)."""
        if not runs:
            return
        now = time.time()
        if counters is None:
            agg = C.Counters()
            for r in runs:
                if r.task is not None:
                    agg.incr_all(r.task.reporter.counters)
            counters = agg.to_dict()
        aids = []
        with self._lock:
            for r in runs:
                st = r.status
                st.state = P.SUCCEEDED
                st.finish_time = now
                st.progress = 1.0
                st.device_time = device_time
                st.output = output
                aids.append(st.attempt_id)
                self.running.pop(st.attempt_id, None)
            self._bulk.append({"attempts": aids, "device_time": device_time, "finish_time": now,
                               "counters": counters, "output": output})
        self.tasks_done += len(runs)
        if TRACE.on:
            TRACE.instant("tt.finish", n=len(runs), state=P.SUCCEEDED,
                          where=(output or {}).get("where"))
        self._news.set()

    def maps_done_news(self, job_ids):
        """Finished GPU map batches of ``job_ids`` are queued for the next
        heartbeat: wake the JobTracker now unless each of those jobs has an
        early collective reduce running here — its completion (a few device
        kernels later) reports them together, one heartbeat instead of two
        (the JobTracker's per-heartbeat work bounds multi-rank scaling).
        ``hbmr.tracker.defer.map.reports`` = false always reports at once."""
        if self._expect_jobs and all(j in self._expect_jobs for j in job_ids):
            self._news.set()
            return
        if self._gated_jobs and all(j in self._gated_jobs or j in self._expect_jobs
                                    for j in job_ids):
            # the job's reduce launch is on its way (it rides on this tracker's
            # next response): report these with the reduce, not on their own
            self._news.set()
            self._arm_defer_flush()
            return
        self.notify_jobtracker()

    def _arm_defer_flush(self):
        """Liveness bound of deferred map reports: unreported batches go out
        after defer_max_s even if no reduce completion carried them."""
        with self._lock:
            if self._defer_timer is not None:
                return
            t = self._defer_timer = threading.Timer(self.defer_max_s, self._defer_flush)
        t.daemon = True
        t.start()

    def _defer_flush(self):
        with self._lock:
            self._defer_timer = None
            # (deferred batch reports, or per-attempt statuses of a report
            # group waiting for its last map)
            pending = bool(self._bulk) or bool(self._changed)
        if pending:
            self.notify_jobtracker()

    def outputs_lost(self, aids, worker_lost=False):
        with self._lock:
            self._lost.extend(aids)
            self._worker_lost = self._worker_lost or worker_lost
        self.notify_jobtracker()

    def notify_jobtracker(self):
        """Finished tasks are reported now.  While the heartbeat long-polls,
        the news goes to the JobTracker directly (JobTracker.report: processed
        there, and the long-poll is rung to assign into the freed slots);
        otherwise the heartbeat thread is between calls and takes it along on
        its next one.  The fallback cuts the long-poll short (wakeup); the
        notification count lets the JobTracker tell a wakeup that carries news
        the pending heartbeat lacks from a stale one (TaskTrackerStatus.notify_seq)."""
        with self._lock:
            self._notify_seq += 1
            seq = self._notify_seq
            polling = self._polling
            if polling and self.report_news and self._reporting:
                # a report is in flight: it goes again with this news
                self._report_again = True
                self._news.set()
                return
            if polling and self.report_news:
                self._reporting = True
        self._news.set()
        if not polling:
            return
        if self.report_news and getattr(self.jt, "report", None) is not None:
            done = False
            try:
                while True:
                    if not self._report_once(seq):
                        return
                    with self._lock:
                        if not self._report_again:
                            # the reporter stands down under the lock that saw no
                            # more news: a notification after this reports itself
                            # (clearing the flag in `finally`, after
                            # the lock was dropped, lost one arriving in between)
                            self._reporting = False
                            done = True
                            return
                        self._report_again = False
                        seq = self._notify_seq
            finally:
                if not done:
                    with self._lock:
                        # (news left by a failed round went to the heartbeat: _news)
                        self._reporting = self._report_again = False
        elif self.report_news:
            with self._lock:
                self._reporting = False
        try:
            self.jt.wakeup(self.name, seq)
        except Exception:  # noqa: BLE001
            pass

    def _report_once(self, seq) -> bool:
        """One report of the drained news; True if it was delivered."""
        st = self.status()
        try:
            r = self.jt.report(st.to_dict(), self.report_assign) if self.report_assign \
                else self.jt.report(st.to_dict())
            if not (isinstance(r, dict) and r.get("reinit")):
                # (assign form) the response carries this tracker's new work:
                # handled here, the long-poll stays parked
                self._apply(r or {})
                return True
        except Exception:  # noqa: BLE001
            # the JobTracker may have processed it: take back its reply
            self._recover_lost_reply()
        self._requeue(st)      # not delivered: the heartbeat thread sends it
        try:
            self.jt.wakeup(self.name, seq)
        except Exception:  # noqa: BLE001
            pass
        return False

    def _requeue(self, st):
        """A drained status whose report did not reach the JobTracker: its
        contents go out with the next heartbeat."""
        with self._lock:
            self._requeued.append(st)
            self._news.set()

    # -- lifecycle -----------------------------------------------------------------------
    def start(self):
        if self.gpu_runtime is not None:
            self.gpu_runtime.start()  # a GPU worker process must be up before the probe
        if self.health.enabled:
            self.health.check_now()   # before the first heartbeat advertises slots
        t = threading.Thread(target=self._hb_loop, name=f"{self.name}-hb", daemon=True)
        t.start()
        self._threads.append(t)
        return self

    def stop(self):
        self._stop.set()
        self._news.set()
        if self.gpu_runtime is not None:
            self.gpu_runtime.stop()
        for t in self._threads:
            t.join(timeout=5)
        self.cpu_pool.shutdown(wait=False, cancel_futures=True)
        self.reduce_pool.shutdown(wait=False, cancel_futures=True)
        if self.child_manager is not None:
            self.child_manager.shutdown()
        pipes_app = sys.modules.get("hbmr.pipes.application")
        if pipes_app is not None:
            pipes_app.POOL.close_all()      # reused Pipes children (hbmr.pipes.child.reuse)

    def _hb_loop(self):
        initial = True
        more = False
        while not self._stop.is_set():
            try:
                self._news.clear()
                # (set before the status is built: news from here on is
                # either in it or reported to the JobTracker by the notifier)
                with self._lock:
                    self._polling = not (initial or more)
                st = self.status()
                block = 0.0 if (st.task_reports or initial or more) else self.interval
                if block == 0.0:
                    with self._lock:
                        self._polling = False
                if TRACE.on:
                    TRACE.instant("tt.heartbeat.send", reports=len(st.task_reports), block=block)
                initial_sent = initial
                try:
                    resp = self.jt.heartbeat(st.to_dict(), initial=initial,
                                             accept_new_tasks=True, block=block)
                finally:
                    with self._lock:
                        self._polling = False
                if TRACE.on:
                    TRACE.instant("tt.heartbeat.recv", actions=len(resp.get("actions", [])))
                self.heartbeats += 1
                initial = False
                more = bool(resp.get("more"))
                if initial_sent:
                    with self._resp_cond:
                        self._next_seq = 1       # a (re-)registered tracker: new numbering
                        self._skipped.clear()
                        self._resp_cond.notify_all()
                self._apply(resp)
                if self._reinit:
                    self._reinit = False
                    initial = True
                    continue
                if not resp.get("actions") and not st.task_reports and block == 0.0 and not more:
                    self._news.wait(self.interval)
                self._check_timeouts()
                self.health.maybe_check()
            except Exception as e:  # noqa: BLE001
                if self._stop.is_set():
                    break
                log.warning("heartbeat to JobTracker failed: %s", e)
                self._stop.wait(min(1.0, self.interval * 5))

    def _check_timeouts(self):
        """markUnresponsiveTasks: fail attempts without progress for mapred.task.timeout.
        At most every 0.1 s: the heartbeat loop turns over once per completion
        notification, and a scan of every running attempt each time showed up
        in control-plane profiles (timeouts are whole seconds or more)."""
        now = time.time()
        if now - getattr(self, "_last_timeout_scan", 0.0) < 0.1:
            return
        self._last_timeout_scan = now
        with self._lock:
            runs = list(self.running.values())
        for r in runs:
            if r.status.state != P.RUNNING or r.task is None:
                continue
            # the job's mapred.task.timeout (TaskTracker.java:2834), else the tracker's
            limit = r.job.conf.get_int("mapred.task.timeout", -1) / 1000.0 \
                if r.job.conf.get("mapred.task.timeout") is not None else self.task_timeout
            if limit > 0 and now - r.task.reporter.last_progress > limit:
                r.kill.set()
                self._finish(r, P.FAILED, f"Task {r.spec.attempt_id} failed to report status "
                                          f"for {limit:g} seconds. Killing!")

    # -- actions -------------------------------------------------------------------------
    def _apply(self, resp):
        """Apply a JobTracker response's actions in the JobTracker's order: a
        response numbered ``seq`` waits (up to 2 s) until every earlier one has
        been applied by whichever thread received it — a report's response and
        the long-poll's can come back in either order."""
        acts = resp.get("actions") or ()
        seq = resp.get("seq")
        if seq is None:
            for act in acts:
                self._handle(act)
            return
        with self._resp_cond:
            deadline = time.time() + 2.0
            while seq > self._next_seq and time.time() < deadline:
                self._resp_cond.wait(deadline - time.time())
            if seq < self._next_seq and seq not in self._skipped:
                return                       # applied already (a resent response)
            try:
                for act in acts:
                    self._handle(act)
            finally:
                if seq in self._skipped:
                    self._skipped.discard(seq)           # a late one a wait gave up on
                else:
                    # (seq > _next_seq: the 2 s wait timed out; the numbers
                    # passed over may still arrive and are applied then)
                    self._skipped.update(range(self._next_seq, seq))
                    self._next_seq = seq + 1
                while len(self._skipped) > 256:
                    self._skipped.discard(min(self._skipped))
                self._resp_cond.notify_all()

    def _recover_lost_reply(self):
        """A report whose reply was lost after the JobTracker processed it: take
        back the numbered responses after the last one applied here (their
        launches / approvals / kills would otherwise be lost, and a later
        response would wait 2 s for the missing number)."""
        fn = getattr(self.jt, "resend", None)
        if fn is None:
            return
        with self._resp_cond:
            after = self._next_seq - 1
        try:
            r = fn(self.name, after)
        except Exception:  # noqa: BLE001
            return
        for q, acts in (r or {}).get("responses", ()):
            self._apply({"seq": q, "actions": acts})

    def _handle(self, act):
        """Apply one JobTracker action.  Actions arrive from the heartbeat
        thread and (JobTracker.report with assign) from the thread that
        reported finished tasks, so two responses may be applied out of the
        order the JobTracker built them in: the first launch of a job on this
        tracker carries the job's configuration, and a launch of a job not yet
        known here without it is held until that one arrives."""
        with self._act_lock:
            self._handle_locked(act)

    def _handle_locked(self, act):
        typ = act["type"]
        if typ in ("launch_batch", "launch"):
            jid = act["job_id"] if typ == "launch_batch" else act["task"]["job_id"]
            conf = act.get("conf") if typ == "launch_batch" else act["task"].get("conf")
            if jid not in self.jobs and not conf:
                self._deferred.setdefault(jid, []).append(act)
                return
            if typ == "launch_batch":
                self._launch_batch(act)
            else:
                self._launch(P.TaskSpec.from_dict(act["task"]))
            for later in self._deferred.pop(jid, ()):
                self._handle_locked(later)
        elif typ == "kill_job" and act["job_id"] in self._deferred:
            self._deferred.pop(act["job_id"], None)
            self._handle_kill_job(act)
        elif typ == "kill_task":
            with self._lock:
                r = self.running.get(act["attempt_id"])
                if r is None:
                    # not launched here yet (its launch may still be held):
                    # the launch is dropped when it comes
                    self._early_kills[act["attempt_id"]] = None
                    while len(self._early_kills) > 4096:
                        self._early_kills.pop(next(iter(self._early_kills)))
            if r is not None:
                r.kill.set()
                if r.task is not None and getattr(r.task, "kill_event", None) is not None:
                    r.task.kill_event.set()
                if getattr(self.gpu_runtime, "remote", False):
                    self.gpu_runtime.kill(act["attempt_id"])
        elif typ == "close_gate":
            if self.gpu_runtime is not None and hasattr(self.gpu_runtime, "close_gate"):
                self.gpu_runtime.close_gate(act["job_id"])
        elif typ == "restart_gpu_worker":
            if getattr(self.gpu_runtime, "remote", False):
                self.gpu_runtime.restart(act["generation"])
        elif typ == "commit":
            with self._lock:
                r = self.running.get(act["attempt_id"])
            if r is not None:
                r.status.commit_granted = True  # picked up by the waiting task
        elif typ == "kill_job":
            self._handle_kill_job(act)
        elif typ == "reinit":
            # the JobTracker does not know us (it restarted, or expired us):
            # drop every attempt and job, re-advertise the HBM-resident splits
            # and register again (TaskTracker.java:1705 ReinitTrackerAction)
            log.warning("%s asked to reinitialise", self.name)
            with self._lock:
                runs = list(self.running.values())
                self.running.clear()
                self._changed.clear()
            for r in runs:
                r.kill.set()
                if r.task is not None and getattr(r.task, "kill_event", None) is not None:
                    r.task.kill_event.set()
            self.jobs.clear()
            self.split_cache.readvertise()
            if getattr(self.gpu_runtime, "remote", False):
                self.gpu_runtime.readvertise()
            self._reinit = True
        elif typ == "shutdown":
            self._stop.set()

    #: every tracker that can run a reduce of this tracker's maps lives in this
    #: process (set by LocalCluster, and by a one-rank node): only then may map
    #: outputs stay in memory (hbmr/mapred/mapoutput.py).  A tracker of a
    #: multi-rank node has reduces in other processes reading its files, even
    #: when its JobTracker is in-process (rank 0 below 8 ranks).
    all_trackers_local = False

    def _memory_outputs(self) -> bool:
        return self.all_trackers_local

    def _handle_kill_job(self, act):
        """KillJobAction: the job is finished or killed; purge its state here
        and in the GPU worker (held device map outputs, worker JobState), its
        in-memory map outputs and (purgeJob / removeJobFiles) its local dir."""
        jid = act["job_id"]
        jdir = os.path.join(self.local_dir, jid)
        mapoutput.STORE.drop_prefix(jdir + os.sep)
        js = self.jobs.pop(jid, None)
        if js is not None and os.path.isdir(jdir) and \
                not js.conf.get_boolean("keep.failed.task.files", False) and \
                not js.conf.get("keep.task.files.pattern"):
            threading.Thread(target=shutil.rmtree, args=(jdir, True), daemon=True,
                             name=f"{self.name}-purge").start()
        with self._lock:
            self._gated_jobs.discard(jid)
            self._expect_jobs.discard(jid)
        if js is not None and js.result is not None:
            self._results[jid] = js.result
            while len(self._results) > 64:
                self._results.pop(next(iter(self._results)))
        if getattr(self.gpu_runtime, "remote", False):
            self.gpu_runtime.drop_job(jid)
        if self.child_manager is not None:
            self.child_manager.job_done(jid)

    def _job(self, spec: P.TaskSpec) -> JobState:
        js = self.jobs.get(spec.job_id)
        if js is None:
            conf = JobConf()
            if spec.conf:
                for k, v in spec.conf.items():
                    conf.set(k, v)
            # DistributedCache: localize the job's side files once per tracker
            self.cache_manager.localize(spec.job_id, conf)
            js = JobState(spec.job_id, conf)
            self.jobs[spec.job_id] = js
        return js

    def _launch(self, spec: P.TaskSpec):
        if self._early_kills.pop(spec.attempt_id, 0) is None:
            return          # killed before it got here (the JobTracker already knows)
        js = self._job(spec)
        st = P.TaskStatus(attempt_id=spec.attempt_id, is_map=spec.is_map, state=P.RUNNING,
                          run_on_gpu=spec.run_on_gpu, gpu_device_id=spec.gpu_device_id,
                          start_time=time.time())
        run = _Running(spec, st, js)
        with self._lock:
            self.running[spec.attempt_id] = run
            if not spec.is_map and spec.expect and self.defer_map_reports:
                self._expect_jobs.add(spec.job_id)
        remote = getattr(self.gpu_runtime, "remote", False) and js.split_job is not None
        if spec.is_map and spec.run_on_gpu:
            if js.split_job is None:
                # classic job with a GPU Pipes executable: a child process per
                # attempt, told its device (the fork's model, B1 fixed)
                self.gpu_pipes_pool.submit(self._run_cpu_map, run)
            else:
                self.gpu_runtime.submit(run)
        elif remote:
            # split-job CPU maps and reduces run where the job's map outputs
            # live: in the GPU worker process
            if spec.is_map:
                self.gpu_runtime.submit_cpu(run)
            else:
                self.gpu_runtime.submit_reduce(run)
        elif spec.is_map:
            self.cpu_pool.submit(self._run_cpu_map, run)
        elif spec.collective and js.split_job is not None:
            # a collective reduce gets a thread of its own: it may wait for maps
            # held behind an earlier job's reduce (pre-staging), which a bounded
            # pool could starve; one per job and tracker (pinned gang member)
            threading.Thread(target=self._run_reduce, args=(run,), daemon=True,
                             name=f"{self.name}-coll-{spec.attempt_id[-12:]}").start()
        else:
            self.reduce_pool.submit(self._run_reduce, run)

    def _launch_batch(self, act):
        """Bulk LaunchTaskAction (JobTracker.launch_gpu_batch): GPU maps of one
        split job on one device, handed to the device runtime as they are built."""
        jid = act["job_id"]
        js = self.jobs.get(jid)
        if js is None:
            js = self._job(P.TaskSpec(attempt_id="", job_id=jid, is_map=True, partition=0,
                                      conf=act.get("conf")))
        dev = act["device"]
        nm, nr, coll = act["num_maps"], act["num_reduces"], act["collective"]
        now = time.time()
        tasks = act["tasks"]
        split_job = js.split_job is not None and self.gpu_runtime is not None
        submit_many = getattr(self.gpu_runtime, "submit_many", None) if split_job else None
        # an idle device starts on the first few tasks while the rest are built
        # (per-task bookkeeping is a few µs here and again in the GPU worker)
        first = self.conf.get_int("hbmr.gpu.first.chunk", 4) if submit_many else len(tasks)
        for lo, hi in ((0, min(first, len(tasks))), (min(first, len(tasks)), len(tasks))):
            if lo >= hi:
                continue
            runs = []
            gate = act.get("gate")
            if gate is not None and coll and self.defer_gated and \
                    jid not in self._gated_jobs:
                with self._lock:
                    self._gated_jobs.add(jid)
            for aid, part, split in tasks[lo:hi]:
                if self._early_kills.pop(aid, 0) is None:
                    continue    # killed before its launch arrived
                spec = P.TaskSpec(aid, jid, True, part, True, dev, split, nm, nr, (), coll,
                                  gate=gate)
                st = P.TaskStatus(aid, True, P.RUNNING, 0.0, True, dev, now)
                runs.append(_Running(spec, st, js, _Flag()))
            with self._lock:
                for r in runs:
                    self.running[r.spec.attempt_id] = r
            if not split_job:
                # not a split job: the per-attempt GPU Pipes path, one report
                # per batch (hbmr.tracker.batch.reports)
                grp = _ReportGroup(len(runs)) if len(runs) > 1 and self.batch_reports \
                    else None
                self._prelaunch_pipes(js, runs)
                for r in runs:
                    r.group = grp
                    self.gpu_pipes_pool.submit(self._run_cpu_map, r)
                continue
            if TRACE.on:
                TRACE.instant("tt.launch_batch", n=len(runs))
            if submit_many is not None:
                submit_many(runs)
            else:
                for r in runs:
                    self.gpu_runtime.submit(r)

    def _prelaunch_pipes(self, js, runs):
        """A bulk launch of GPU Pipes maps whose child reads its own input
        through the device's shared child (hbmr/pipes/mux.py): send their
        RUN_MAPs now, from here, so the child runs them back to back while
        the task threads set up (``hbmr.pipes.gpu.prelaunch``, default on).
        Each thread's PipesGPUMapRunner then takes over its map's messages
        (mux.PRELAUNCHED); a map that could not be sent ahead (full FIFO, no
        child) goes the ordinary way."""
        conf = js.conf
        # (only for apps that take one conf per job: an attempt's own task
        # conf — work dir, input file, ... — is built by its task thread)
        if len(runs) < 2 or not conf.get_gpu_executable() or \
                not conf.get_boolean("hbmr.pipes.gpu.prelaunch", True) or \
                not conf.get_boolean("hbmr.pipes.gpu.mux", True) or \
                not conf.get_boolean("hbmr.pipes.gpu.mux.shared.conf", False) or \
                conf.get_boolean("hadoop.pipes.java.recordreader", False):
            return
        from ..pipes import mux
        from ..pipes.runner import PipesGPUMapRunner, _work_dir
        if conf.get_gpu_map_runner_class() is not PipesGPUMapRunner:
            return
        exe, depth = conf.get_gpu_executable(), conf.get_int(mux.DEPTH, 8)
        nred = conf.get_num_reduce_tasks()
        for r in runs:
            spec = r.spec
            if r.kill.is_set():
                continue
            try:
                tconf = type(conf)(conf)
                tconf.set("mapred.task.id", spec.attempt_id)
                dev = spec.gpu_device_id
                child = mux.REGISTRY.get(tconf, exe, dev,
                                         lambda c=tconf, d=dev: _work_dir(c, f"gpumux{d}"), depth)
                split = _split_from_dict(spec.split)
                sb = split.serialize() if hasattr(split, "serialize") else bytes(split or b"")
                t = child.prelaunch(tconf, sb, nred)
            except Exception:  # noqa: BLE001 — the task thread reports it its own way
                return
            if t is None:
                return
            mux.PRELAUNCHED[spec.attempt_id] = (child, t)

    def _maybe_inject_fault(self, run):
        if self.fault_p > 0 and self._rng.random() < self.fault_p:
            raise RuntimeError(f"injected fault (hbmr.faultinject.probability={self.fault_p})")

    # -- CPU maps --------------------------------------------------------------------------
    def _run_cpu_map(self, run: _Running):
        spec, js = run.spec, run.job
        run.status.start_time = time.time()
        if TRACE.on:
            TRACE.instant("tt.map.start", attempt=spec.attempt_id)
        try:
            if run.kill.is_set():
                pm = sys.modules.get("hbmr.pipes.mux")
                if pm is not None:
                    pm.PRELAUNCHED.pop(spec.attempt_id, None)
                self._group_wake(run, False)
                self._finish(run, P.KILLED, "killed before start")
                return
            self._maybe_inject_fault(run)
            if js.split_job is not None:
                from ..gpu.splitexec import run_split_cpu_map
                run_split_cpu_map(self, run)
                return
            if use_child_process(js.conf):
                path = self._run_in_child(run, is_map=True)
                self._keep_task_files(spec, js, failed=False)
                self._finish(run, P.SUCCEEDED, output={"tracker": self.name, "path": path},
                             wake=self._group_wake(run, True))
                return
            split = _split_from_dict(spec.split)
            aid = TaskAttemptID.for_name(spec.attempt_id)
            task = MapTask(js.conf, aid, spec.partition, split)
            task.memory_outputs = self._memory_outputs()
            task.setRunOnGPU(spec.run_on_gpu)
            task.setGPUDeviceId(spec.gpu_device_id)
            task.kill_event = run.kill
            run.task = task
            path = run_profiled(js.conf, spec.attempt_id, True, spec.partition, task.run,
                                os.path.join(self.local_dir, spec.job_id, spec.attempt_id))
            self._keep_task_files(spec, js, failed=False)
            self._finish(run, P.SUCCEEDED, output={"tracker": self.name, "path": path},
                         wake=self._group_wake(run, True))
        except BaseException as e:  # noqa: BLE001
            state = P.KILLED if run.kill.is_set() else P.FAILED
            if state == P.FAILED:
                self._keep_task_files(spec, js, failed=True)
            pm = sys.modules.get("hbmr.pipes.mux")
            if pm is not None:
                pm.PRELAUNCHED.pop(spec.attempt_id, None)   # (never taken over)
            self._group_wake(run, False)
            self._finish(run, state, f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")

    def _group_wake(self, run: _Running, ok: bool) -> bool:
        """Does this attempt's completion ring the JobTracker now?  Always for
        a failure or an attempt of no report group; a success of a group only
        as the group's last (the others ride on its report; the defer timer
        bounds how long they wait if the last one is slow)."""
        g = run.group
        if g is None:
            return True
        last = g.done_one()
        if ok and not last:
            self._news.set()
            self._arm_defer_flush()
            return False
        return True

    def _keep_task_files(self, spec, js, failed):
        """Keep a map attempt's task conf and split for IsolationRunner
        (TaskTracker.java keepFailedTaskFiles / keepTaskFiles pattern):
        ``<local>/<job>/<attempt>/job.xml`` and ``split.dta``."""
        conf = js.conf
        pat = conf.get("keep.task.files.pattern")
        keep = (failed and conf.get_boolean("keep.failed.task.files", False)) or \
            (pat is not None and re.fullmatch(pat, spec.attempt_id) is not None)
        if not keep or spec.split is None:
            return
        try:
            d = os.path.join(self.local_dir, spec.job_id, spec.attempt_id)
            os.makedirs(d, exist_ok=True)
            tc = JobConf(conf)
            tc.set("mapred.task.id", spec.attempt_id)
            tc.set_int("mapred.task.partition", spec.partition)
            tc.set_boolean("mapred.task.is.map", True)
            tc.set("mapred.local.dir", self.local_dir)
            tc.write_xml(os.path.join(d, "job.xml"))
            with open(os.path.join(d, "split.dta"), "w") as f:
                json.dump(spec.split, f)
        except OSError as e:
            log.warning("could not keep task files of %s: %s", spec.attempt_id, e)

    # -- reduces ---------------------------------------------------------------------------
    def _run_reduce(self, run: _Running):
        spec, js = run.spec, run.job
        run.status.start_time = time.time()
        if TRACE.on:
            TRACE.instant("tt.reduce.start", attempt=spec.attempt_id)
        try:
            self._maybe_inject_fault(run) if not spec.collective else None
            if js.split_job is not None:
                from ..gpu.splitexec import run_split_reduce
                dev = None if self.gpu_runtime is None else \
                    self.gpu_runtime.torch_device(self.gpu_devices[0])
                run_split_reduce(self, run, dev)
                return
            if use_child_process(js.conf):
                self._run_in_child(run, is_map=False)
                self._finish(run, P.SUCCEEDED, output={"tracker": self.name})
                return
            aid = TaskAttemptID.for_name(spec.attempt_id)
            task = ReduceTask(js.conf, aid, spec.partition, spec.num_maps)
            task.kill_event = run.kill
            run.task = task
            for _tid, map_aid, out in spec.map_outputs:
                task.add_map_output(MapOutputLocation(map_aid, out["path"]))
            if len(spec.map_outputs) < spec.num_maps:
                # slow-start: the rest of the map outputs arrive as completion events
                jt, jid = self.jt, spec.job_id
                task.event_source = lambda start: jt.map_completion_events(jid, start, 0.05)
            run_profiled(js.conf, spec.attempt_id, False, spec.partition, task.run,
                         os.path.join(self.local_dir, spec.job_id, spec.attempt_id))
            self._finish(run, P.SUCCEEDED, output={"tracker": self.name})
        except BaseException as e:  # noqa: BLE001
            state = P.KILLED if run.kill.is_set() else P.FAILED
            self._finish(run, state, f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}")

    # -- child processes (TaskRunner / JvmManager) --------------------------------------------
    def _children(self):
        with self._lock:
            if self.child_manager is None:
                from .child import ChildManager
                self.child_manager = ChildManager(self.name, self.local_dir, self.conf)
            return self.child_manager

    def _run_in_child(self, run: _Running, is_map: bool):
        spec, js = run.spec, run.job
        rep = TaskReporter()
        shim = _SplitTaskShim(rep)
        shim.kill_event = run.kill
        run.task = shim
        work = os.path.join(self.local_dir, spec.job_id, spec.attempt_id)
        payload = {
            "attempt_id": spec.attempt_id, "is_map": is_map, "partition": spec.partition,
            "split": spec.split, "run_on_gpu": spec.run_on_gpu,
            "gpu_device_id": spec.gpu_device_id, "num_maps": spec.num_maps,
            "map_outputs": [(a, o["path"]) for _tid, a, o in spec.map_outputs] if not is_map
            else [],
            "conf": js.conf.to_dict(), "work_dir": work,
            "log_dir": os.path.join(self.local_dir, "userlogs", spec.attempt_id),
            "progress_interval": js.conf.get_int("hbmr.task.progress.interval.ms", 1000) / 1e3,
        }

        def _progress(p):
            run.status.progress = float(p)
        return self._children().run_task(spec.job_id, js.conf, payload, rep, run.kill,
                                         progress_cb=_progress)

    def job_result(self, job_id):
        js = self.jobs.get(str(job_id))
        if js is None:
            return self._results.get(str(job_id))
        return js.result


def _lower_priority(nice):
    if nice > 0 and hasattr(os, "setpriority"):
        try:
            os.setpriority(os.PRIO_PROCESS, threading.get_native_id(), nice)
        except OSError:
            pass


class _SplitTaskShim:
    def __init__(self, reporter):
        self.reporter = reporter
        self.kill_event = threading.Event()


def _split_from_dict(d):
    if d.get("kind") == "class":
        cls = load_class(d["cls"])
        return cls.deserialize(bytes.fromhex(d["data"]))
    raise ValueError(f"cannot rebuild split {d}")


_ = queue
