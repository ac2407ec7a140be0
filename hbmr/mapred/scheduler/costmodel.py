"""Profiled CPU-vs-GPU cost model (the fork's scheduler inputs, redesigned).

The reference recomputes mean CPU/GPU map-task times by regenerating every
TaskReport of every running job on every heartbeat under the JobTracker lock
(JobInProgress.java:508-618 → JobTracker.getMapTaskReports),
takes the accel factor from the last job only (B5) and leaves its
min-makespan solver commented out (JobQueueTaskScheduler.java:181-220, G3).

Here:
* per job *signature* (mapper/input format/split size), O(1) running stats of
  completed CPU and GPU map-task durations (mean + EWMA), shared across jobs of
  the same signature so iterative jobs (K-Means iterations) start profiled;
* running attempts give a censored lower bound: a CPU probe that has run for
  t seconds proves t_cpu ≥ t, so the GPU/CPU ratio is bounded before the probe
  finishes (a sampled probe's elapsed time is scaled to a whole split);
* GPU attempts wait in a device queue behind each other: their age is queue
  time, not execution time, so it never raises a GPU estimate that completed
  tasks already give (it did, and the inflated t_gpu handed maps to CPUs);
* the min-makespan split of P pending maps over C CPU and G GPU slots,
  ``min_x max(ceil(x/C)·t_c, ceil((P-x)/G)·t_g)``, is solved exactly in O(P/C).
"""
from __future__ import annotations

import math
import threading
from dataclasses import dataclass, field


GPU_WINDOW = 64      # tasks per decay step of a batched (GPU) estimate


@dataclass
class TimeStats:
    n: int = 0
    total: float = 0.0
    ewma: float = 0.0
    min: float = math.inf
    max: float = 0.0
    running: dict = field(default_factory=dict)   # attempt -> start time
    lower_bound: float = 0.0   # censored: killed/failed attempts ran at least this long
    probe: str | None = None   # the first attempt on this slot type (profiling probe)
    queued: bool = False       # attempts wait in a queue (GPU): age is not run time
    scale: dict = field(default_factory=dict)     # attempt -> 1/fraction (sampled probes)
    # the estimate is a ratio of decayed sums (time / tasks), one decay step
    # per completion event: a single task or a whole batch of GPU tasks (whose
    # device time is the part of the batch's interval no other batch covered —
    # hbmr/gpu/busy.py — so the batches of two slot streams alternate large and
    # small shares; a per-task EWMA that a batch of n tasks stepped n times
    # tracked the last batch's share alone: 15 µs against 0.25 ms per split)
    wnum: float = 0.0
    wden: float = 0.0
    # GPU batches of jobs not folded into (wnum, wden) yet: job -> [time, tasks].
    # A job's batches' shares of the device sum to its busy time only over the
    # whole job (the first batches of each slot stream get most of the union,
    # the last ones little), so the decay steps once per job — a step per
    # window of tasks weighted a job's cheap tail and read ~14 % low at job end
    open_jobs: dict = field(default_factory=dict)

    def _refresh(self):
        num, den = self.wnum, self.wden
        for t, k in self.open_jobs.values():
            num += t
            den += k
        self.ewma = num / den if den > 0 else 0.0

    def _decay(self, dt_total: float, n: int, alpha: float, per: float = 1.0):
        # one step of (1 - alpha) per ``per`` tasks
        keep = (1.0 - alpha) ** (n / per)
        self.wnum = keep * self.wnum + dt_total
        self.wden = keep * self.wden + n
        self._refresh()

    def add_job_batch(self, job, dt_total: float, n: int, alpha: float, keep_open: int = 2):
        """A batch of ``n`` tasks of ``job`` charged ``dt_total`` seconds.  The
        ``keep_open`` latest jobs stay whole; an older one folds in with one
        decay step of (1 - alpha)."""
        acc = self.open_jobs.get(job)
        if acc is None:
            while len(self.open_jobs) >= keep_open:
                t, k = self.open_jobs.pop(next(iter(self.open_jobs)))
                self.wnum = (1.0 - alpha) * self.wnum + t
                self.wden = (1.0 - alpha) * self.wden + k
            acc = self.open_jobs[job] = [0.0, 0]
        acc[0] += dt_total
        acc[1] += n
        self._refresh()

    def add(self, dt: float, alpha: float):
        self.n += 1
        self.total += dt
        self._decay(dt, 1, alpha)
        self.min = min(self.min, dt)
        self.max = max(self.max, dt)

    @property
    def mean(self):
        return self.total / self.n if self.n else 0.0

    def estimate(self, now: float):
        """(estimate seconds or None, is_lower_bound)."""
        sc = self.scale
        if self.n:
            est = self.ewma
            if self.queued:
                return est, False
            # a running attempt older than the estimate raises it (stragglers)
            oldest = max(((now - s) * sc.get(a, 1.0) for a, s in self.running.items()),
                         default=0.0)
            if oldest > 2 * est:
                return oldest, True
            return est, False
        lb = max([(now - s) * sc.get(a, 1.0) for a, s in self.running.items()] +
                 [self.lower_bound])
        if lb > 0:
            return lb, True
        return None, False


class CostModel:
    def __init__(self, alpha: float = 0.3):
        self.alpha = alpha
        self._lock = threading.Lock()
        self._stats: dict[str, dict[str, TimeStats]] = {}

    def _get(self, sig):
        d = self._stats.get(sig)
        if d is None:
            d = self._stats[sig] = {"cpu": TimeStats(), "gpu": TimeStats(queued=True)}
        return d

    def is_probe(self, sig, attempt, on_gpu) -> bool:
        with self._lock:
            return self._get(sig)["gpu" if on_gpu else "cpu"].probe == attempt

    def task_started(self, sig, attempt, on_gpu, t, fraction=1.0):
        """``fraction`` < 1: a sampled probe timed on that fraction of a split."""
        with self._lock:
            st = self._get(sig)["gpu" if on_gpu else "cpu"]
            st.running[attempt] = t
            if fraction < 1.0:
                st.scale[attempt] = 1.0 / fraction
            if st.probe is None and st.n == 0:
                st.probe = attempt

    def tasks_started(self, sig, attempts, on_gpu, t):
        with self._lock:
            st = self._get(sig)["gpu" if on_gpu else "cpu"]
            if st.probe is None and st.n == 0 and attempts:
                st.probe = attempts[0]
            run = st.running
            for a in attempts:
                run[a] = t

    def tasks_finished(self, sig, attempts, on_gpu, dt_each, job=None):
        """A batch of attempts of ``job`` that each took ``dt_each`` seconds
        (GPU tasks completed by one event pair share its device time)."""
        with self._lock:
            st = self._get(sig)["gpu" if on_gpu else "cpu"]
            pop = st.running.pop
            for a in attempts:
                pop(a, None)
            if dt_each >= 0 and attempts:
                n = len(attempts)
                if job is not None:
                    st.add_job_batch(job, dt_each * n, n, self.alpha)
                else:
                    # no job identity: a step per GPU_WINDOW tasks (about a
                    # 128-split job's worth of batches)
                    st._decay(dt_each * n, n, self.alpha, GPU_WINDOW)
                st.n += n
                st.total += dt_each * n
                st.min = min(st.min, dt_each)
                st.max = max(st.max, dt_each)

    def task_finished(self, sig, attempt, on_gpu, start, finish, succeeded=True):
        with self._lock:
            st = self._get(sig)["gpu" if on_gpu else "cpu"]
            st.running.pop(attempt, None)
            k = st.scale.pop(attempt, 1.0)
            if succeeded and finish >= start:
                st.add(finish - start, self.alpha)
            elif not succeeded and finish > start:
                # a killed attempt (e.g. a CPU probe overtaken by its GPU backup)
                # still proves the task takes at least this long on that slot type
                st.lower_bound = max(st.lower_bound, (finish - start) * k)

    def stats(self, sig, on_gpu) -> TimeStats:
        with self._lock:
            return self._get(sig)["gpu" if on_gpu else "cpu"]

    def finished_counts(self, sig):
        with self._lock:
            d = self._get(sig)
            return d["cpu"].n, d["gpu"].n

    def mean_times(self, sig):
        with self._lock:
            d = self._get(sig)
            return d["cpu"].mean, d["gpu"].mean

    def acceleration(self, sig, now: float):
        """GPU speed-up t_cpu / t_gpu (the reference's accelarationFactor,
        JobQueueTaskScheduler.java:175-177), or None when unknown.  Returns
        (value, is_lower_bound)."""
        with self._lock:
            d = self._get(sig)
            tc, tc_lb = d["cpu"].estimate(now)
            tg, _ = d["gpu"].estimate(now)
        if tc is None or tg is None or tg <= 0:
            return None, False
        return tc / tg, tc_lb

    def snapshot(self):
        with self._lock:
            return {sig: {k: {"n": v.n, "mean": v.mean, "ewma": v.ewma, "running": len(v.running),
                              "lower_bound": v.lower_bound} for k, v in d.items()}
                    for sig, d in self._stats.items()}


def min_makespan_cpu_tasks(pending: int, cpu_slots: int, gpu_slots: int, t_cpu: float,
                           t_gpu: float, gpu_backlog: int = 0) -> int:
    """Number of the ``pending`` tasks to give CPU slots so the makespan
    max(ceil(x/C)·t_c, ceil((B+P-x)/G)·t_g) is minimal (Shirahata et al.'s
    objective, made live); B = tasks already queued on the GPUs (a deep GPU
    queue is work the CPUs can shorten).  Ties go to fewer CPU tasks."""
    if pending <= 0:
        return 0
    if gpu_slots <= 0:
        return pending
    if cpu_slots <= 0 or t_cpu is None or t_gpu is None:
        return 0
    b = max(0, gpu_backlog)
    best_x, best = 0, math.ceil((pending + b) / gpu_slots) * t_gpu
    waves = math.ceil(pending / cpu_slots)
    for w in range(1, waves + 1):
        x = min(pending, w * cpu_slots)
        cost = max(w * t_cpu, math.ceil((pending + b - x) / gpu_slots) * t_gpu)
        if cost < best * (1 - 1e-9):
            best, best_x = cost, x
    if best_x:
        # the optimum's CPU wave need not be full: the fewest CPU tasks that
        # still let the GPUs finish the rest within ``best``
        fit = math.floor(best / t_gpu * (1 + 1e-9)) * gpu_slots
        best_x = min(best_x, max(1, pending + b - fit))
    return best_x


def makespan_estimates(pending, cpu_slots, gpu_slots, t_cpu, t_gpu):
    """CPU-only, GPU-only, greedy and optimal makespan estimates (the quantities
    the reference logs at JobQueueTaskScheduler.java:181-220)."""
    out = {}
    if t_cpu and cpu_slots:
        out["cpu_only"] = math.ceil(pending / cpu_slots) * t_cpu
    if t_gpu and gpu_slots:
        out["gpu_only"] = math.ceil(pending / gpu_slots) * t_gpu
    if t_cpu and t_gpu and cpu_slots and gpu_slots:
        x = min_makespan_cpu_tasks(pending, cpu_slots, gpu_slots, t_cpu, t_gpu)
        out["optimal"] = max(math.ceil(x / cpu_slots) * t_cpu if x else 0.0,
                             math.ceil((pending - x) / gpu_slots) * t_gpu)
        out["optimal_cpu_tasks"] = x
        # greedy: every slot takes the next task as it frees
        tc = [0.0] * cpu_slots
        tg = [0.0] * gpu_slots
        for _ in range(pending):
            ic = min(range(cpu_slots), key=lambda i: tc[i])
            ig = min(range(gpu_slots), key=lambda i: tg[i])
            if tc[ic] <= tg[ig]:
                tc[ic] += t_cpu
            else:
                tg[ig] += t_gpu
        out["greedy"] = max(max(tc), max(tg))
    return out
