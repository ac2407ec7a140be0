"""GPU-aware Fair and Capacity schedulers.

The reference's contrib FairScheduler and CapacityTaskScheduler treat GPU
slots as generic map slots (FairScheduler.java:534,
CapacityTaskScheduler.java:1021-1022).  Here both share CPU map
slots, GPU map slots (× queue depth) and reduce slots *separately*, and keep
the hybrid policy's per-job CPU gating and data/HBM locality: they only
decide which job gets the next slot of each kind (on top of
:class:`~hbmr.mapred.scheduler.hybrid.HybridTaskScheduler`).

FairScheduler (contrib/fairscheduler): jobs belong to pools
(``mapred.fairscheduler.pool``, else the property named by
``mapred.fairscheduler.poolnameproperty``, default ``user.name``).  Pool
``p`` has ``hbmr.fair.pool.<p>.weight`` (1.0), ``.minMaps`` / ``.minGpuMaps`` /
``.minReduces`` (0) and ``.mode`` (fair|fifo).  Shares are water-filled:
min shares first, then by weight, never above a pool's demand; inside a pool
jobs split equally (fair) or in submit order (fifo).  The most starved job
(running / share) is served first.

Pools can instead (or as well) be described by the reference's allocation
file (``mapred.fairscheduler.allocation.file``, see
:mod:`~hbmr.mapred.scheduler.pools`), reloaded while the JobTracker runs.
Job limits (FairScheduler.updateRunnability): jobs are made runnable in
priority/submit order while their pool has fewer than ``maxRunningJobs``
(``poolMaxJobsDefault``) and their user fewer than the user's
``maxRunningJobs`` (``userMaxJobsDefault``) runnable jobs; the others get no
slots until one finishes.  ``maxMaps`` / ``maxGpuMaps`` / ``maxReduces`` cap a
pool's demand (so its share) per slot kind.

Preemption (FairScheduler.preemptTasksIfNecessary, FairScheduler.java:837),
with ``mapred.fairscheduler.preemption`` = true: a pool below its min share for
``hbmr.fair.pool.<p>.minSharePreemptionTimeout`` seconds (default 60), or below
half its fair share for ``mapred.fairscheduler.fairSharePreemptionTimeout``
seconds (default 600), gets slots back by killing the most recently launched
attempts of pools above their fair share (never taking a pool below it).
Preempted attempts are KILLED, not FAILED: their TIPs go back to pending.

CapacityScheduler (contrib/capacity-scheduler): queues
``mapred.queue.names`` with ``mapred.capacity-scheduler.queue.<q>.capacity``
percent and an optional hard ``.maximum-capacity``; a job's queue is
``mapred.job.queue.name``.  Unused capacity flows to queues with demand.
Job limits (CapacitySchedulerQueue.java:378-400, 1227-1345, CapacitySchedulerConf
keys ``mapred.capacity-scheduler.maximum-system-jobs`` (5000),
``…queue.<q>.init-accept-jobs-factor`` (10),
``…queue.<q>.maximum-initialized-active-tasks`` (200000) and
``…-per-user`` (100000)): a queue initialises at most ceil(system jobs ×
capacity%) jobs and a user ceil(that × minimum-user-limit%), within the
active-task limits; uninitialised jobs wait (no slots).  Submission is
refused when the queue already holds init × factor jobs (user: likewise) or
a job has more tasks than the per-user active-task limit.
Inside a queue jobs run in priority/submit order, and each user is capped at
max(queue share × ``.minimum-user-limit-percent`` / 100, queue share / active
users) (CapacitySchedulerQueue.java:724 user limits).  Memory matching
(CapacityTaskScheduler.java:315-340): with ``mapred.cluster.map.memory.mb`` /
``mapred.cluster.reduce.memory.mb`` set, a job asking for
``mapred.job.map.memory.mb`` / ``mapred.job.reduce.memory.mb`` above the slot
size occupies ceil(job / slot) slots per task, and a job larger than
``mapred.cluster.max.map.memory.mb`` is rejected at submission.
"""
from __future__ import annotations

import logging
import math
import time

from .hybrid import HybridTaskScheduler, _prio
from .pools import INF, PoolManager

log = logging.getLogger("hbmr.scheduler.fair")

KINDS = ("gpu", "cpu", "reduce")


def water_fill(total, demands, weights, mins=None):
    """Share ``total`` slots among claimants: mins first, then ∝ weight, capped
    by demand; returns fractional shares."""
    n = len(demands)
    share = [0.0] * n
    mins = mins or [0.0] * n
    left = float(total)
    for i in range(n):
        s = min(mins[i], demands[i], left)
        share[i] = s
        left -= s
    active = [i for i in range(n) if share[i] < demands[i]]
    while left > 1e-9 and active:
        wsum = sum(weights[i] for i in active) or 1.0
        given = 0.0
        nxt = []
        for i in active:
            add = left * weights[i] / wsum
            room = demands[i] - share[i]
            take = min(add, room)
            share[i] += take
            given += take
            if share[i] < demands[i] - 1e-9:
                nxt.append(i)
        left -= given
        if given <= 1e-12:
            break
        active = nxt
    return share


class _ShareScheduler(HybridTaskScheduler):
    """Common machinery: per-kind demand/running, shares, starvation order."""

    def admitted(self, jobs):
        """Jobs allowed to take slots this round (job limits); default all."""
        return set(jobs)

    def begin_round(self, tr, total_cpu, total_gpu):
        jt = self.jt
        self.jobs = [j for j in jt.job_queue if not j.completed()]
        ok = self.admitted(self.jobs)
        totals = {"gpu": total_gpu * self.queue_depth, "cpu": total_cpu,
                  "reduce": sum(t.status.max_reduce_slots for t in jt.trackers.values()
                                if not t.blacklisted)}
        self.running = {}
        self.demand = {}
        for j in self.jobs:
            pend = len(j.pending_maps)
            red_run = sum(1 for t in j.reduces if t.is_running())
            red_pend = sum(1 for t in j.reduces if not t.is_complete() and not t.is_running()) \
                if j.maps_complete() else 0
            self.running[j] = {"gpu": j.running_gpu, "cpu": j.running_cpu, "reduce": red_run}
            if j not in ok:
                self.demand[j] = {"gpu": 0, "cpu": 0, "reduce": 0}
                continue
            self.demand[j] = {"gpu": (pend + j.running_gpu) if j.gpu_capable else 0,
                              "cpu": (pend + j.running_cpu) if j.cpu_capable else 0,
                              "reduce": red_pend + red_run}
        self.shares = {j: {} for j in self.jobs}
        for kind in KINDS:
            self.compute_shares(kind, totals[kind])

    def compute_shares(self, kind, total):
        raise NotImplementedError

    def job_limit(self, jip, kind):
        sh = self.shares.get(jip, {}).get(kind)
        if sh is None:
            return 1 << 30
        return max(0, math.ceil(sh - 1e-9) - self.running[jip][kind])

    def job_order(self, tr):
        def starve(j):
            worst = 1e9
            for kind in ("gpu", "cpu"):
                sh = self.shares[j].get(kind, 0.0)
                if sh > 0:
                    worst = min(worst, self.running[j][kind] / sh)
            return (worst, _prio(j.priority), j.submit_time)
        return sorted(self.jobs, key=starve)


class FairScheduler(_ShareScheduler):
    def __init__(self, jt, conf):
        super().__init__(jt, conf)
        self.preemption = conf.get_boolean("mapred.fairscheduler.preemption", False)
        self.pools = PoolManager(conf)
        self._fair_timeout = conf.get_float("mapred.fairscheduler.fairSharePreemptionTimeout",
                                            600.0)
        self.preempted = 0
        self._below_min: dict = {}    # (pool, kind) -> since
        self._below_fair: dict = {}
        self.pool_shares: dict = {}   # kind -> {pool: share}

    def pool_of(self, jip):
        c = jip.conf
        p = c.get("mapred.fairscheduler.pool")
        if p:
            return p
        prop = self.conf.get("mapred.fairscheduler.poolnameproperty", "user.name")
        return c.get(prop) or c.get_user()

    @property
    def fair_timeout(self):
        return self.pools.fair_share_timeout(self._fair_timeout)

    def _pool_conf(self, pool, key, default):
        return self.pools.pool_value(pool, key, default)

    def admitted(self, jobs):
        """FairScheduler.updateRunnability: runnable in priority/submit order
        within the pool's and the user's running-job limits."""
        self.pools.reload_if_necessary()
        per_pool: dict = {}
        per_user: dict = {}
        ok = set()
        for j in sorted(jobs, key=lambda j: (_prio(j.priority), j.submit_time)):
            p, u = self.pool_of(j), j.conf.get_user()
            if per_pool.get(p, 0) < self.pools.pool_max_jobs(p) and \
                    per_user.get(u, 0) < self.pools.user_max_jobs(u):
                per_pool[p] = per_pool.get(p, 0) + 1
                per_user[u] = per_user.get(u, 0) + 1
                ok.add(j)
        self.runnable = ok
        return ok

    def compute_shares(self, kind, total):
        pools: dict = {}
        for j in self.jobs:
            pools.setdefault(self.pool_of(j), []).append(j)
        names = sorted(pools)
        maxkey = {"gpu": "maxGpuMaps", "cpu": "maxMaps", "reduce": "maxReduces"}[kind]
        demands = []
        for p in names:
            cap = self._pool_conf(p, maxkey, INF)
            if kind == "gpu" and cap == INF:
                cap = self._pool_conf(p, "maxMaps", INF)
            demands.append(min(sum(self.demand[j][kind] for j in pools[p]), cap))
        weights = [self._pool_conf(p, "weight", 1.0) for p in names]
        minkey = {"gpu": "minGpuMaps", "cpu": "minMaps", "reduce": "minReduces"}[kind]
        mins = [float(self._pool_conf(p, minkey, 0)) for p in names]
        pshare = water_fill(total, demands, weights, mins)
        self.pool_shares[kind] = {p: (ps, mn, pools[p]) for p, ps, mn in zip(names, pshare, mins)}
        for p, ps in zip(names, pshare):
            js = sorted(pools[p], key=lambda j: (_prio(j.priority), j.submit_time))
            if self._pool_conf(p, "mode", "fair") == "fifo":
                left = ps
                for j in js:
                    s = min(left, self.demand[j][kind])
                    self.shares[j][kind] = s
                    left -= s
            else:
                ds = [self.demand[j][kind] for j in js]
                for j, s in zip(js, water_fill(ps, ds, [1.0] * len(js))):
                    self.shares[j][kind] = s


class CapacityScheduler(_ShareScheduler):
    PRE = "mapred.capacity-scheduler.queue"

    def __init__(self, jt, conf):
        super().__init__(jt, conf)
        self.initialized: set = set()       # job ids admitted (initialised) so far

    def _limits(self, q):
        """(maxJobsToInit, maxJobsPerUserToInit, maxActiveTasks,
        maxActiveTasksPerUser, initToAcceptFactor) of queue ``q``."""
        c = self.conf
        names = [x.strip() for x in c.get("mapred.queue.names", "default").split(",") if x.strip()]
        cap = c.get_float(f"{self.PRE}.{q}.capacity", 100.0 / max(1, len(names)))
        ul = c.get_float(f"{self.PRE}.{q}.minimum-user-limit-percent", 100.0)
        sys_jobs = c.get_int("mapred.capacity-scheduler.maximum-system-jobs", 5000)
        if sys_jobs <= 0:
            raise ValueError(f"Invalid maximum system jobs: {sys_jobs}")
        factor = c.get_int(f"{self.PRE}.{q}.init-accept-jobs-factor",
                           c.get_int("mapred.capacity-scheduler.default-init-accept-jobs-factor",
                                     10))
        if factor <= 0:
            raise ValueError(f"Invalid maximum jobs per user configuration {factor}")
        tasks = c.get_int(f"{self.PRE}.{q}.maximum-initialized-active-tasks", c.get_int(
            "mapred.capacity-scheduler.default-maximum-active-tasks-per-queue", 200000))
        tasks_u = c.get_int(f"{self.PRE}.{q}.maximum-initialized-active-tasks-per-user", c.get_int(
            "mapred.capacity-scheduler.default-maximum-active-tasks-per-user", 100000))
        jobs = math.ceil(sys_jobs * cap / 100.0)
        jobs_u = math.ceil(sys_jobs * cap / 100.0 * ul / 100.0)
        return jobs, jobs_u, tasks, tasks_u, factor

    @staticmethod
    def _tasks(j):
        return len(j.maps) + len(j.reduces)

    def check_submission(self, jip):
        """CapacitySchedulerQueue.checkJobSubmissionLimits: a refusal reason or None."""
        q, u = self.queue_of(jip), jip.conf.get_user()
        jobs, jobs_u, _tasks, tasks_u, factor = self._limits(q)
        if self._tasks(jip) > tasks_u:
            return (f"Job '{jip.job_id}' from user '{u}' rejected since it has "
                    f"{self._tasks(jip)} tasks which exceeds the limit of {tasks_u} tasks "
                    f"per-user which can be initialized for queue '{q}'")
        live = [j for j in self.jt.job_queue + [w for ws in self.jt.waiting.values() for w in ws]
                if not j.completed() and j is not jip and self.queue_of(j) == q]
        if len(live) >= jobs * factor:
            return (f"Job '{jip.job_id}' from user '{u}' rejected since queue '{q}' already "
                    f"has {len(live)} jobs - Exceeds limit of {jobs * factor} jobs to accept")
        mine = sum(1 for j in live if j.conf.get_user() == u)
        if mine >= jobs_u * factor:
            return (f"Job '{jip.job_id}' rejected since user '{u}' already has {mine} jobs - "
                    f"Exceeds limit of {jobs_u * factor} jobs to accept in queue '{q}'")
        return None

    def admitted(self, jobs):
        """JobInitializationPoller + initializeJobForQueue/ForUser: jobs are
        initialised in priority/submit order within the queue and user job
        and active-task limits; an initialised job stays so until it ends."""
        live = {j.job_id for j in jobs}
        self.initialized &= live
        ok = set()
        stats: dict = {}
        order = sorted(jobs, key=lambda j: (j.job_id not in self.initialized, _prio(j.priority),
                                            j.submit_time))
        for j in order:
            q, u = self.queue_of(j), j.conf.get_user()
            jobs_q, jobs_u, tasks_q, tasks_u, _f = self._limits(q)
            st = stats.setdefault(q, {"jobs": 0, "tasks": 0, "ujobs": {}, "utasks": {}})
            n = self._tasks(j)
            if j.job_id not in self.initialized:
                if st["jobs"] >= jobs_q or st["tasks"] + n > tasks_q or \
                        st["ujobs"].get(u, 0) >= jobs_u or st["utasks"].get(u, 0) + n > tasks_u:
                    continue
                self.initialized.add(j.job_id)
            st["jobs"] += 1
            st["tasks"] += n
            st["ujobs"][u] = st["ujobs"].get(u, 0) + 1
            st["utasks"][u] = st["utasks"].get(u, 0) + n
            ok.add(j)
        return ok

    def slots_per_task(self, jip, kind):
        """Memory-based slot matching: slots a task of ``jip`` occupies."""
        kk = "reduce" if kind == "reduce" else "map"
        slot = self.conf.get_int(f"mapred.cluster.{kk}.memory.mb", -1)
        need = jip.conf.get_int(f"mapred.job.{kk}.memory.mb", -1)
        if slot <= 0 or need <= 0:
            return 1
        return max(1, math.ceil(need / slot))

    def queue_of(self, jip):
        return jip.conf.get("mapred.job.queue.name", "default")

    def compute_shares(self, kind, total):
        names = [q.strip() for q in self.conf.get("mapred.queue.names", "default").split(",")
                 if q.strip()]
        queues: dict = {q: [] for q in names}
        for j in self.jobs:
            queues.setdefault(self.queue_of(j), []).append(j)
        names = list(queues)
        pre = "mapred.capacity-scheduler.queue"
        caps = [self.conf.get_float(f"{pre}.{q}.capacity", 100.0 / max(1, len(names)))
                for q in names]
        maxcaps = [self.conf.get_float(f"{pre}.{q}.maximum-capacity", -1.0) for q in names]
        # demand in slots (high-memory tasks take several), capped by max capacity
        demands = []
        for q, mx in zip(names, maxcaps):
            d = sum(self.demand[j][kind] * self.slots_per_task(j, kind) for j in queues[q])
            if mx > 0:
                d = min(d, total * mx / 100.0)
            demands.append(d)
        guaranteed = [total * c / 100.0 for c in caps]
        # guaranteed capacity first, then the unused remainder ∝ capacity
        qshare = water_fill(total, demands, [max(c, 1e-6) for c in caps], guaranteed)
        for q, qs in zip(names, qshare):
            ul = self.conf.get_float(f"{pre}.{q}.minimum-user-limit-percent", 100.0)
            users: dict = {}
            for j in queues[q]:
                users.setdefault(j.conf.get_user(), []).append(j)
            active = [u for u, js in users.items() if any(self.demand[j][kind] for j in js)]
            user_cap = max(qs * ul / 100.0, qs / max(1, len(active)))
            used: dict = {}
            left = qs
            for j in sorted(queues[q], key=lambda j: (_prio(j.priority), j.submit_time)):
                u = j.conf.get_user()
                spt = self.slots_per_task(j, kind)
                room = min(left, user_cap - used.get(u, 0.0))
                s = max(0.0, min(room, self.demand[j][kind] * spt))
                self.shares[j][kind] = s / spt      # tasks
                used[u] = used.get(u, 0.0) + s
                left -= s


def _fair_begin_round(self, tr, total_cpu, total_gpu):
    _ShareScheduler.begin_round(self, tr, total_cpu, total_gpu)
    if self.preemption:
        self.preempt_if_necessary(time.time())


def _preempt_if_necessary(self, now):
    """FairScheduler.preemptTasksIfNecessary: per slot kind, pools starved past
    their timeout take slots back from pools above their fair share."""
    for kind, pools in self.pool_shares.items():
        running = {p: sum(self.running[j][kind] for j in jobs)
                   for p, (_sh, _mn, jobs) in pools.items()}
        want = 0
        for p, (share, mn, _jobs) in pools.items():
            tmin = float(self._pool_conf(p, "minSharePreemptionTimeout", 60.0))
            key = (p, kind)
            target = 0
            if running[p] < min(mn, share) - 1e-9:
                since = self._below_min.setdefault(key, now)
                if now - since >= tmin:
                    target = max(target, math.ceil(min(mn, share) - running[p]))
            else:
                self._below_min.pop(key, None)
            if running[p] < share / 2 - 1e-9:
                since = self._below_fair.setdefault(key, now)
                if now - since >= self.fair_timeout:
                    target = max(target, math.ceil(share - running[p]))
            else:
                self._below_fair.pop(key, None)
            want += target
        if want > 0:
            self._preempt(kind, pools, running, want, now)


def _preempt(self, kind, pools, running, want, now):
    # victims: attempts of pools above their fair share, newest first, without
    # taking any pool below its share
    cands = []
    for p, (share, _mn, jobs) in pools.items():
        over = running[p] - math.ceil(share - 1e-9)
        if over <= 0:
            continue
        mine = []
        for j in jobs:
            tips = j.reduces if kind == "reduce" else j.maps
            for tip in tips:
                for a in tip.running_attempts():
                    if kind == "reduce" or (a.run_on_gpu == (kind == "gpu")):
                        mine.append(a)
        mine.sort(key=lambda a: -a.start)
        cands += mine[:over]
    cands.sort(key=lambda a: -a.start)
    for a in cands[:want]:
        self._below_min.clear()
        self._below_fair.clear()
        self.jt.preempt_attempt(a, f"preempted by the fair scheduler ({kind} slots)")
        self.preempted += 1


FairScheduler.begin_round = _fair_begin_round
FairScheduler.preempt_if_necessary = _preempt_if_necessary
FairScheduler._preempt = _preempt
