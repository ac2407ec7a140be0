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

CapacityScheduler (contrib/capacity-scheduler): queues
``mapred.queue.names`` with ``mapred.capacity-scheduler.queue.<q>.capacity``
percent; a job's queue is ``mapred.job.queue.name``.  Unused capacity flows to
queues with demand; inside a queue jobs run in priority/submit order.
"""
from __future__ import annotations

import math

from .hybrid import HybridTaskScheduler, _prio

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

    def begin_round(self, tr, total_cpu, total_gpu):
        jt = self.jt
        self.jobs = [j for j in jt.job_queue if not j.completed()]
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
    def pool_of(self, jip):
        c = jip.conf
        p = c.get("mapred.fairscheduler.pool")
        if p:
            return p
        prop = self.conf.get("mapred.fairscheduler.poolnameproperty", "user.name")
        return c.get(prop) or c.get_user()

    def _pool_conf(self, pool, key, default):
        v = self.conf.get(f"hbmr.fair.pool.{pool}.{key}")
        return type(default)(v) if v is not None else default

    def compute_shares(self, kind, total):
        pools: dict = {}
        for j in self.jobs:
            pools.setdefault(self.pool_of(j), []).append(j)
        names = sorted(pools)
        demands = [sum(self.demand[j][kind] for j in pools[p]) for p in names]
        weights = [self._pool_conf(p, "weight", 1.0) for p in names]
        minkey = {"gpu": "minGpuMaps", "cpu": "minMaps", "reduce": "minReduces"}[kind]
        mins = [float(self._pool_conf(p, minkey, 0)) for p in names]
        pshare = water_fill(total, demands, weights, mins)
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
    def queue_of(self, jip):
        return jip.conf.get("mapred.job.queue.name", "default")

    def compute_shares(self, kind, total):
        names = [q.strip() for q in self.conf.get("mapred.queue.names", "default").split(",")
                 if q.strip()]
        queues: dict = {q: [] for q in names}
        for j in self.jobs:
            queues.setdefault(self.queue_of(j), []).append(j)
        names = list(queues)
        caps = [self.conf.get_float(f"mapred.capacity-scheduler.queue.{q}.capacity",
                                    100.0 / max(1, len(names))) for q in names]
        demands = [sum(self.demand[j][kind] for j in queues[q]) for q in names]
        guaranteed = [total * c / 100.0 for c in caps]
        # guaranteed capacity first, then the unused remainder ∝ capacity
        qshare = water_fill(total, demands, [max(c, 1e-6) for c in caps], guaranteed)
        for q, qs in zip(names, qshare):
            left = qs
            for j in sorted(queues[q], key=lambda j: (_prio(j.priority), j.submit_time)):
                s = min(left, self.demand[j][kind])
                self.shares[j][kind] = s
                left -= s
