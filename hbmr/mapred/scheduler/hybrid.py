"""GPU-aware map-task schedulers.

:class:`HybridTaskScheduler` is the redesign of the fork's
JobQueueTaskScheduler (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/
JobQueueTaskScheduler.java:86-575).  Per heartbeat of a
tracker it fills free GPU slots (device by device, data-locality first, every
GPU attempt told its device id) and then decides how many CPU map tasks a job
should get, under ``hbmr.scheduler.policy``:

* ``stock``    – GPU-unaware FIFO: every free slot takes the next task (the
                 baseline of Shirahata et al. and of the non-GPU-aware
                 schedulers, B10);
* ``optional`` – the fork's live rule (JobQueueTaskScheduler.java:290-291): CPU
                 slots stay idle while ``pending < accel × total GPU slots``;
* ``hybrid``   – (default) the fork's dead min-makespan solver made live
                 (JobQueueTaskScheduler.java:181-220): CPU slots take a task only
                 while the job's running CPU tasks are below the count x* that
                 minimises max(ceil(x/C)·t_cpu, ceil((P-x)/G)·t_gpu).  Before a
                 CPU profile exists one probe task runs on a CPU slot; a running
                 probe already bounds t_cpu from below (costmodel.py).

Locality (``obtain_map``): split resident in this device's HBM > resident on
this tracker > node-local by split locations > any, with delay scheduling
(``hbmr.locality.delay.heartbeats``) before a GPU takes a non-local split.
Reduces: classic reduces go to free reduce slots once all maps are done;
collective (RCCL) reduces are gang-launched, one pinned to each tracker.
"""
from __future__ import annotations

import logging
import time

from .costmodel import min_makespan_cpu_tasks

log = logging.getLogger("hbmr.scheduler")


class TaskScheduler:
    def __init__(self, jt, conf):
        self.jt = jt
        self.conf = conf

    def assign_tasks(self, tracker):
        raise NotImplementedError


class HybridTaskScheduler(TaskScheduler):
    def __init__(self, jt, conf):
        super().__init__(jt, conf)
        self.policy = conf.get("hbmr.scheduler.policy", "hybrid").lower()
        if conf.get_boolean("mapred.jobtracker.map.optionalscheduling", False) and \
                self.policy == "hybrid" and conf.get("hbmr.scheduler.policy.explicit") is None:
            self.policy = "optional"
        self.queue_depth = max(1, conf.get_int("hbmr.gpu.queue.depth", 4))
        self.locality_wait = conf.get_int("hbmr.locality.wait.ms", 500) / 1000.0
        # a classic (per-attempt) job's GPU maps for one device in one
        # response go out as one bulk launch too: the tracker then sends
        # Pipes maps to the device's child ahead of their threads and
        # reports them once per batch (TaskTracker._prelaunch_pipes,
        # _ReportGroup)
        self.classic_bulk = conf.get_boolean("hbmr.scheduler.gpu.bulk.classic", True)
        self.max_reduces_per_hb = conf.get_int("hbmr.scheduler.max.reduces.per.heartbeat", 4)
        self.speculate_after = conf.get_float("hbmr.speculative.slowdown", 3.0)
        # stock Hadoop only backs up attempts that ran > SPECULATIVE_LAG (60 s,
        # TaskInProgress.java) and lag in progress; the GPU-aware early backup
        # of CPU stragglers is part of the hybrid design
        self.stock_lag = conf.get_int("hbmr.speculative.stock.lag.ms", 60000) / 1000.0
        # split jobs are CPU-profiled by a sampled probe: the map on the first
        # 1/32 of one split, timed and scaled, while the GPUs run every real task
        self.probe_fraction = conf.get_float("hbmr.costmodel.probe.fraction", 1 / 32)
        # cap map launches per heartbeat response so a tracker can start the
        # first tasks while the rest are still being assigned (the response
        # says "more" and the tracker calls right back)
        self.max_maps_per_hb = max(1, conf.get_int("hbmr.scheduler.max.maps.per.heartbeat", 256))
        self._skips: dict = {}
        self.decisions = 0

    # -- cluster capacity ----------------------------------------------------------------
    def _totals(self):
        # cached until the cluster's capacity changes (JobTracker.cap_epoch):
        # this ran on every assignment call, O(trackers) each
        ep = getattr(self.jt, "cap_epoch", None)
        if ep is not None and getattr(self, "_tot_epoch", None) == ep:
            return self._tot
        cpu = gpu = ndev = 0
        for t in self.jt.trackers.values():
            if t.blacklisted:
                continue
            cpu += t.status.max_cpu_map_slots
            gpu += sum(g["max_slots"] for g in t.status.gpus)
            ndev += len(t.status.gpus)
        self._devices = ndev
        self._tot = (cpu, gpu)
        self._tot_epoch = ep
        return cpu, gpu

    def _gpu_servers(self, jip, total_gpu):
        """G of the makespan model.  A split job's GPU task time is the device's
        busy time per task (its slot streams overlap on one device: the time is
        de-overlapped by the runtime), so G counts devices; a per-attempt GPU
        Pipes task is timed on its slot, so G counts slots."""
        if jip.split_job is not None:
            return max(1, getattr(self, "_devices", 0)) if total_gpu else 0
        return total_gpu

    def _cpu_allowed(self, jip, total_cpu, total_gpu, now):
        total_gpu = self._gpu_servers(jip, total_gpu)
        if not jip.cpu_capable:
            return 0
        running_cpu = jip.running_maps(on_gpu=False)
        pending = jip.pending_map_count()
        if not jip.gpu_capable or total_gpu == 0:
            return pending
        if self.policy == "stock":
            return pending
        cm = self.jt.cost_model
        sig = jip.signature
        if self.policy == "optional":
            accel, _ = cm.acceleration(sig, now)
            if accel is None:
                accel = 1.0
            # !(optional && pendingMaps < accel * gpuSlots)  → CPU may take work
            return pending if not (pending < accel * total_gpu) else 0
        # hybrid (min-makespan)
        cs, gs = cm.stats(sig, False), cm.stats(sig, True)
        t_cpu, cpu_lb = cs.estimate(now)
        t_gpu, _ = gs.estimate(now)
        if t_cpu is None:
            if self._sampled_probing(jip):
                return 0   # the sampled probe (assign_tasks) profiles the CPU
            # profile: one CPU probe per signature (if none is running)
            return 1 if running_cpu == 0 and not cs.running else 0
        if cs.n == 0 and cpu_lb and cs.probe in cs.running:
            # only a censored bound while the probe still runs: wait for it
            # rather than betting more slots on a still-growing estimate
            return 0
        if t_gpu is None:
            return 0 if running_cpu else min(1, pending)
        x = min_makespan_cpu_tasks(pending + running_cpu, total_cpu, total_gpu, t_cpu, t_gpu,
                                   gpu_backlog=jip.running_maps(on_gpu=True))
        return max(0, x - running_cpu)

    # -- main entry -----------------------------------------------------------------
    def assign_tasks(self, tr):
        jt = self.jt
        actions = []
        now = time.time()
        total_cpu, total_gpu = self._totals()
        cpu_free = tr.status.max_cpu_map_slots - tr.running_cpu
        reduce_free = tr.status.max_reduce_slots - tr.running_reduce
        # stock Hadoop knows no queue behind a slot: one task per GPU slot
        depth = 1 if self.policy == "stock" else self.queue_depth
        # maps of staged jobs wait behind their gate (in the GPU worker, not on
        # the device queue) and have a budget of their own (_stage_maps): they
        # must not take the queue from the job they wait for — whose maps
        # beyond one queue's worth would otherwise never launch, and whose
        # reduce the gate waits on
        held = {}
        if jt.staged:
            name = tr.name
            for g in tr.status.gpus:
                dev = g["device"]
                n = sum(j.staged_launched.get((name, dev), 0) for j in jt.staged)
                if n:
                    held[dev] = n
        gpu_free = {g["device"]: g["max_slots"] * depth - tr.running_gpu.get(g["device"], 0) +
                    held.get(g["device"], 0) for g in tr.status.gpus}
        budget = self.max_maps_per_hb
        tr.more = False
        self.begin_round(tr, total_cpu, total_gpu)
        for jip in self.job_order(tr):
            if jip.completed():
                continue
            # ---- reduces
            if jip.reduces and self._reduces_may_start(jip):
                reduce_free = self._assign_reduces(tr, jip, reduce_free, actions)
            if not jip.pending_maps:
                # ---- speculative backups of stragglers onto idle GPUs
                if jip.speculative and jip.gpu_capable and not jip.maps_complete() and \
                        not jip.expect_mode:
                    self._speculate(tr, jip, gpu_free, now, actions)
                continue
            # ---- CPU maps (first, as the fork's loop order, JobQueueTaskScheduler.java
            # :295-387: the cost model decides how many; a CPU profile probe must
            # not be starved by the GPUs' much larger queue budget)
            if cpu_free > 0 and total_gpu > 0 and self._needs_sampled_probe(jip):
                actions.append(jt.launch(tr, jip.maps[0], on_gpu=False,
                                         profile_fraction=self.probe_fraction))
                cpu_free -= 1
                budget -= 1
            reserve = 0     # pending maps the min-makespan plan keeps for later CPU waves
            if jip.pending_maps and self.policy == "hybrid" and total_gpu > 0 and \
                    total_cpu > 0 and jip.cpu_capable and \
                    self.jt.cost_model.stats(jip.signature, False).n > 0:
                reserve = self._cpu_allowed(jip, total_cpu, total_gpu, now)
            if cpu_free > 0 and jip.pending_maps:
                allowed = min(self._cpu_allowed(jip, total_cpu, total_gpu, now),
                              self.job_limit(jip, "cpu"))
                spt = self.slots_per_task(jip, "cpu")
                while cpu_free >= spt and allowed > 0 and jip.pending_maps:
                    if budget <= 0:
                        tr.more = True
                        break
                    got = jip.obtain_map(tr, False, -1, allow_nonlocal=True)
                    if got is None:
                        break
                    tip, _ = got
                    actions.append(jt.launch(tr, tip, on_gpu=False, slots=spt))
                    cpu_free -= spt
                    allowed -= 1
                    reserve -= 1
                    budget -= 1
                    self.decisions += 1
            # ---- GPU maps
            if jip.gpu_capable:
                glim = self.job_limit(jip, "gpu")
                bulk = jip.split_job is not None   # split jobs: one bulk launch per device
                for dev in sorted(gpu_free):
                    batch = []
                    if bulk:
                        # one obtain_maps call takes the device's share at once
                        budget, glim = self._bulk_gpu(tr, jip, dev, gpu_free, reserve, budget,
                                                      glim, now, actions)
                        continue
                    # the min-makespan plan's later CPU waves stay pending: a deep GPU
                    # queue must not swallow them (they free the GPUs' tail)
                    while gpu_free[dev] > 0 and len(jip.pending_maps) > max(0, reserve) and \
                            glim > 0:
                        if budget <= 0:
                            tr.more = True
                            break
                        # delay scheduling: a GPU waits up to locality_wait for a
                        # split it holds in HBM / that names it before it steals a
                        # non-local one (a non-local split must be re-materialised)
                        key = (str(jip.job_id), tr.name, dev)
                        first = self._skips.get(key)
                        allow_nonlocal = self.policy == "stock" or (
                            first is not None and now - first >= self.locality_wait) or \
                            not jip.locality_possible()
                        got = jip.obtain_map(tr, True, dev, allow_nonlocal=allow_nonlocal)
                        if got is None:
                            if first is None:
                                self._skips[key] = now
                            break
                        tip, level = got
                        if level < 3:
                            self._skips.pop(key, None)
                        if self.classic_bulk:
                            batch.append(tip)
                        else:
                            actions.append(jt.launch(tr, tip, on_gpu=True, device=dev))
                        gpu_free[dev] -= 1
                        budget -= 1
                        glim -= 1
                        self.decisions += 1
                    if batch:
                        actions.append(jt.launch_gpu_batch(tr, batch, dev))
            if jip.speculative and jip.gpu_capable and not jip.pending_maps and \
                    not jip.expect_mode:
                self._speculate(tr, jip, gpu_free, now, actions)
        # ---- staged jobs (JobTracker._maybe_stage): GPU maps gated on the job
        # they wait for, and their collective reduce once every map is launched
        for jip in list(jt.staged):
            if jip.completed() or jip.staged_on is None:
                continue
            # maps first: once this tracker's maps are staged the reduce may
            # go out in the same response instead of a heartbeat of its own
            if jip.pending_maps and jip.gpu_capable:
                self._stage_maps(tr, jip, depth, actions)
            if jip.reduces and self._reduces_may_start(jip):
                reduce_free = self._assign_reduces(tr, jip, reduce_free, actions)
        return actions

    def _bulk_gpu(self, tr, jip, dev, gpu_free, reserve, budget, glim, now, actions):
        """A split job's maps for one device in one bulk launch: as many as
        the device's free queue, the plan's CPU reserve, the job's GPU limit
        and the response budget allow, local levels first (delay scheduling:
        a device waits up to locality_wait before it takes non-local splits)."""
        want = min(gpu_free[dev], len(jip.pending_maps) - max(0, reserve), glim)
        if want <= 0:
            return budget, glim
        if budget < want:
            tr.more = True
            want = budget
            if want <= 0:
                return budget, glim
        key = (str(jip.job_id), tr.name, dev)
        first = self._skips.get(key)
        allow_nonlocal = self.policy == "stock" or (
            first is not None and now - first >= self.locality_wait) or \
            not jip.locality_possible()
        got = jip.obtain_maps(tr, True, dev, want, allow_nonlocal=allow_nonlocal)
        if any(lv < 3 for _t, lv in got):
            self._skips.pop(key, None)
        if len(got) < want and key not in self._skips:
            self._skips[key] = now
        n = len(got)
        if n:
            actions.append(self.jt.launch_gpu_batch(tr, [t for t, _lv in got], dev))
            gpu_free[dev] -= n
            self.decisions += n
        return budget - n, glim - n

    def _assign_reduces(self, tr, jip, reduce_free, actions):
        jt = self.jt
        n_red = 0
        expect = jip.expect_mode and not jip.maps_complete()
        if jip.collective_reduce and jip.reduce_by_tracker:
            # a gang member per tracker: only this tracker's pinned reduce
            mine = jip.reduce_by_tracker.get(tr.name)
            tips = () if mine is None else (mine,)
        else:
            tips = jip.reduces
        for tip in tips:
            if jip.collective_reduce and tip.pinned_tracker != tr.name:
                continue
            if tip.is_complete() or tip.is_running():
                continue
            if jip.collective_reduce:
                pass
            elif reduce_free < self.slots_per_task(jip, "reduce") or \
                    n_red >= self.max_reduces_per_hb or \
                    n_red >= self.job_limit(jip, "reduce"):
                break
            extra = {"map_outputs": jt.reduce_inputs(jip, tr.name, expect=expect)}
            if expect:
                extra["expect"] = True
            spt = 1 if jip.collective_reduce else self.slots_per_task(jip, "reduce")
            actions.append(jt.launch(tr, tip, extra=extra, slots=spt))
            n_red += 1
            reduce_free -= spt
        return reduce_free

    def plan_staged(self, jip):
        """Whole-job placement of a just-staged split job: every GPU tracker's
        HBM-resident / node-local maps in one bulk launch per device, and —
        once no map is left pending — each tracker's collective reduce member
        (expect mode) in the same per-tracker record.  The records ride on
        each tracker's next response (tr.extra_actions) instead of being
        pulled one tracker heartbeat at a time, where a tracker whose maps
        were staged before the job's last ones needed a heartbeat of its own
        for its reduce.  What cannot be placed locally now stays pending for
        the per-heartbeat path (_stage_maps / assign_tasks)."""
        jt = self.jt
        if not jip.gpu_capable or jip.staged_on is None:
            return
        depth = 1 if self.policy == "stock" else self.queue_depth
        trackers = [t for _n, t in sorted(jt.trackers.items())
                    if t.status.gpus and t.status.healthy and not t.blacklisted]
        for tr in trackers:
            acts = []
            self._stage_maps(tr, jip, depth, acts)
            tr.extra_actions += acts
            tr.planned += _attempts_in(acts)
        if jip.pending_maps or not jip.reduces or not self._reduces_may_start(jip):
            return
        for tr in trackers:
            acts = []
            self._assign_reduces(tr, jip, tr.status.max_reduce_slots - tr.running_reduce, acts)
            tr.extra_actions += acts
            tr.planned += _attempts_in(acts)

    def _stage_maps(self, tr, jip, depth, actions):
        """Launch a staged job's pending maps that are local to this tracker's
        GPUs (HBM-resident / node-local splits), gated on the job it waits for;
        up to one queue depth per device."""
        for g in tr.status.gpus:
            dev = g["device"]
            cap = g["max_slots"] * depth - jip.staged_launched.get((tr.name, dev), 0)
            batch = [t for t, _lv in jip.obtain_maps(tr, True, dev, cap, allow_nonlocal=False)] \
                if cap > 0 and jip.pending_maps else []
            if batch:
                actions.append(self.jt.launch_gpu_batch(tr, batch, dev, gate=jip.staged_on))

    def _reduces_may_start(self, jip) -> bool:
        """Reduce slow-start (JobInProgress.java:879-881): classic reduces launch
        once ``mapred.reduce.slowstart.completed.maps`` of the maps are done and
        copy the rest as they complete (map ∥ shuffle); a collective reduce gang
        needs every map, as do reduces in child processes (their inputs are fixed
        at launch)."""
        if jip.maps_complete():
            return True
        if jip.collective_reduce and jip.split_job is not None and self.jt.prestage and \
                self._expect_ready(jip):
            # every map is launched, once, on a GPU: the gang can start now and
            # take each output as its kernels are enqueued ("expect" mode)
            jip.expect_mode = True
            return True
        if jip.collective_reduce or jip.split_job is not None or jip.reduce_in_child:
            return False
        return jip.maps_done >= jip.slowstart_maps

    @staticmethod
    def _expect_ready(jip) -> bool:
        if jip.expect_mode:
            return True
        if jip.pending_maps or jip.running_cpu:
            return False
        # cheap necessary condition first (this runs on every heartbeat until
        # it holds): one running GPU attempt per unfinished map
        if jip.running_gpu != len(jip.maps) - jip.maps_done:
            return False
        # the map scan once per state of those counts (this runs per tracker
        # per heartbeat for every staged job)
        sig = (jip.running_gpu, jip.maps_done, jip.jt.kill_epoch)
        if jip.__dict__.get("_expect_sig") == sig:
            return False
        for t in jip.maps:
            if t.successful is None:
                ra = t.running_attempts()
                if len(ra) != 1 or not ra[0].run_on_gpu:
                    jip._expect_sig = sig
                    return False
        return True

    def _speculate(self, tr, jip, gpu_free, now, actions):
        """Back up stragglers on fully idle GPUs (JobInProgress.java:2312's
        speculation, aimed at the slow CPU attempts of a hybrid job)."""
        for dev in sorted(gpu_free):
            if gpu_free[dev] < tr.gpu_capacity(dev) * self.queue_depth:
                continue  # only fully idle devices back up stragglers
            if self.job_limit(jip, "gpu") <= 0:
                break     # a backup is a running task too (maxRunningTasksPerJob)
            tip = self._straggler(jip, now)
            if tip is None:
                break
            actions.append(self.jt.launch(tr, tip, on_gpu=True, device=dev, speculative=True))
            gpu_free[dev] -= 1

    def _sampled_probing(self, jip) -> bool:
        return (self.policy in ("hybrid", "optional") and self.probe_fraction > 0 and
                jip.split_job is not None and jip.cpu_capable and jip.gpu_capable)

    def _needs_sampled_probe(self, jip) -> bool:
        if not self._sampled_probing(jip):
            return False
        cs = self.jt.cost_model.stats(jip.signature, False)
        return cs.n == 0 and not cs.running and cs.lower_bound == 0

    # -- policy hooks (FIFO by priority here; fair/capacity override) --------------------
    def begin_round(self, tr, total_cpu, total_gpu):
        pass

    def job_order(self, tr):
        return sorted(self.jt.job_queue, key=lambda j: (_prio(j.priority), j.submit_time))

    def slots_per_task(self, jip, kind) -> int:
        """Slots one task of ``jip`` occupies (memory matching; 1 by default)."""
        return 1

    def job_limit(self, jip, kind) -> int:
        """Most new tasks of ``kind`` (gpu/cpu/reduce) this job may take now."""
        return 1 << 30

    def _straggler(self, jip, now):
        """A running map whose only attempt is on a CPU (or has run > slowdown ×
        the GPU estimate) and has no backup yet."""
        # a scan finds the earliest time any running attempt can become a
        # straggler; until then (at most 0.25 s, so attempts launched since are
        # looked at soon) idle-GPU heartbeats skip the O(maps) scan
        if now < getattr(jip, "_no_straggler_until", 0.0):
            return None
        cm = self.jt.cost_model
        t_gpu, _ = cm.stats(jip.signature, True).estimate(now)
        next_check = now + 0.25
        for tip in jip.maps:
            if tip.is_complete():
                continue
            run = tip.running_attempts()
            if len(run) != 1:
                continue
            a = run[0]
            elapsed = now - a.start
            if self.policy == "stock":
                if elapsed > self.stock_lag:
                    return tip
                next_check = min(next_check, a.start + self.stock_lag)
                continue
            if t_gpu is None:
                continue
            limit = t_gpu * 2 if not a.run_on_gpu else self.speculate_after * t_gpu + 1.0
            if elapsed > limit:
                return tip
            next_check = min(next_check, a.start + limit)
        jip._no_straggler_until = next_check
        return None


def _attempts_in(acts) -> int:
    """Attempts a list of launch actions carries."""
    return sum(len(a["tasks"]) if a["type"] == "launch_batch" else 1 for a in acts
               if a["type"] in ("launch", "launch_batch"))


def _prio(p):
    return {"VERY_HIGH": 0, "HIGH": 1, "NORMAL": 2, "LOW": 3, "VERY_LOW": 4}.get(str(p).upper(), 2)
