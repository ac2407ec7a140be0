"""JobTracker: job queue, task bookkeeping, heartbeat-driven scheduling, failure handling.

Behaviour modelled on hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/
JobTracker.java (heartbeat :3308, processHeartbeat :3670, updateTaskStatuses
:4717, ExpireTrackers :440, lostTaskTracker :4811, FaultyTrackersInfo :814),
JobInProgress.java (initTasks :789, findNewMapTask :2371, completedTask :2673,
speculation :2312, finishedCPU/GPUMapTasks :114-115, 2780-2784) and
TaskInProgress.java (attempts, speculation, generateSingleReport :481).

Differences by design (SURVEY.md §2.1 bugs B1-B13):
* heartbeats are event-driven (a tracker calls in as soon as a slot frees)
  and the interval defaults to 100 ms, not a 3 s floor (B13);
* per-task CPU/GPU timings update an O(1) cost model on completion instead of
  being rebuilt from every TaskReport per heartbeat (B6);
* a lost tracker decrements only the counters of the tasks it really ran (B5);
* reports carry the placement of the *successful* attempt (G11);
* locality includes "split resident in this GPU's HBM".
"""
from __future__ import annotations

import collections
import itertools
import json
import logging
import math
import operator
import os
import shutil
import threading
import time

from ..utils.reflection import load_class, new_instance
from . import counters as C
from . import protocol as P
from .counters import Counters
from .ids import JobID, TaskAttemptID, TaskID
from .jobclient import FAILED, KILLED, PREP, RUNNING, SUCCEEDED, JobStatus, RunningJob
from .scheduler.costmodel import CostModel
from ..net.topology import DEFAULT_RACK, Topology
from ..utils.metrics import METRICS
from ..utils.trace import TRACE

# a job submitted with this key holds until that job succeeds (JobControl)
DEPENDS_KEY = "hbmr.job.depends.on"

log = logging.getLogger("hbmr.jobtracker")


def _listdir(d):
    try:
        return os.listdir(d)
    except OSError:
        return []


class TrackerInfo:
    def __init__(self, status: P.TaskTrackerStatus, now):
        self.name = status.tracker_name
        self.status = status
        self.last_seen = now
        self.running: set[str] = set()           # attempt ids
        self.running_gpu: dict[int, int] = {}    # device -> running GPU attempts
        self.running_cpu = 0
        self.running_reduce = 0
        self.cached: set[tuple] = set()          # (split_key, device)
        self.failures = 0
        self.blacklisted = False
        self.jobs_seen: set[str] = set()
        self.wake = False
        self.wake_seq = 0    # highest TaskTracker notification count seen by wakeup()
        # long-poll doorbell: set by wakeup() (no JobTracker lock needed, so a
        # tracker's completion thread never queues behind a heartbeat) and by
        # _kick() when new work may exist for every tracker
        self.bell = threading.Event()
        self.more = False    # the last assignment stopped at the per-heartbeat cap
        # responses carrying actions are numbered (under the JobTracker lock):
        # the tracker applies them in this order whichever thread receives them
        self.resp_seq = 0
        # the last numbered responses (seq, actions): resent when a tracker
        # lost a reply (JobTracker.resend; the reference resends its last
        # heartbeat response by responseId, JobTracker.java:3308-3437)
        self.sent: collections.deque = collections.deque(maxlen=32)
        self.rack = DEFAULT_RACK
        self.kills: set[str] = set()   # attempts to kill on the next heartbeat
        self.kill_epoch = -1           # JobTracker.kill_epoch this tracker was last scanned at
        self.cap_sig = None            # slot capacities last reported (JobTracker.cap_epoch)
        # running attempt ids by job id: a job ending scans only its own
        # attempts here for kills, not every running attempt of the tracker
        self.running_by_job: dict = {}
        self.extra_actions: list = []  # e.g. restart_gpu_worker, sent on the next heartbeat
        # attempts launched into extra_actions (a staged job's plan) and not yet
        # delivered: they count in ``running`` but the tracker knows nothing of them
        self.planned = 0
        # not worth ending a long-poll for (KillJobAction purges of finished
        # jobs): they ride on the next response the tracker gets anyway
        self.lazy_actions: list = []

    def gpu_devices(self):
        return [g["device"] for g in self.status.gpus]

    def gpu_capacity(self, dev):
        for g in self.status.gpus:
            if g["device"] == dev:
                return g["max_slots"]
        return 0


_PARTITION = operator.attrgetter("partition")
_LIVE = (P.RUNNING, P.COMMIT_PENDING)


class Attempt:
    """One attempt of a TIP.  The fields most attempts never change are class
    defaults (an instance sets only its own): a bulk launch builds one per map
    of every job on the JobTracker's critical path."""
    progress = 0.0
    finish = 0.0
    counters: dict = {}          # replaced (never mutated) when a report carries them
    output: dict = {}
    diagnostic = ""
    speculative = False
    device_time = 0.0
    _released = False
    profile_only = False         # a CPU profiling probe left running after its TIP won
    profile_fraction = 0.0       # >0: sampled probe, timed on this fraction of a split
    slots = 1                    # CPU / reduce slots held (memory matching)
    gated = False                # launched staged, behind another job's reduce
    tombstone = False            # its job was retired while it still ran
    state = P.RUNNING

    def __init__(self, aid, tip, tracker, run_on_gpu, device, speculative=False, start=None):
        self.aid = aid
        self.tip = tip
        self.tracker = tracker
        self.run_on_gpu = run_on_gpu
        self.device = device
        if speculative:
            self.speculative = True
        self.start = time.time() if start is None else start


class TaskInProgress:
    """A task (map or reduce) of a job and its attempts.  As with Attempt,
    the fields most TIPs never change are class defaults: init_tasks builds
    one per split of every job."""
    pinned_tracker = None
    next_attempt = 0
    failures = 0
    failed_trackers: frozenset | set = frozenset()   # a set once an attempt fails
    successful = None            # the winning Attempt
    commit_granted = None
    killed = False

    def __init__(self, job, tid: TaskID, split=None, partition=0, pinned_tracker=None,
                 aid_prefix=None):
        self.job = job
        self.tid = tid
        self.split = split
        self.partition = partition
        if pinned_tracker is not None:
            self.pinned_tracker = pinned_tracker
        self.attempts: dict[str, Attempt] = {}
        self._aid_prefix = aid_prefix or ("attempt" + tid._s[4:] + "_")

    @property
    def is_map(self):
        return self.tid.is_map

    def is_complete(self):
        return self.successful is not None

    def running_attempts(self):
        at = self.attempts
        if len(at) == 1:                 # the common case: one attempt
            for a in at.values():
                return [a] if a.state in _LIVE else []
        return [a for a in at.values() if a.state in _LIVE]

    def is_running(self):
        return bool(self.running_attempts())

    def new_attempt_id(self) -> TaskAttemptID:
        aid = TaskAttemptID(self.tid, self.next_attempt)
        self.next_attempt += 1
        return aid

    def locations(self):
        return (self.split or {}).get("locations", []) if isinstance(self.split, dict) else []

    def split_key(self):
        return (self.split or {}).get("key") if isinstance(self.split, dict) else None

    def report(self):
        """TaskReport of the successful attempt (else the latest one), with its
        placement (fixes G11, which tagged the first attempt)."""
        from .local_runner import TaskReport
        a = self.successful
        if a is None and self.attempts:
            a = max(self.attempts.values(), key=lambda x: x.start)
        if a is None:
            return TaskReport(self.tid, 0.0, P.UNASSIGNED, 0.0, 0.0, Counters())
        state = P.SUCCEEDED if self.successful else a.state
        return TaskReport(self.tid, 1.0 if self.successful else a.progress, state, a.start,
                          a.finish, Counters.from_dict(a.counters), a.run_on_gpu, a.device,
                          a.tracker)


class JobInProgress:
    def __init__(self, jt, job_id: JobID, conf):
        self.jt = jt
        self.fold_lock = threading.RLock()   # counters() holds it around fold_counters
        self.acc_lock = threading.Lock()     # loc_counts / pending_counters writers + swap
        self.job_id = job_id
        self.conf = conf
        self.status = JobStatus(job_id, PREP)
        self.counters = Counters()
        self.maps: list[TaskInProgress] = []
        self.reduces: list[TaskInProgress] = []
        self.done = threading.Event()
        self.split_job = None
        self.collective_reduce = False
        self.priority = conf.get("mapred.job.priority", "NORMAL")
        self.submit_time = time.time()
        self.launch_time = 0.0
        self.release_time = 0.0     # a dependent job: when its dependency succeeded
        self.t_first_map = 0.0       # first map attempt launched
        self.t_maps_done = 0.0       # last map completed
        self.t_first_reduce = 0.0    # first reduce attempt launched
        self.maps_done = 0
        self.reduces_done = 0
        self.running_cpu = 0         # running CPU map attempts (O(1) for the scheduler)
        self.running_gpu = 0
        self.pending_counters: list = []
        self._loc_index: dict = {}
        self.reduce_by_tracker: dict = {}   # collective gang: tracker -> its pinned reduce
        self._front: dict = {}          # re-queued TIPs (add_pending front) -> order key
        self._front_seq = 0
        self.finished_cpu_maps = 0
        self.finished_gpu_maps = 0
        self.completion_events: list = []     # (map TaskID, attempt id, output)
        # notified when completion events are added or the job ends: reduces
        # long-poll map_completion_events on it instead of sleeping
        self.events_cond = threading.Condition(threading.Lock())
        self.pending_maps: dict = {}   # TIP -> None: not yet started, insertion (FIFO) order
        self.by_split_key: dict = {}
        self.signature = conf.get("hbmr.job.signature") or self._signature(conf)
        self.gpu_capable = conf.is_gpu_capable()
        self.cpu_capable = conf.get_boolean("hbmr.job.cpu.capable", True)
        self.speculative = conf.get_map_speculative_execution()
        self.max_map_attempts = conf.get_max_map_attempts()
        self.max_reduce_attempts = conf.get_max_reduce_attempts()
        self.result = None
        self.conf_dict = conf.to_dict()
        from .child import use_child_process
        self.reduce_in_child = use_child_process(conf)
        self.slowstart = conf.get_float("mapred.reduce.slowstart.completed.maps", 0.05)
        self.slowstart_maps = 0
        # pre-staging (hbmr/gpu/gates.py): the job this one's GPU maps are
        # gated on while it waits for it, its staged launches per (tracker,
        # device), a finish deferred until that job succeeded, and whether its
        # collective reduce was launched before its maps finished ("expect")
        self.staged_on: str | None = None
        self.staged_launched: dict = {}
        # map TIPs by the trackers their attempts were launched on: a collective
        # reduce collects its tracker's outputs from here, not from every map
        self.launched_on: dict = {}
        self.loc_counts = [0, 0, 0]     # HBM-local, data-local, rack-local maps
        self.pending_finish = False
        self.expect_mode = False
        self.probe_aids: list = []      # sampled CPU probes (attempts of no TIP)
        self.retired = None             # its summary once its task state is dropped

    @staticmethod
    def _signature(conf):
        return "|".join(str(conf.get(k, "")) for k in (
            "hbmr.splitjob.class", "mapred.mapper.class", "hadoop.pipes.executable",
            "hadoop.pipes.gpu.executable", "mapred.input.format.class", "hbmr.split.size"))

    def committer(self):
        cls = self.conf.get_output_committer()
        from .committer import FileOutputCommitter
        return cls() if isinstance(cls, type) else (cls or FileOutputCommitter())

    # -- init ---------------------------------------------------------------------
    def init_tasks(self):
        conf = self.conf
        sj_cls = conf.get("hbmr.splitjob.class")
        trackers = self.jt.tracker_names()
        if sj_cls:
            self.split_job = new_instance(sj_cls, conf)
            splits = self.split_job.get_splits(conf, trackers)
            self.collective_reduce = bool(getattr(self.split_job, "collective_reduce", True))
            from ..gpu.splitjob import SplitJob
            if type(self.split_job).map_gpu is not SplitJob.map_gpu:
                self.gpu_capable = True   # the split job has a device map
            # a split list memoised across iteration jobs keeps its dicts too
            split_dicts = [s.__dict__.get("_wire") or s.__dict__.setdefault("_wire", s.to_dict())
                           for s in splits]
        else:
            # job setup (the reference's setup task: FileOutputCommitter.setupJob)
            self.committer().setup_job(conf)
            informat = new_instance(conf.get_input_format(), conf)
            splits = informat.getSplits(conf, conf.get_num_map_tasks())
            split_dicts = [{"kind": "class", "cls": f"{type(s).__module__}:{type(s).__qualname__}",
                            "data": s.serialize().hex(),
                            "locations": list(s.getLocations() or []),
                            "length": s.getLength()} for s in splits]
        jid = self.job_id
        tpre = f"task_{jid.jt}_{jid.id:04d}_m_"
        apre = f"attempt_{jid.jt}_{jid.id:04d}_m_"
        maps = self.maps = [TaskInProgress(self, TaskID(jid, True, i, tpre + f"{i:06d}"),
                                           split=sd, partition=i,
                                           aid_prefix=apre + f"{i:06d}_")
                            for i, sd in enumerate(split_dicts)]
        self.pending_maps = dict.fromkeys(maps)
        self.by_split_key = {sd["key"]: tip for tip, sd in zip(maps, split_dicts)
                             if sd.get("key")}
        if self.collective_reduce and self.split_job is not None:
            # one pinned reduce per tracker: the collective (RCCL) reduce gang
            nred = len(trackers) if getattr(self.split_job, "needs_reduce", True) else 0
            for r in range(nred):
                self.reduces.append(TaskInProgress(self, TaskID(self.job_id, False, r),
                                                   partition=r, pinned_tracker=trackers[r]))
                self.reduce_by_tracker[trackers[r]] = self.reduces[-1]
        else:
            for r in range(conf.get_num_reduce_tasks()):
                self.reduces.append(TaskInProgress(self, TaskID(self.job_id, False, r),
                                                   partition=r))
        self.slowstart_maps = math.ceil(min(1.0, max(0.0, self.slowstart)) * len(self.maps))
        self.status.state = RUNNING
        self.launch_time = time.time()
        self.jt.history.log("JOB_INITED", job=str(self.job_id), maps=len(self.maps),
                            reduces=len(self.reduces), signature=self.signature)

    # -- scheduling helpers ----------------------------------------------------------------
    def pending_map_count(self):
        return len(self.pending_maps)

    def running_maps(self, on_gpu=None):
        if on_gpu is None:
            return self.running_cpu + self.running_gpu
        return self.running_gpu if on_gpu else self.running_cpu

    def maps_complete(self):
        return self.maps_done == len(self.maps)

    def fold_counters(self) -> Counters:
        """Merge the counters of newly succeeded attempts (and the locality
        levels counted by obtain_map) into the job's.  Under fold_lock: a
        client reading counters while the job-finish path folds must not
        return before the batch the other thread swapped out is merged."""
        with self.fold_lock:
            return self._fold_counters_locked()

    def add_counters(self, d):
        """A succeeded attempt's counters, folded lazily (fold_counters)."""
        with self.acc_lock:
            self.pending_counters.append(d)

    def _fold_counters_locked(self) -> Counters:
        # swap both accumulators under acc_lock (the lock their writers take),
        # merge outside it: no increment or append can land in a swapped-out one
        with self.acc_lock:
            lc, self.loc_counts = self.loc_counts, [0, 0, 0]
            pend, self.pending_counters = self.pending_counters, []
        if any(lc):
            hbm, data, rack = lc
            for name, v in (("HBM_LOCAL_MAPS", hbm), ("DATA_LOCAL_MAPS", data),
                            ("RACK_LOCAL_MAPS", rack)):
                if v:
                    self.counters.incr(C.JOB_GROUP, name, v)
        if pend:
            self.counters.incr_dicts(pend)
        return self.counters

    def _index(self, tracker: TrackerInfo, on_gpu, device):
        """Per-(tracker, device) queues of pending TIPs by locality level, built
        once per job and consumed with lazy deletion: O(1) amortised per
        assignment instead of the reference's scan of every TIP.  A build
        visits only what is local to the tracker — its HBM-resident split keys
        (by_split_key) and the job's TIPs naming it (_by_location) — not every
        pending TIP, so a job's index costs O(maps) over all trackers, not
        O(maps x trackers)."""
        key = (tracker.name, device if on_gpu else None)
        idx = self._loc_index.get(key)
        if idx is None or idx[4] != len(tracker.cached):
            pend = self.pending_maps
            byk = self.by_split_key
            lv0, lv1 = [], []
            if byk and tracker.cached:
                # one pass: a split cached on this device is level 0, on
                # another of the tracker's devices level 1 (once: a split may
                # be cached on several)
                dev0 = device if on_gpu else None
                for k, d in tracker.cached:
                    tip = byk.get(k)
                    if tip is not None and tip in pend:
                        (lv0 if d == dev0 else lv1).append(tip)
                if len(tracker.status.gpus) > 1 or not on_gpu:
                    s0 = set(lv0)
                    lv1 = [t for t in dict.fromkeys(lv1) if t not in s0]
            seen = set(lv0)
            seen.update(lv1)
            # stacks popped from the end, in pending order: re-queued TIPs
            # (failed / lost outputs, add_pending(front=True)) first, newest
            # first, then map index order (findNewMapTask takes failed maps first)
            front = self._front
            order = (lambda lv: sorted(lv, key=_PARTITION, reverse=True)) if not front else \
                (lambda lv: sorted(lv, key=lambda t: front.get(t, t.partition),  # noqa: E731
                                   reverse=True))
            # level 2 (node-local by split location) is built on first use: on
            # one host every split names this node, so building it eagerly
            # visited every map of the job per (tracker, device) even when the
            # HBM-resident level 0 serves them all
            idx = [order(lv0), order(lv1), None, None, len(tracker.cached), seen]
            self._loc_index[key] = idx
        return idx

    def _node_level(self, tracker, idx):
        if idx[2] is None:
            pend = self.pending_maps
            seen = idx[5]
            lv2 = []
            byloc = self._by_location()
            for loc in (tracker.name, tracker.status.host):
                for tip in byloc.get(loc, ()):
                    if tip in pend and tip not in seen:
                        lv2.append(tip)
                        seen.add(tip)
            front = self._front
            idx[2] = sorted(lv2, key=(lambda t: front.get(t, t.partition)) if front else _PARTITION,
                            reverse=True)
        return idx[2]

    def _by_location(self):
        """location (tracker name / host) -> the job's map TIPs naming it."""
        bl = self.__dict__.get("_byloc")
        if bl is None:
            bl = {}
            for tip in self.maps:
                sp = tip.split
                if sp.__class__ is dict:
                    for loc in sp.get("locations") or ():
                        got = bl.get(loc)
                        if got is None:
                            bl[loc] = [tip]
                        else:
                            got.append(tip)
            self._byloc = bl
        return bl

    def _rack_level(self, tracker, idx):
        if idx[3] is None:
            topo = self.jt.topology
            seen = idx[5]
            rest = [t for t in self.pending_maps if t not in seen and t.locations()]
            idx[3] = [t for t in rest if tracker.rack in topo.resolve(t.locations())][::-1]
            idx[5] = None
        return idx[3]

    def obtain_map(self, tracker: TrackerInfo, on_gpu: bool, device: int, allow_nonlocal=True):
        """findNewMapTask with locality levels: 0 split cached in this device's
        HBM > 1 cached elsewhere on this tracker > 2 node-local (split locations)
        > 3 rack-local > 4 any.  Levels ≥ 3 need ``allow_nonlocal`` (delay
        scheduling): for a GPU the split must be re-materialised either way."""
        if not self.pending_maps:
            return None
        ntr = len(self.jt.trackers)
        multi = ntr > 1

        def avoid(tip):
            # a TIP avoids trackers it failed on, unless it failed on all of them
            # (JobInProgress.findNewMapTask: hasFailedOnMachine vs numUniqueHosts)
            return multi and tracker.name in tip.failed_trackers and \
                len(tip.failed_trackers) < ntr
        idx = self._index(tracker, on_gpu, device)
        for level in (0, 1, 2, 3):
            if level == 3 and not allow_nonlocal:
                return None
            stack = idx[level] if level < 2 else self._node_level(tracker, idx) if level == 2 \
                else self._rack_level(tracker, idx)
            while stack:
                tip = stack.pop()
                if tip in self.pending_maps and not avoid(tip):
                    self._take(tip)
                    self._count_locality(level)
                    return tip, level
        for tip in self.pending_maps:
            if avoid(tip):
                continue
            self._take(tip)
            self._count_locality(4)
            return tip, 4
        return None

    def obtain_maps(self, tracker: TrackerInfo, on_gpu: bool, device: int, n: int,
                    allow_nonlocal=True):
        """Up to ``n`` maps for one device in one call — obtain_map's levels
        and order, with the index looked up once and the stacks drained in a
        loop (a bulk launch takes a device's whole queue depth at once)."""
        out = []
        pend = self.pending_maps
        if n <= 0 or not pend:
            return out
        ntr = len(self.jt.trackers)
        multi = ntr > 1
        name = tracker.name
        idx = self._index(tracker, on_gpu, device)
        for level in (0, 1, 2, 3):
            if level == 3 and not allow_nonlocal:
                break
            stack = idx[level] if level < 2 else self._node_level(tracker, idx) if level == 2 \
                else self._rack_level(tracker, idx)
            front = self._front
            while stack and len(out) < n:
                tip = stack.pop()
                if tip in pend and not (multi and tip.failed_trackers and
                                        name in tip.failed_trackers and
                                        len(tip.failed_trackers) < ntr):
                    del pend[tip]
                    if front:
                        front.pop(tip, None)
                    out.append((tip, level))
            if len(out) >= n:
                break
        else:
            for tip in list(pend):
                if len(out) >= n:
                    break
                if multi and name in tip.failed_trackers and len(tip.failed_trackers) < ntr:
                    continue
                self._take(tip)
                out.append((tip, 4))
        if out:
            counts = [0, 0, 0]
            for _t, lv in out:
                if lv == 0:
                    counts[0] += 1
                if lv <= 2:
                    counts[1] += 1
                elif lv == 3:
                    counts[2] += 1
            with self.acc_lock:
                lc = self.loc_counts
                lc[0] += counts[0]
                lc[1] += counts[1]
                lc[2] += counts[2]
        return out

    def locality_possible(self) -> bool:
        """Does any split name a live tracker (by tracker name, host or rack)?
        If not, waiting for a local slot (delay scheduling) cannot help."""
        live = self.jt.trackers
        key = len(live)
        if getattr(self, "_loc_possible", None) is not None and self._loc_possible[0] == key:
            return self._loc_possible[1]
        names = set(live) | {t.status.host for t in live.values()}
        ok = any(loc in names for tip in self.maps for loc in tip.locations()) or \
            any(tip.split_key() for tip in self.maps)   # HBM-resident splits
        self._loc_possible = (key, ok)
        return ok

    def _count_locality(self, level):
        # JobInProgress.Counter DATA_LOCAL_MAPS / RACK_LOCAL_MAPS (+ hbmr's
        # HBM-resident level): plain ints, folded into the counters on read
        with self.acc_lock:
            lc = self.loc_counts
            if level == 0:
                lc[0] += 1
            if level <= 2:
                lc[1] += 1
            elif level == 3:
                lc[2] += 1

    def _take(self, tip):
        del self.pending_maps[tip]
        if self._front:
            self._front.pop(tip, None)

    def add_pending(self, tip, front=False):
        if tip in self.pending_maps:
            return
        if front:
            self.pending_maps = {tip: None, **self.pending_maps}
            self._front_seq -= 1
            self._front[tip] = self._front_seq      # (negative: before every index)
        else:
            self.pending_maps[tip] = None
        self._loc_index.clear()

    def completed(self):
        return self.status.is_complete()

    def maps_per_tracker(self) -> dict:
        """Succeeded maps per tracker (kept past retirement)."""
        if self.retired is not None:
            return dict(self.retired["maps_per_tracker"])
        per = {}
        for t in self.maps:
            if t.successful is not None:
                per[t.successful.tracker] = per.get(t.successful.tracker, 0) + 1
        return per

    def retire(self):
        """Drop a completed job's task state (JobTracker._retire_jobs); its
        attempt ids go to ``retired_aids`` for the JobTracker's index."""
        if self.retired is not None:
            return
        self.retired = {"maps_per_tracker": self.maps_per_tracker(),
                        "maps": len(self.maps), "reduces": len(self.reduces)}
        aids = list(self.probe_aids)
        for tip in self.maps:
            aids.extend(tip.attempts)
        for tip in self.reduces:
            aids.extend(tip.attempts)
        self.retired_aids = aids
        self.maps, self.reduces = [], []
        self.pending_maps, self.by_split_key, self.reduce_by_tracker = {}, {}, {}
        self.completion_events, self.launched_on, self._loc_index = [], {}, {}
        self.staged_launched, self._front, self.probe_aids = {}, {}, []
        self.__dict__.pop("_byloc", None)

    def timeline(self) -> dict:
        """Phase breakdown in seconds (submit → first map launch → last map done
        → first reduce launch → finish); a dependent job counts from its release."""
        st = self.status
        t0 = self.release_time or self.submit_time
        rel = lambda t: round(t - t0, 6) if t else None  # noqa: E731
        return {"first_map": rel(self.t_first_map), "maps_done": rel(self.t_maps_done),
                "first_reduce": rel(self.t_first_reduce), "finish": rel(st.finish_time)}


class JobHistory:
    """Job history event log (JobHistory.java) as JSON lines; the hbmr twist is
    that every map attempt records run_on_gpu / device (the fork's history did not)."""

    def __init__(self, path=None):
        self.path = path
        self._lock = threading.Lock()
        self.events: list[dict] = []
        self.max_events = 200_000

    def log(self, event, **kw):
        kw["ts"] = time.time()
        kw["event"] = event
        if len(self.events) < self.max_events:
            self.events.append(kw)     # list.append is atomic under the GIL
        if self.path:
            import json
            with self._lock, open(self.path, "a") as f:
                f.write(json.dumps(kw) + "\n")


class _JTJobHandle:
    """RunningJob backend for jobs submitted to an in-process JobTracker."""

    def __init__(self, jip: JobInProgress):
        self.jip = jip

    def status(self):
        return self.jip.status

    def counters(self):
        # folding needs no JobTracker lock (pending_counters is swapped
        # atomically and Counters locks itself): a client reading counters must
        # not stall every tracker's heartbeat
        with self.jip.fold_lock:
            return self.jip.fold_counters()

    def wait(self, timeout=None):
        return self.jip.done.wait(timeout)

    def kill(self):
        self.jip.jt.kill_job(self.jip.job_id)

    def task_reports(self, is_map=True):
        return [t.report() for t in (self.jip.maps if is_map else self.jip.reduces)]

    @property
    def result(self):
        return self.jip.result


class JobTracker:
    def __init__(self, conf, name=None):
        self.conf = conf
        self.name = name or time.strftime("%Y%m%d%H%M")
        self.lock = threading.RLock()
        self.cv = threading.Condition(self.lock)
        self.jobs: dict[str, JobInProgress] = {}
        from ..security import JobTokenSecretManager
        self.job_tokens = JobTokenSecretManager()
        self.job_queue: list[JobInProgress] = []
        self.waiting: dict[str, list] = {}   # job id -> dependent jobs held for it
        # dependent jobs whose GPU maps may already be launched, gated on the
        # job they wait for (hbmr/gpu/gates.py); chains up to prestage.depth
        self.staged: list[JobInProgress] = []
        self.kill_epoch = 0    # bumped when attempts may have become killable
        # bumped when the cluster's slot capacity may have changed (a tracker
        # joined / was lost / blacklisted, or reported other slot counts): the
        # scheduler's capacity totals are recomputed only then, not per call
        self.cap_epoch = 0
        self.prestage = conf.get_boolean("hbmr.job.prestage", True)
        self.prestage_depth = max(1, conf.get_int("hbmr.job.prestage.depth", 2))
        # trackers get their new work back in the report of a finished task
        # (TaskTracker.report_assign, the same cluster key)
        self.report_assign_expected = conf.get_boolean("hbmr.tracker.report.assign", True)
        # a staged split job is placed on every tracker at once (maps + reduce
        # gang member per tracker: HybridScheduler.plan_staged)
        self.plan_staged = conf.get_boolean("hbmr.scheduler.plan.staged", True)
        self.trackers: dict[str, TrackerInfo] = {}
        self.attempt_index: dict[str, Attempt] = {}
        self.cost_model = CostModel(conf.get_float("hbmr.costmodel.ewma.alpha", 0.3))
        self.topology = Topology(conf)
        sched_cls = conf.get("mapred.jobtracker.taskScheduler",
                             "hbmr.mapred.scheduler.hybrid:HybridTaskScheduler")
        self.scheduler = load_class(sched_cls)(self, conf)
        self.history = JobHistory(conf.get("hbmr.history.file"))
        self.heartbeat_interval = conf.get_int("hbmr.heartbeat.interval.ms", 100) / 1000.0
        self.tracker_expiry = conf.get_int("mapred.tasktracker.expiry.interval", 600000) / 1000.0
        self.max_tracker_failures = conf.get_int("mapred.max.tracker.failures", 4)
        self._seq = itertools.count(1)
        self._expire_thread = None
        self._stop = threading.Event()
        self.listeners = []
        # job retirement (JobTracker.RetireJobs, mapred.jobtracker.completeuserjobs
        # .maximum): the newest completed jobs keep their task state; older ones
        # drop it (TIPs, attempts, completion events: a long K-Means run adds
        # ~1,500 objects per iteration job that every full collection would
        # walk and every attempt lookup would index), keeping status, counters,
        # result and a per-tracker map summary; beyond hbmr.jobtracker.retired
        # .jobs.maximum they are forgotten
        self.keep_completed = max(1, conf.get_int("mapred.jobtracker.completeuserjobs.maximum",
                                                  100))
        self.keep_retired = max(0, conf.get_int("hbmr.jobtracker.retired.jobs.maximum", 1000))
        self._completed: collections.deque = collections.deque()
        self._retired: collections.deque = collections.deque()
        self.start_time = time.time()
        self.system_dir = conf.get("mapred.system.dir")
        # job files exist for restart recovery only: without it a submit does
        # no file-system work on the job's critical path
        self.recover = conf.get_boolean("mapred.jobtracker.restart.recover", False)
        self.worker_generation = 0     # GPU worker gang (communicator) generation
        self.restart_count = 0
        self._to_recover: list[str] = []
        self._recover_trackers = 0
        self._recover_deadline = 0.0
        if self.system_dir:
            info = self._load_info()
            if info or any(n.startswith("job_") for n in _listdir(self.system_dir)):
                self.restart_count = int(info.get("restart_count", 0)) + 1
            if conf.get_boolean("mapred.jobtracker.restart.recover", False):
                self._to_recover = sorted(n for n in _listdir(self.system_dir)
                                          if n.startswith("job_") and os.path.exists(
                                              os.path.join(self.system_dir, n, "job.json")))
                self._recover_trackers = int(info.get("trackers", 0))
                self._recover_deadline = self.start_time + conf.get_int(
                    "hbmr.jobtracker.recovery.grace.ms", 3000) / 1000.0
            else:
                for n in _listdir(self.system_dir):   # stale job files of a previous run
                    if n.startswith("job_"):
                        shutil.rmtree(os.path.join(self.system_dir, n), ignore_errors=True)
            self._save_info()
        METRICS.register_gauges(self._gauges)

    def _gauges(self):
        """Sampled at scrape time (JobTrackerMetricsSource's gauges)."""
        with self.lock:
            trs = list(self.trackers.values())
            yield "hbmr_trackers", {}, len(trs)
            yield "hbmr_trackers_blacklisted", {}, sum(1 for t in trs if t.blacklisted)
            yield "hbmr_running_maps", {"where": "cpu"}, sum(t.running_cpu for t in trs)
            yield "hbmr_running_maps", {"where": "gpu"}, sum(sum(t.running_gpu.values())
                                                             for t in trs)
            yield "hbmr_running_reduces", {}, sum(t.running_reduce for t in trs)
            yield "hbmr_cpu_map_slots", {}, sum(t.status.max_cpu_map_slots for t in trs)
            yield "hbmr_gpu_slots", {}, sum(g["max_slots"] for t in trs for g in t.status.gpus)
            yield "hbmr_jobs_running", {}, len(self.job_queue)
            yield "hbmr_hbm_resident_splits", {}, sum(len(t.cached) for t in trs)
    # -- trackers -------------------------------------------------------------------
    def tracker_names(self):
        with self.lock:
            return sorted(self.trackers, key=lambda n: (self.trackers[n].status.rank, n))

    def wait_for_trackers(self, n, timeout=60.0):
        t0 = time.time()
        while time.time() - t0 < timeout:
            with self.lock:
                if len(self.trackers) >= n:
                    return True
            time.sleep(0.005)
        return False

    def start_expiry_thread(self):
        if self._expire_thread is None:
            self._expire_thread = threading.Thread(target=self._expire_loop, daemon=True,
                                                   name="ExpireTrackers")
            self._expire_thread.start()

    def _expire_loop(self):
        while not self._stop.wait(min(1.0, self.tracker_expiry / 4)):
            now = time.time()
            with self.lock:
                for name, tr in list(self.trackers.items()):
                    if now - tr.last_seen > self.tracker_expiry:
                        self.lost_tracker(name, "expired")

    def lost_tracker(self, name, why="lost"):
        """lostTaskTracker (JobTracker.java:4811): fail its running attempts and
        re-execute its completed maps whose output lived on it."""
        with self.lock:
            tr = self.trackers.pop(name, None)
            self.cap_epoch += 1
            if tr is None:
                return
            log.warning("tracker %s %s", name, why)
            self.history.log("TRACKER_LOST", tracker=name, why=why)
            for aid in list(tr.running):
                a = self.attempt_index.get(aid)
                if a is not None:
                    self._attempt_failed(a, f"tracker {name} {why}", killed=True)
            for jip in self.jobs.values():
                if jip.completed():
                    continue
                for tip in jip.maps:
                    a = tip.successful
                    if a is not None and a.tracker == name and jip.reduces:
                        # its map output is gone with the tracker
                        tip.successful = None
                        jip.maps_done -= 1
                        jip.t_maps_done = 0.0
                        if a.run_on_gpu:
                            jip.finished_gpu_maps -= 1
                        else:
                            jip.finished_cpu_maps -= 1
                        jip.add_pending(tip)

    # -- jobs -----------------------------------------------------------------------
    def new_job_id(self):
        while True:
            jid = JobID(self.name, next(self._seq))
            if str(jid) not in self.jobs:   # recovered jobs keep their ids
                return jid

    # -- restart recovery ---------------------------------------------------------------
    # RecoveryManager (JobTracker.java:1203, mapred.jobtracker.restart.recover :2394):
    # every submitted job's conf is kept in mapred.system.dir/<jobid>/job.json until
    # the job finishes (JobInProgress.garbageCollect deletes it).  A JobTracker that
    # starts with recovery on re-submits each job it finds there, under its old id,
    # once the trackers that were registered before the restart have re-joined (or
    # after hbmr.jobtracker.recovery.grace.ms).  Recovery is job-level: the attempts
    # of a recovered job re-run (a restarted tracker has dropped its in-flight
    # attempts and map outputs anyway; committed outputs are idempotent renames).
    def _sysdir(self, jid=None):
        if not self.system_dir:
            return None
        return os.path.join(self.system_dir, str(jid)) if jid is not None else self.system_dir

    def _persist_job(self, jid, conf):
        d = self._sysdir(jid) if self.recover else None
        if d is None:
            return
        os.makedirs(d, exist_ok=True)
        tmp = os.path.join(d, f"job.json.{os.getpid()}.{threading.get_ident()}.tmp")
        with open(tmp, "w") as f:
            json.dump({"conf": conf.to_dict(), "submit_time": time.time()}, f)
        os.replace(tmp, os.path.join(d, "job.json"))

    def _forget_job(self, jid):
        d = self._sysdir(jid) if self.recover else None
        if d is not None:
            shutil.rmtree(d, ignore_errors=True)

    def _save_info(self):
        d = self._sysdir()
        if d is None:
            return
        os.makedirs(d, exist_ok=True)
        # a temp name of this writer's own: two JobTrackers (processes, or the
        # heartbeat threads of one) sharing a system dir must not rename each
        # other's file away
        tmp = os.path.join(d, f"jobtracker.json.{os.getpid()}.{threading.get_ident()}.tmp")
        with open(tmp, "w") as f:
            json.dump({"restart_count": self.restart_count, "trackers": len(self.trackers)}, f)
        os.replace(tmp, os.path.join(d, "jobtracker.json"))

    def _load_info(self):
        d = self._sysdir()
        try:
            with open(os.path.join(d, "jobtracker.json")) as f:
                return json.load(f)
        except (OSError, ValueError, TypeError):
            return {}

    def _maybe_recover(self, now):
        if not self._to_recover:
            return
        if len(self.trackers) < self._recover_trackers and now < self._recover_deadline:
            return
        todo, self._to_recover = self._to_recover, []
        for jid_s in todo:
            try:
                with open(os.path.join(self._sysdir(jid_s), "job.json")) as f:
                    doc = json.load(f)
            except (OSError, ValueError) as e:
                log.warning("cannot recover %s: %s", jid_s, e)
                continue
            from .jobconf import JobConf
            conf = JobConf()
            for k, v in doc["conf"].items():
                conf.set(k, v)
            self.history.log("JOB_RECOVERED", job=jid_s, restart=self.restart_count)
            METRICS.inc("hbmr_jobs_recovered_total", help="jobs re-submitted after a JT restart")
            self.submit_job(conf, job_id=JobID.for_name(jid_s))
        log.info("recovered %d job(s) after restart %d", len(todo), self.restart_count)

    def submit_job(self, conf, job_id=None) -> RunningJob:
        if TRACE.on:
            TRACE.instant("jt.submit")
        METRICS.inc("hbmr_jobs_submitted_total", help="jobs submitted")
        from .. import security as SEC
        if SEC.acls_enabled(self.conf) and job_id is None:
            ugi = SEC.UserGroupInformation.get_current_user()
            SEC.QueueManager(self.conf).check_submit(conf.get("mapred.job.queue.name",
                                                              "default"), ugi)
            conf.set("user.name", ugi.user)   # the authenticated submitter owns the job
        jid = job_id or self.new_job_id()
        conf.set("mapred.job.id", str(jid))
        self.job_tokens.add_job(jid)
        self._persist_job(jid, conf)
        jip = JobInProgress(self, jid, conf)
        if TRACE.on:
            TRACE.instant("jt.jip_created")
        too_big = self._memory_violation(conf)
        init_error = None
        if not too_big:
            self.history.log("JOB_SUBMITTED", job=str(jid), name=conf.get_job_name(),
                             user=conf.get_user())
            # splits, TIPs and job setup outside the JobTracker lock (the job
            # is not visible yet): heartbeats are not held up by a submission
            try:
                jip.init_tasks()
                if TRACE.on:
                    TRACE.instant("jt.tasks_inited", maps=len(jip.maps))
            except Exception as e:  # noqa: BLE001
                log.exception("job init failed")
                init_error = e
        with self.lock:
            self.jobs[str(jid)] = jip
            if too_big:
                self._finish_job(jip, FAILED, too_big)
                return RunningJob(jid, _JTJobHandle(jip), conf)
            if init_error is not None:
                e = init_error
                self._finish_job(jip, FAILED, f"init failed: {type(e).__name__}: {e}")
                return RunningJob(jid, _JTJobHandle(jip), conf)
            check = getattr(self.scheduler, "check_submission", None)
            refused = check(jip) if check is not None else None
            if refused:
                # the scheduler's job-submission limits (capacity scheduler)
                self._finish_job(jip, FAILED, refused)
                return RunningJob(jid, _JTJobHandle(jip), conf)
            dep = conf.get(DEPENDS_KEY)
            dj = self.jobs.get(dep) if dep else None
            if dep and dj is None:
                # a typo, or a job this JobTracker never saw (retired, or finished
                # before a restart): nothing to wait for, but say so
                log.warning("job %s depends on unknown job %s: scheduling it now", jid, dep)
                self.history.log("JOB_DEPENDENCY_UNKNOWN", job=str(jid), depends_on=dep)
            if dj is not None and not dj.completed():
                # a dependent job (JobControl's ControlledJob): initialised now,
                # scheduled the moment the job it depends on succeeds — and,
                # when both are collective split jobs, staged at once
                jip.status.state = PREP
                self.waiting.setdefault(dep, []).append(jip)
                self._maybe_stage(jip, dj)
                return RunningJob(jid, _JTJobHandle(jip), conf)
            if dj is not None and dj.status.state != SUCCEEDED:
                self._finish_job(jip, FAILED, f"job {dep} it depends on {dj.status.state}")
                return RunningJob(jid, _JTJobHandle(jip), conf)
            self.job_queue.append(jip)
            if not jip.maps and not jip.reduces:
                self._finish_job(jip, SUCCEEDED)
            self._kick()
        for cb in self.listeners:
            cb("submitted", jip)
        return RunningJob(jid, _JTJobHandle(jip), conf)

    def _stage_depth(self, jip) -> int:
        d = 0
        while jip is not None and jip.staged_on is not None:
            d += 1
            jip = self.jobs.get(jip.staged_on)
        return d

    def _maybe_stage(self, w: JobInProgress, j: JobInProgress):
        """Stage dependent job ``w`` on ``j`` (running, or staged itself): its
        GPU map attempts may be launched now, each gated on j's collective
        reduce on its tracker (the device runs w's maps right after j's reduce
        result, with no JobTracker round trip in between); w still completes
        only after j succeeded.  Both must be collective split jobs."""
        if not self.prestage or w.staged_on is not None or w.completed() or j.completed():
            return
        if w.split_job is None or not w.collective_reduce or not w.gpu_capable or \
                j.split_job is None or not j.collective_reduce:
            return
        if j.status.state != RUNNING and j.staged_on is None:
            return          # j itself still waits, unstaged
        if self._stage_depth(j) + 1 > self.prestage_depth:
            return
        w.staged_on = str(j.job_id)
        self.staged.append(w)
        self.history.log("JOB_STAGED", job=str(w.job_id), gate=str(j.job_id))
        plan = getattr(self.scheduler, "plan_staged", None)
        if plan is not None and self.plan_staged:
            plan(w)
        # the new job's maps cannot run before j's reduce has completed on
        # their tracker, and a tracker with work running reports each
        # completion (JobTracker.report assigns), which carries the plan: only
        # the trackers with nothing delivered running are rung — they have no
        # report coming (one that ran its share of the chain ahead of the
        # others would otherwise hold the new job's launches until its
        # long-poll expired); attempts of plans still queued for a tracker
        # count in its running set but not as work it knows of.  (Ringing every
        # tracker when j itself was already released cost each tracker a
        # long-poll return per job: 2.6 instead of 5.1 heartbeats per job and
        # -15 to -19 % JobTracker CPU at 1-8 ranks in the rehearsal.)
        if not self.report_assign_expected:
            self._kick()
        else:
            for tr in list(self.trackers.values()):
                if tr.extra_actions and len(tr.running) <= tr.planned:
                    tr.bell.set()

    def _memory_violation(self, conf):
        """JobTracker.checkMemoryRequirements: a job asking for more memory per
        task than ``mapred.cluster.max.{map,reduce}.memory.mb`` is rejected."""
        for kind in ("map", "reduce"):
            mx = self.conf.get_int(f"mapred.cluster.max.{kind}.memory.mb", -1)
            need = conf.get_int(f"mapred.job.{kind}.memory.mb", -1)
            if mx > 0 and need > mx:
                return (f"job's {kind} memory {need} MB exceeds the cluster maximum "
                        f"mapred.cluster.max.{kind}.memory.mb = {mx} MB")
        return None

    def get_job(self, job_id) -> RunningJob | None:
        """JobClient.getJob: a handle on a known (e.g. recovered) job."""
        with self.lock:
            jip = self.jobs.get(str(job_id))
        return None if jip is None else RunningJob(jip.job_id, _JTJobHandle(jip), jip.conf)

    def check_access(self, job_id, op):
        """JobACLsManager check for the current (RPC or doAs) user; raises
        AccessControlException (mapred.acls.enabled)."""
        from .. import security as SEC
        jip = self.jobs.get(str(job_id))
        if jip is None:
            raise KeyError(f"unknown job {job_id}")
        SEC.check_job_access(self.conf, jip.conf, SEC.UserGroupInformation.get_current_user(),
                             SEC.MODIFY_JOB if op == "modify" else SEC.VIEW_JOB)
        return jip

    def kill_job(self, job_id):
        if str(job_id) in self.jobs:
            self.check_access(job_id, "modify")
        with self.lock:
            jip = self.jobs.get(str(job_id))
            if jip is None or jip.completed():
                return
            self._finish_job(jip, KILLED, "killed by user")

    def _finish_job(self, jip: JobInProgress, state, info=""):
        if jip.completed():
            return
        if jip.running_cpu or jip.running_gpu or any(r.is_running() for r in jip.reduces):
            # its attempts still running anywhere get killed (a job that
            # succeeded has none: no tracker need scan its running attempts)
            self.kill_epoch += 1
        st = jip.status
        st.state = state
        st.failure_info = info
        st.finish_time = time.time()
        if state == SUCCEEDED:
            st.map_progress = st.reduce_progress = 1.0
        for tip in jip.maps + jip.reduces:
            tip.killed = state != SUCCEEDED
        if jip in self.job_queue:
            self.job_queue.remove(jip)
        if jip in self.staged:
            self.staged.remove(jip)
        jip.staged_on = None
        jip.fold_counters()
        jip.counters.incr(C.JOB_GROUP, C.CPU_MAP_TASKS, jip.finished_cpu_maps)
        jip.counters.incr(C.JOB_GROUP, C.GPU_MAP_TASKS, jip.finished_gpu_maps)
        self.history.log("JOB_FINISHED", job=str(jip.job_id), state=state,
                         makespan=st.finish_time - jip.submit_time,
                         cpu_maps=jip.finished_cpu_maps, gpu_maps=jip.finished_gpu_maps,
                         info=info)
        if state == SUCCEEDED and jip.split_job is not None:
            try:
                jip.split_job.job_succeeded(jip)
            except Exception:  # noqa: BLE001
                log.exception("job_succeeded hook failed")
        elif jip.split_job is None and jip.maps is not None:
            # job cleanup (the reference's cleanup task: commitJob / abortJob)
            try:
                com = jip.committer()
                com.commit_job(jip.conf) if state == SUCCEEDED else com.abort_job(jip.conf)
            except Exception:  # noqa: BLE001
                log.exception("job cleanup failed")
        if TRACE.on:
            TRACE.instant("jt.job_finished", job=str(jip.job_id), state=state)
        METRICS.inc("hbmr_jobs_completed_total", help="jobs finished, by final state",
                    state=state)
        hdir = _history_dir(self.conf) or _history_dir(jip.conf)
        if hdir:
            try:
                from ..webui.history import write_job_history
                jip.history_file = write_job_history(jip, hdir)
            except Exception:  # noqa: BLE001
                log.exception("writing job history failed")
        self._forget_job(jip.job_id)
        # KillJobAction to every tracker that holds state of the job (the
        # reference purges finished jobs from trackers the same way): its GPU
        # worker frees the job's device map outputs
        jid_s = str(jip.job_id)
        for t in self.trackers.values():
            if jid_s in t.jobs_seen:
                t.jobs_seen.discard(jid_s)
                t.lazy_actions.append(P.kill_job_action(jid_s))
        jip.done.set()
        with jip.events_cond:
            jip.events_cond.notify_all()      # reduces long-polling for events
        for w in self.waiting.pop(str(jip.job_id), []):
            if w.completed():
                continue             # killed while it waited
            if state == SUCCEEDED:
                if w in self.staged:
                    self.staged.remove(w)
                w.staged_on = None
                w.status.state = RUNNING
                w.launch_time = w.release_time = time.time()
                if w.pending_finish:
                    # every task of the staged job finished before this one did
                    self._finish_job(w, SUCCEEDED)
                    continue
                self.job_queue.append(w)
                # jobs waiting for w may now be staged on it
                for x in self.waiting.get(str(w.job_id), []):
                    self._maybe_stage(x, w)
            else:
                self._finish_job(w, FAILED, f"job {jip.job_id} it depends on {state}")
        if state == SUCCEEDED and self._assignable():
            self._kick()
        for cb in self.listeners:
            cb("finished", jip)
        self._retire_jobs(jip)

    def _retire_jobs(self, jip):
        self._completed.append(jip)
        while len(self._completed) > self.keep_completed:
            old = self._completed.popleft()
            old.retire()
            index = self.attempt_index
            for aid in old.retired_aids:
                a = index.get(aid)
                if a is not None and a.state not in P.TERMINAL:
                    # still running (a sampled CPU probe is never killed; a failed
                    # or killed job's attempts may be mid-flight): keep it indexed
                    # as a tombstone so its last report frees the tracker's slot
                    # and the cost model's running entry
                    a.tombstone = True
                    continue
                index.pop(aid, None)
            old.retired_aids = ()
            self._retired.append(str(old.job_id))
            self.history.log("JOB_RETIRED", job=str(old.job_id))
        while len(self._retired) > self.keep_retired:
            self.jobs.pop(self._retired.popleft(), None)

    def _assignable(self) -> bool:
        """Work a long-polling tracker could be handed now: a queued job with
        pending maps or reduces not yet running (staged jobs' maps are already
        launched; their trackers report before those maps can run)."""
        for jip in self.job_queue:
            if jip.pending_maps or (jip.reduces and self._reduces_waiting(jip)):
                return True
        return False

    # -- heartbeat ----------------------------------------------------------------------
    def wakeup(self, tracker_name: str, seq: int | None = None):
        """A tracker has news (a task finished): end its long-poll heartbeat now.
        Lock-free: dict lookup + attribute store + Event.set.  ``seq`` is the
        tracker's notification count: it survives the heartbeat entry's reset,
        so news that arrives while the heartbeat is in flight is never lost."""
        tr = self.trackers.get(tracker_name)
        if tr is not None:
            if seq is None:
                tr.wake = True
            elif seq > tr.wake_seq:
                tr.wake_seq = seq
            tr.bell.set()

    def report(self, status: dict, assign: bool = False):
        """A tracker's news (finished attempts, lost outputs, cache changes)
        while its heartbeat long-polls.

        ``assign`` (hbmr.tracker.report.assign): processed like a heartbeat
        WITH assignment, and the actions (new launches, commit approvals,
        kills) return in this call's response — the long-poll stays parked.
        One RPC per tracker and job in the steady state of chained jobs
        (the reduce's report, carrying its deferred map completions, gets the
        next staged job's launches back), where the ring-the-long-poll form
        cost the report, the long-poll's return and a new long-poll; the
        JobTracker's per-tracker work is what bounds multi-rank jobs.

        Otherwise: processed without assignment and the long-poll is rung to
        assign into any freed slots and return what that yields."""
        name = status["tracker_name"] if isinstance(status, dict) else status.tracker_name
        tr = self.trackers.get(name)
        if tr is None:
            return {"reinit": True}
        if assign:
            resp = self._heartbeat(status, False, True)
            return {"actions": resp["actions"], "seq": resp.get("seq")}
        resp = self._heartbeat(status, False, False, number=False)
        if resp["actions"]:
            with self.lock:
                tr.extra_actions += resp["actions"]
        tr.bell.set()
        return {}

    def _kick(self):
        """New work may be assignable: ring every long-polling tracker."""
        for tr in list(self.trackers.values()):
            tr.bell.set()

    def notify(self):
        self._kick()

    def heartbeat(self, status: dict, initial: bool = False, accept_new_tasks: bool = True,
                  block: float = 0.0):
        """Process a tracker's status and return {"actions": [...], "interval": s}.

        With ``block`` > 0 and nothing to hand out, the call long-polls (up to
        ``block`` seconds) until new work exists or the tracker calls wakeup(),
        so idle trackers learn about new tasks immediately instead of on their
        next periodic heartbeat (the reference's 3 s floor, B13)."""
        name = status["tracker_name"] if isinstance(status, dict) else status.tracker_name
        seen = (status.get("notify_seq", 0) if isinstance(status, dict)
                else getattr(status, "notify_seq", 0))
        tr0 = self.trackers.get(name)
        if tr0 is not None:
            # clear before this call's assignment: a ring from here on re-polls
            tr0.bell.clear()
            tr0.wake = False
        if TRACE.on:
            with TRACE.span("jt.heartbeat", block=block):
                resp = self._heartbeat(status, initial, accept_new_tasks)
        else:
            resp = self._heartbeat(status, initial, accept_new_tasks)
        if getattr(self, "_shutdown_trackers", False):
            resp["actions"].append(P.shutdown_action())
            return resp
        if resp["actions"] or block <= 0 or not accept_new_tasks:
            return self._with_lazy(tr0 or self.trackers.get(name), resp)
        deadline = time.time() + block
        tr = self.trackers.get(name)
        if tr is None:
            return resp
        while not resp["actions"]:
            if tr.wake or tr.wake_seq > seen or self._stop.is_set():
                break
            left = deadline - time.time()
            if left <= 0:
                break
            tr.bell.wait(left)
            tr.bell.clear()
            if TRACE.on:
                TRACE.instant("jt.longpoll.wake", wake=tr.wake or tr.wake_seq > seen)
            if tr.wake or tr.wake_seq > seen or self.trackers.get(name) is not tr:
                break
            if getattr(self, "_shutdown_trackers", False):
                resp["actions"].append(P.shutdown_action())
                break
            with self.lock:
                if tr.extra_actions:
                    resp["actions"] += tr.extra_actions
                    tr.extra_actions = []
                    tr.planned = 0
                if tr.kills:
                    resp["actions"] += [P.kill_task_action(aid) for aid in sorted(tr.kills)]
                    tr.kills.clear()
                if tr.status.healthy and not tr.blacklisted:
                    resp["actions"] += self.scheduler.assign_tasks(tr)
                    if TRACE.on:
                        TRACE.instant("jt.assigned", n=len(resp["actions"]))
                if resp["actions"]:
                    self._number(tr, resp)
        tr.wake = False
        resp["more"] = tr.more
        return self._with_lazy(tr, resp)

    @staticmethod
    def _number(tr, resp):
        """Give a response that goes back to its tracker the next sequence
        number (the order its actions were produced in; callers hold the lock)
        and keep it for a resend."""
        tr.resp_seq += 1
        resp["seq"] = tr.resp_seq
        tr.sent.append((tr.resp_seq, list(resp["actions"])))

    def resend(self, tracker_name, after_seq):
        """The numbered responses after ``after_seq`` that this JobTracker
        still holds — a tracker whose report reply was lost (the RPC failed
        after the JobTracker processed it) takes back the launches, commit
        approvals and kills it carried; the tracker skips any it applied."""
        tr = self.trackers.get(tracker_name)
        if tr is None:
            return {"responses": []}
        with self.lock:
            return {"responses": [[q, acts] for q, acts in tr.sent if q > after_seq]}

    def _with_lazy(self, tr, resp):
        if tr is not None and tr.lazy_actions:
            with self.lock:
                resp["actions"] += tr.lazy_actions
                tr.lazy_actions = []
                if "seq" not in resp:
                    self._number(tr, resp)
                else:
                    for i, (q, _a) in enumerate(tr.sent):
                        if q == resp["seq"]:
                            tr.sent[i] = (q, list(resp["actions"]))
        return resp

    def _heartbeat(self, status, initial, accept_new_tasks, number=True):
        # number=False: the caller re-queues the actions (report without
        # assignment) and they are numbered where they are finally returned
        st = P.TaskTrackerStatus.from_dict(status) if isinstance(status, dict) else status
        now = time.time()
        actions = []
        with self.lock:
            tr = self.trackers.get(st.tracker_name)
            if tr is None:
                if not initial:
                    # unknown tracker (e.g. after JT restart / expiry): re-initialise
                    return {"actions": [P.reinit_action()], "interval": self.heartbeat_interval}
                tr = self.trackers[st.tracker_name] = TrackerInfo(st, now)
                tr.rack = self.topology.rack(st.host)
                if self.system_dir:
                    self._save_info()
                self.history.log("TRACKER_JOINED", tracker=st.tracker_name, host=st.host,
                                 rack=tr.rack,
                                 cpu_slots=st.max_cpu_map_slots,
                                 gpus=[g["device"] for g in st.gpus])
            tr.status = st
            tr.last_seen = now
            cap = (st.max_cpu_map_slots, st.max_reduce_slots,
                   tuple((g["device"], g["max_slots"]) for g in st.gpus))
            if cap != tr.cap_sig:
                tr.cap_sig = cap
                self.cap_epoch += 1
            for k in st.cached_splits_added:
                tr.cached.add(tuple(k))
            for k in st.cached_splits_removed:
                tr.cached.discard(tuple(k))
            # batched map completions first: they precede any reduce report
            # that rides with them (TaskTracker.maps_done_news)
            for bulk in st.bulk_reports:
                self._bulk_succeeded(tr, bulk)
            for rep in st.task_reports:
                self._update_task_status(tr, P.TaskStatus.from_dict(rep), actions)
            if st.lost_outputs:
                self._outputs_lost(tr, st.lost_outputs)
            if self._to_recover:
                self._maybe_recover(now)
            tr.more = False
            if accept_new_tasks and st.healthy and not tr.blacklisted:
                actions += self.scheduler.assign_tasks(tr)
            # kill attempts of jobs that are done / tasks already completed
            # (CPU profiling probes excepted: a sampled probe rides on a TIP that
            # the GPUs finish long before it, and killing it would leave the cost
            # model a censored bound instead of the CPU time)
            # (a scan per heartbeat over every running attempt was a top cost of
            # the JobTracker at 4-8 ranks; only a job ending or a TIP won by one
            # of several attempts can create work here — kill_epoch counts those)
            if tr.kill_epoch != self.kill_epoch:
                tr.kill_epoch = self.kill_epoch
                for aid in list(tr.running):
                    a = self.attempt_index.get(aid)
                    if a is not None and not a.profile_only and not a.profile_fraction and (
                            a.tip.job.completed() or
                            (a.tip.successful is not None and a.tip.successful is not a)):
                        tr.kills.add(aid)
            if tr.kills:
                actions += [P.kill_task_action(aid) for aid in sorted(tr.kills)]
                tr.kills.clear()
            if st.gpu_worker_lost:
                self._restart_gpu_gang(tr)
            if tr.extra_actions:
                # a closed gate goes before this response's launches: a staged
                # map launched here must not pass the gate of a restarted job
                pre = [x for x in tr.extra_actions if x["type"] == "close_gate"]
                actions = pre + actions + [x for x in tr.extra_actions
                                           if x["type"] != "close_gate"]
                tr.extra_actions = []
                tr.planned = 0
            resp = {"actions": actions, "interval": self.heartbeat_interval, "more": tr.more}
            if actions and number:
                # numbered under the lock that drained the tracker's queues:
                # the numbering is the order the actions were produced in
                self._number(tr, resp)
        return resp

    def _update_task_status(self, tr: TrackerInfo, ts: P.TaskStatus, actions):
        a = self.attempt_index.get(ts.attempt_id)
        if a is None or a.state in P.TERMINAL:
            return
        if a.tombstone:
            self._retired_attempt_status(a, ts, actions)
            return
        a.progress = ts.progress
        a.counters = ts.counters or a.counters
        if ts.start_time:
            a.start = ts.start_time
        jip = a.tip.job
        if ts.state == P.SUCCEEDED:
            a.finish = ts.finish_time or time.time()
            a.output = ts.output
            a.device_time = ts.device_time
            self._attempt_succeeded(a)
        elif ts.state in (P.FAILED, P.KILLED, P.FAILED_UNCLEAN):
            a.finish = ts.finish_time or time.time()
            self._attempt_failed(a, ts.diagnostic, killed=ts.state == P.KILLED)
        elif ts.state == P.COMMIT_PENDING:
            a.state = P.COMMIT_PENDING
            tip = a.tip
            if tip.commit_granted is None and tip.successful is None:
                tip.commit_granted = a.aid
                actions.append(P.commit_action(a.aid))
            elif tip.commit_granted != a.aid:
                actions.append(P.kill_task_action(a.aid))
        self._update_progress(jip)

    def _retired_attempt_status(self, a: Attempt, ts: P.TaskStatus, actions):
        """A report for an attempt whose job has been retired: once it ends,
        free what it held (tracker slot, the cost model's running entry; a
        sampled probe still contributes its measured time) and drop it; one
        waiting for a commit is told to die (its job is over)."""
        if ts.state == P.COMMIT_PENDING:
            actions.append(P.kill_task_action(a.aid))
            return
        if ts.state not in P.TERMINAL and ts.state != P.FAILED_UNCLEAN:
            return
        jip = a.tip.job
        now = ts.finish_time or time.time()
        self._release(a)
        if a.tip.is_map:
            if ts.state == P.SUCCEEDED and a.profile_fraction:
                meas = ts.device_time if ts.device_time > 0 else now - a.start
                self.cost_model.task_finished(jip.signature, a.aid, False, a.start,
                                              a.start + max(0.0, meas) / a.profile_fraction)
            else:
                self.cost_model.task_finished(jip.signature, a.aid, a.run_on_gpu, a.start, now,
                                              succeeded=False)
        a.state = ts.state if ts.state in P.TERMINAL else P.FAILED
        self.attempt_index.pop(a.aid, None)

    def _release(self, a: Attempt):
        if a.tip.is_map and not a._released:
            jip = a.tip.job
            if a.gated:
                key = (a.tracker, a.device)
                jip.staged_launched[key] = max(0, jip.staged_launched.get(key, 1) - 1)
            if a.run_on_gpu:
                jip.running_gpu = max(0, jip.running_gpu - 1)
            else:
                jip.running_cpu = max(0, jip.running_cpu - 1)
        a._released = True
        tr = self.trackers.get(a.tracker)
        if tr is not None and a.aid in tr.running:
            tr.running.discard(a.aid)
            if a.tip.is_map:
                if a.run_on_gpu:
                    tr.running_gpu[a.device] = max(0, tr.running_gpu.get(a.device, 1) - 1)
                else:
                    tr.running_cpu = max(0, tr.running_cpu - a.slots)
            else:
                tr.running_reduce = max(0, tr.running_reduce - a.slots)

    def _attempt_succeeded(self, a: Attempt):
        tip = a.tip
        jip = tip.job
        a.state = P.SUCCEEDED
        self._release(a)
        if a.profile_fraction:
            # sampled profiling probe: its only product is the CPU time estimate
            # (measured on the sample, scaled to a whole split)
            # (its own compute time when the tracker reports it: the launch and
            # report latency around it would be multiplied by 1/fraction too)
            meas = a.device_time if a.device_time > 0 else a.finish - a.start
            dt = max(0.0, meas) / a.profile_fraction
            self.cost_model.task_finished(jip.signature, a.aid, False, a.start, a.start + dt)
            self.history.log("PROFILE_FINISHED", attempt=a.aid, tracker=a.tracker,
                             fraction=a.profile_fraction, est_seconds=dt)
            return
        if tip.is_map:
            if a.run_on_gpu and a.device_time > 0:
                # GPU attempts are timed by HIP events: device time, not queue time
                self.cost_model.task_finished(jip.signature, a.aid, True, 0.0, a.device_time)
            else:
                self.cost_model.task_finished(jip.signature, a.aid, a.run_on_gpu, a.start,
                                              a.finish)
        if tip.successful is not None or tip.killed:
            return  # a speculative twin already won
        tip.successful = a
        if len(tip.attempts) > 1:
            self.kill_epoch += 1      # its twins (speculative / probe) may need killing
        if tip.is_map:
            jip.maps_done += 1
        else:
            jip.reduces_done += 1
        jip.add_counters(a.counters)
        if not tip.is_map and isinstance(a.output, dict) and a.output.get("result") is not None:
            if jip.result is None:
                jip.result = {}
            jip.result[tip.partition] = a.output["result"]
        if tip.is_map:
            if a.run_on_gpu:
                jip.finished_gpu_maps += 1
            else:
                jip.finished_cpu_maps += 1
            jip.completion_events.append((tip.tid, a.aid, a.output))
            with jip.events_cond:
                jip.events_cond.notify_all()
        # kill other running attempts of this TIP
        for other in tip.running_attempts():
            if other is not a:
                if tip.is_map and not other.run_on_gpu and \
                        self.cost_model.stats(jip.signature, False).n == 0 and \
                        self.cost_model.is_probe(jip.signature, other.aid, False):
                    # the signature's CPU profiling probe lost to its GPU backup:
                    # let it finish detached (output ignored, slot held) so the
                    # cost model learns the real CPU time instead of a censored
                    # bound that would invite more doomed CPU attempts
                    other.profile_only = True
                    continue
                other.state = P.KILLED
                self._release(other)
                tr_o = self.trackers.get(other.tracker)
                if tr_o is not None:
                    tr_o.kills.add(other.aid)
                if tip.is_map:
                    self.cost_model.task_finished(jip.signature, other.aid, other.run_on_gpu,
                                                  other.start, time.time(), succeeded=False)
        self.history.log("TASK_FINISHED", attempt=a.aid, tracker=a.tracker,
                         gpu=a.run_on_gpu, device=a.device, start=a.start, finish=a.finish,
                         device_time=a.device_time)
        METRICS.inc("hbmr_tasks_succeeded_total", help="successful task attempts",
                    type="map" if tip.is_map else "reduce", where="gpu" if a.run_on_gpu else "cpu")
        if tip.is_map and jip.maps_complete():
            jip.t_maps_done = time.time()
        self._check_job_done(jip)
        if tip.is_map and jip.reduces and (jip.maps_complete() or
                                           jip.maps_done == jip.slowstart_maps) and \
                self._reduces_waiting(jip):
            self._kick()  # reduces became schedulable: wake long-polling trackers

    @staticmethod
    def _reduces_waiting(jip) -> bool:
        """Any reduce neither done nor running (an early collective reduce
        gang already runs: ringing every tracker would find nothing to do)."""
        return any(t.successful is None and not t.is_running() for t in jip.reduces)

    def _bulk_succeeded(self, tr: TrackerInfo, rep: dict):
        """A batch of GPU map attempts that completed together (one HIP event
        pair): the lean path of _attempt_succeeded — per attempt only the TIP
        bookkeeping; counters, cost model, history and metrics once per batch."""
        aids = rep["attempts"]
        dt = float(rep.get("device_time", 0.0))
        fin = rep.get("finish_time") or time.time()
        out = rep.get("output") or {}
        index = self.attempt_index
        done = []
        odd = []
        terminal = P.TERMINAL
        succeeded = P.SUCCEEDED
        running = tr.running
        running_gpu = tr.running_gpu
        # per attempt only what is its own; the counts (job, tracker, device,
        # staged budget) are folded once per batch below
        jp = dev = ev = None
        ungated = gated = 0
        for aid in aids:
            a = index.get(aid)
            if a is None or a.state in terminal:
                continue
            tip = a.tip
            if a.profile_fraction or tip.successful is not None or tip.killed or \
                    len(tip.attempts) > 1 or \
                    (jp is not None and (tip.job is not jp or a.device != dev)):
                # speculative twins etc. (and anything not of the batch's job
                # and device): the general path
                odd.append(a)
                continue
            if jp is None:
                jp, dev = tip.job, a.device
                ev = jp.completion_events
            a.progress = 1.0
            a.finish = fin
            a.output = out
            a.device_time = dt
            a.state = succeeded
            if not a._released:
                a._released = True
                running.discard(aid)
                if a.gated:
                    gated += 1
                else:
                    ungated += 1
            tip.successful = a
            # (map id, attempt, output): map_completion_events renders them
            ev.append((tip.tid, aid, out))
            done.append(a)
        if done:
            n = len(done)
            rel = gated + ungated
            if gated:
                key = (tr.name, dev)
                jp.staged_launched[key] = max(0, jp.staged_launched.get(key, gated) - gated)
            jp.running_gpu = max(0, jp.running_gpu - rel)
            running_gpu[dev] = max(0, running_gpu.get(dev, rel) - rel)
            jp.maps_done += n
            jp.finished_gpu_maps += n
            jip = jp
            with jp.events_cond:
                jp.events_cond.notify_all()
            done_ids = [a.aid for a in done]
            self.cost_model.tasks_finished(jip.signature, done_ids, True, dt, jip.job_id)
            if rep.get("counters"):
                jip.add_counters(rep["counters"])
            self.history.log("TASKS_FINISHED", attempts=done_ids, tracker=tr.name,
                             gpu=True, device=dev, finish=fin, device_time=dt)
            METRICS.inc("hbmr_tasks_succeeded_total", n, help="successful task attempts",
                        type="map", where="gpu")
            self._update_progress(jp)
            if jp.maps_complete():
                jp.t_maps_done = time.time()
            self._check_job_done(jp)
            if jp.reduces and jp.maps_complete() and self._reduces_waiting(jp):
                self._kick()
        for a in odd:
            self._update_task_status(tr, P.TaskStatus(
                attempt_id=a.aid, is_map=True, state=P.SUCCEEDED, progress=1.0,
                run_on_gpu=True, gpu_device_id=a.device, finish_time=fin, output=out,
                device_time=dt), [])

    def _restart_gpu_gang(self, origin: TrackerInfo):
        """A GPU worker died while world > 1: its peers may be blocked in a
        collective with it.  Every GPU tracker restarts its worker under a new
        communicator generation (their held map outputs are reported lost and
        re-executed)."""
        self.worker_generation += 1
        g = self.worker_generation
        self.history.log("GPU_GANG_RESTART", origin=origin.name, generation=g)
        log.warning("GPU worker of %s died: restarting every GPU worker (generation %d)",
                    origin.name, g)
        for t in self.trackers.values():
            if t.status.gpus:
                t.extra_actions.append(P.restart_gpu_worker_action(g))
        self._kick()

    def _restart_collective(self, jip: JobInProgress, diag, kill_maps=False):
        """Re-run a split job's collective reduce gang: kill the running members,
        forget finished ones and re-execute the maps (their outputs were consumed
        by finished members or died with a worker).

        Jobs staged on this one (``_maybe_stage``) may already have run maps on
        the failed gang's result — its reduce opens their gates as soon as it has
        enqueued that result, before it finishes: they restart too, their held
        or running map attempts killed (``kill_maps``), and every GPU tracker
        closes this job's gate, so the re-launched maps wait for the new reduce."""
        self.history.log("COLLECTIVE_RESTART", job=str(jip.job_id), diag=diag[:500])
        jip.expect_mode = False
        jip.pending_finish = False
        if kill_maps:
            for tip in jip.maps:
                for a in tip.running_attempts():
                    a.state = P.KILLED
                    self._release(a)
                    t = self.trackers.get(a.tracker)
                    if t is not None:
                        t.kills.add(a.aid)
                if tip.successful is None:
                    jip.add_pending(tip)
        for r in jip.reduces:
            for a in r.running_attempts():
                a.state = P.KILLED
                self._release(a)
                t = self.trackers.get(a.tracker)
                if t is not None:
                    t.kills.add(a.aid)
            if r.successful is not None:
                r.successful = None
                jip.reduces_done -= 1
        jip.result = None
        for tip in jip.maps:
            a = tip.successful
            if a is None:
                continue
            tip.successful = None
            a.state = P.KILLED
            jip.maps_done -= 1
            if a.run_on_gpu:
                jip.finished_gpu_maps -= 1
            else:
                jip.finished_cpu_maps -= 1
            jip.add_pending(tip)
        jip.t_maps_done = 0.0
        self._update_progress(jip)
        jid = str(jip.job_id)
        staged = [w for w in self.staged if w.staged_on == jid and not w.completed()]
        # always: a failed member of the gang may already have opened this job's
        # gate on the trackers (release_dependents runs before its failure), and
        # a job staged on this one AFTER the restart would otherwise launch its
        # maps through that stale open gate onto the failed attempt's result
        for t in self.trackers.values():
            if t.status.gpus:
                t.extra_actions.append(P.close_gate_action(jid))
        for w in staged:
            self.history.log("STAGED_JOB_RESTART", job=str(w.job_id), gate=jid)
            self._restart_collective(w, f"job {jid} it is staged on restarted", kill_maps=True)
        self._kick()

    def preempt_attempt(self, a: Attempt, why="preempted"):
        """Kill a running attempt to give its slot to another pool (fair-share
        preemption): KILLED, not FAILED — its TIP goes back to pending without
        counting a failure (FairScheduler.preemptTasks, JobInProgress
        .killTask(..., shouldFail=false))."""
        if a.state in P.TERMINAL:
            return
        t = self.trackers.get(a.tracker)
        if t is not None:
            t.kills.add(a.aid)
        jip = a.tip.job
        jip.counters.incr(C.JOB_GROUP, "NUM_PREEMPTED_TASKS")
        self.history.log("TASK_PREEMPTED", attempt=a.aid, tracker=a.tracker, why=why)
        self._attempt_failed(a, why, killed=True)
        self._kick()

    def _outputs_lost(self, tr: TrackerInfo, aids):
        """Map outputs held by a tracker's GPU worker are gone (the worker died):
        re-execute those maps if their job still needs them (the per-attempt
        analogue of lostTaskTracker's re-execution, JobInProgress.java:3140-3160)."""
        for aid in aids:
            a = self.attempt_index.get(aid)
            if a is None:
                continue
            tip = a.tip
            jip = tip.job
            if jip.completed() or tip.successful is not a or not jip.reduces:
                continue
            if any(r.is_complete() for r in jip.reduces):
                continue
            tip.successful = None
            a.state = P.KILLED
            jip.maps_done -= 1
            jip.t_maps_done = 0.0
            if a.run_on_gpu:
                jip.finished_gpu_maps -= 1
            else:
                jip.finished_cpu_maps -= 1
            jip.add_pending(tip, front=True)
            self.history.log("MAP_OUTPUT_LOST", attempt=aid, tracker=tr.name)
            if jip.expect_mode:
                self._restart_collective(jip, "map output lost")
        self._kick()

    def _attempt_failed(self, a: Attempt, diag, killed=False):
        tip = a.tip
        jip = tip.job
        if a.state in P.TERMINAL:
            return
        a.state = P.KILLED if killed else P.FAILED
        a.diagnostic = diag
        self._release(a)
        if tip.is_map:
            self.cost_model.task_finished(jip.signature, a.aid, a.run_on_gpu, a.start,
                                          time.time(), succeeded=False)
        if a.profile_fraction:
            self.history.log("PROFILE_FAILED", attempt=a.aid, tracker=a.tracker, diag=diag[:500])
            return
        self.history.log("TASK_FAILED" if not killed else "TASK_KILLED", attempt=a.aid,
                         tracker=a.tracker, gpu=a.run_on_gpu, diag=diag[:500])
        METRICS.inc("hbmr_tasks_failed_total", help="failed or killed task attempts",
                    state="killed" if killed else "failed", where="gpu" if a.run_on_gpu else "cpu")
        if tip.commit_granted == a.aid:
            tip.commit_granted = None
        if jip.completed() or tip.successful is not None:
            return
        if not killed:
            tip.failures += 1
            if not isinstance(tip.failed_trackers, set):
                tip.failed_trackers = set()
            tip.failed_trackers.add(a.tracker)
            jip.counters.incr(C.JOB_GROUP, C.NUM_FAILED_MAPS if tip.is_map else
                              C.NUM_FAILED_REDUCES)
            tr = self.trackers.get(a.tracker)
            if tr is not None:
                tr.failures += 1
                if tr.failures >= self.max_tracker_failures * 4 and len(self.trackers) > 1:
                    tr.blacklisted = True
                    self.cap_epoch += 1
                    self.history.log("TRACKER_BLACKLISTED", tracker=tr.name)
        limit = jip.max_map_attempts if tip.is_map else jip.max_reduce_attempts
        if tip.failures >= limit:
            self._finish_job(jip, FAILED, f"Task {tip.tid} failed {tip.failures} times: {diag}")
            return
        if not tip.running_attempts():
            if tip.is_map:
                jip.add_pending(tip, front=True)  # failed tasks first (findNewMapTask)
                if jip.expect_mode:
                    # the gang was launched expecting this attempt's output
                    self._restart_collective(jip, diag)
            elif jip.collective_reduce:
                # a collective gang cannot restart one member: the whole gang re-runs
                self._restart_collective(jip, diag)

    def _update_progress(self, jip: JobInProgress):
        # O(1): completed fraction (the reference recomputed this from every TIP)
        if jip.maps:
            jip.status.map_progress = jip.maps_done / len(jip.maps)
        if jip.reduces:
            jip.status.reduce_progress = jip.reduces_done / len(jip.reduces)

    def _check_job_done(self, jip: JobInProgress):
        # O(1) on the counters; the TIP scan only confirms the rare final case
        if jip.maps_done < len(jip.maps) or jip.reduces_done < len(jip.reduces):
            return
        if all(t.successful is not None for t in jip.maps) and \
                all(t.successful is not None for t in jip.reduces):
            if jip.staged_on is not None:
                # a staged job ran ahead of the job it depends on: it succeeds
                # when that one does (or fails with it)
                jip.pending_finish = True
                return
            self._finish_job(jip, SUCCEEDED)

    # -- launching (called by the scheduler under the lock) -------------------------------
    def launch(self, tr: TrackerInfo, tip: TaskInProgress, on_gpu=False, device=-1,
               speculative=False, extra=None, profile_fraction=0.0, slots=1):
        jip = tip.job
        aid = tip.new_attempt_id()
        a = Attempt(str(aid), tip, tr.name, on_gpu, device, speculative)
        a.slots = max(1, slots) if not on_gpu else 1
        if profile_fraction:
            # a sampled CPU probe rides on a TIP without being one of its attempts:
            # the TIP stays pending for real execution
            a.profile_fraction = profile_fraction
            a.profile_only = True
            jip.probe_aids.append(a.aid)
            jip.counters.incr(C.JOB_GROUP, "PROFILE_TASKS")
        else:
            tip.attempts[a.aid] = a
        self.attempt_index[a.aid] = a
        tr.running.add(a.aid)
        if tip.is_map:
            jip.launched_on.setdefault(tr.name, []).append(tip)
            if not jip.t_first_map:
                jip.t_first_map = a.start
            if on_gpu:
                tr.running_gpu[device] = tr.running_gpu.get(device, 0) + 1
                jip.running_gpu += 1
            else:
                tr.running_cpu += a.slots
                jip.running_cpu += 1
            self.cost_model.task_started(jip.signature, a.aid, on_gpu, a.start,
                                         fraction=profile_fraction or 1.0)
            if not profile_fraction:
                jip.counters.incr(C.JOB_GROUP, C.TOTAL_LAUNCHED_MAPS)
        else:
            if not jip.t_first_reduce:
                jip.t_first_reduce = a.start
            tr.running_reduce += a.slots
            jip.counters.incr(C.JOB_GROUP, C.TOTAL_LAUNCHED_REDUCES)
        spec = P.TaskSpec(attempt_id=a.aid, job_id=str(jip.job_id), is_map=tip.is_map,
                          partition=tip.partition, run_on_gpu=on_gpu, gpu_device_id=device,
                          split=tip.split or {}, num_maps=len(jip.maps),
                          num_reduces=len(jip.reduces), collective=jip.collective_reduce,
                          profile_fraction=profile_fraction)
        if extra:
            for k, v in extra.items():
                setattr(spec, k, v)
        if str(jip.job_id) not in tr.jobs_seen:
            spec.conf = jip.conf_dict
            tr.jobs_seen.add(str(jip.job_id))
        self.history.log("TASK_LAUNCHED", attempt=a.aid, tracker=tr.name, gpu=on_gpu,
                         device=device, speculative=speculative)
        METRICS.inc("hbmr_tasks_launched_total", help="task attempts launched",
                    type="map" if tip.is_map else "reduce", where="gpu" if on_gpu else "cpu")
        return P.launch_action(spec)

    def launch_gpu_batch(self, tr: TrackerInfo, tips, device, gate=None):
        """One bulk LaunchTaskAction for GPU map attempts of one job on one device
        (the per-task launch() costs ~50 µs of JobTracker time; this ~3 µs).
        The tracker queues them on the device's slots as one batch."""
        jip = tips[0].job
        now = time.time()
        tasks = []
        aids = []
        index = self.attempt_index
        running = tr.running
        name = tr.name
        gated = gate is not None
        jip.launched_on.setdefault(name, []).extend(tips)
        for tip in tips:
            k = tip.next_attempt
            aid = tip._aid_prefix + str(k)
            tip.next_attempt = k + 1
            a = tip.attempts[aid] = index[aid] = Attempt(aid, tip, name, True, device, False, now)
            if gated:
                a.gated = True
            tasks.append([aid, tip.partition, tip.split])
            aids.append(aid)
        running.update(aids)
        n = len(tips)
        tr.running_gpu[device] = tr.running_gpu.get(device, 0) + n
        jip.running_gpu += n
        if not jip.t_first_map:
            jip.t_first_map = now
        self.cost_model.tasks_started(jip.signature, aids, True, now)
        jip.counters.incr(C.JOB_GROUP, C.TOTAL_LAUNCHED_MAPS, n)
        self.history.log("TASKS_LAUNCHED", attempts=aids, tracker=tr.name, gpu=True,
                         device=device)
        METRICS.inc("hbmr_tasks_launched_total", n, help="task attempts launched", type="map",
                    where="gpu")
        act = {"type": "launch_batch", "job_id": str(jip.job_id), "run_on_gpu": True,
               "device": device, "num_maps": len(jip.maps), "num_reduces": len(jip.reduces),
               "collective": jip.collective_reduce, "tasks": tasks}
        if gate is not None:
            act["gate"] = gate
            key = (tr.name, device)
            jip.staged_launched[key] = jip.staged_launched.get(key, 0) + n
        if str(jip.job_id) not in tr.jobs_seen:
            act["conf"] = jip.conf_dict
            tr.jobs_seen.add(str(jip.job_id))
        return act

    def reduce_inputs(self, jip: JobInProgress, tracker_name=None, expect=False):
        """Map outputs a reduce needs: classic = every map's output location;
        collective = the committed map attempts that ran on ``tracker_name``
        (``expect``: plus the single running attempt of every unfinished map)."""
        if jip.collective_reduce:
            out = []
            # only maps launched on this tracker can have outputs here (a TIP
            # re-run elsewhere is listed under that tracker too); map order
            tips = jip.launched_on.get(tracker_name, ())
            live = _LIVE
            for t in sorted(dict.fromkeys(tips), key=_PARTITION):
                a = t.successful
                if a is None and expect:
                    # the single running attempt (running_attempts() inlined:
                    # this runs per map of every staged job's plan)
                    at = t.attempts
                    if len(at) == 1:
                        for a in at.values():
                            if a.state not in live:
                                a = None
                    else:
                        ra = [x for x in at.values() if x.state in live]
                        a = ra[0] if len(ra) == 1 else None
                if a is not None and a.tracker == tracker_name:
                    out.append([t.tid._s, a.aid, a.output or {}])
            return out
        return [[str(t.tid), t.successful.aid, t.successful.output] for t in jip.maps
                if t.successful is not None]

    def map_completion_events(self, job_id, start=0, wait=0.0):
        """TaskUmbilicalProtocol.getMapCompletionEvents (TaskUmbilicalProtocol.java:
        167): successful map outputs from index ``start`` on, for reduces that
        started before every map finished (slow-start).  ``wait`` > 0: with
        nothing new, block up to that long for the next event (the reference's
        GetMapEventsThread polls on a sleep; a copy that waits on a backed-off
        poll starts late)."""
        jip = self.jobs.get(str(job_id))
        if jip is not None and wait > 0 and len(jip.completion_events) <= start:
            with jip.events_cond:
                jip.events_cond.wait_for(
                    lambda: len(jip.completion_events) > start or jip.completed(), timeout=wait)
        with self.lock:
            jip = self.jobs.get(str(job_id))
            if jip is None:
                return {"events": [], "num_maps": 0, "state": "UNKNOWN"}
            evs = jip.completion_events[start:]
            return {"events": [[str(t), aid, out] for t, aid, out in evs],
                    "num_maps": len(jip.maps), "state": jip.status.state,
                    "waited": wait > 0}

    # -- RPC-facing job submission protocol (JobSubmissionProtocol) -------------------------
    def rpc_submit_job(self, conf_dict):
        from .jobconf import JobConf
        conf = JobConf()
        for k, v in conf_dict.items():
            conf.set(k, v)
        return str(self.submit_job(conf).getID())

    def rpc_job_status(self, jid):
        jip = self.check_access(jid, "view")
        st = jip.status
        return {"state": st.state, "map_progress": st.map_progress,
                "reduce_progress": st.reduce_progress, "start_time": st.start_time,
                "finish_time": st.finish_time, "failure_info": st.failure_info,
                "counters": jip.fold_counters().to_dict()}

    def rpc_kill_job(self, jid):
        self.kill_job(jid)

    def rpc_job_result(self, jid):
        return self.check_access(jid, "view").result

    def rpc_list_jobs(self, all_jobs=False):
        """JobSubmissionProtocol.jobsToComplete / getAllJobs."""
        with self.lock:
            out = []
            for jid, jip in self.jobs.items():
                st = jip.status
                if all_jobs or not jip.completed():
                    out.append({"id": jid, "name": jip.conf.get_job_name(), "state": st.state,
                                "user": jip.conf.get_user(), "start": jip.submit_time,
                                "maps": len(jip.maps), "reduces": len(jip.reduces),
                                "map_progress": st.map_progress,
                                "reduce_progress": st.reduce_progress,
                                "cpu_maps": jip.finished_cpu_maps,
                                "gpu_maps": jip.finished_gpu_maps})
            return out

    def rpc_task_reports(self, jid, is_map=True):
        jip = self.check_access(jid, "view")
        with self.lock:
            return [{"task": str(r.getTaskID()), "state": r.state, "progress": r.progress,
                     "start": r.getStartTime(), "finish": r.getFinishTime(),
                     "gpu": r.getRunOnGPU(), "device": r.getGPUDeviceId(),
                     "tracker": getattr(r, "tracker", None)}
                    for r in (t.report() for t in (jip.maps if is_map else jip.reduces))]

    def rpc_cluster_status(self):
        with self.lock:
            return {"trackers": {n: {"cpu_slots": t.status.max_cpu_map_slots,
                                     "gpus": t.gpu_devices(), "running": len(t.running),
                                     "blacklisted": t.blacklisted}
                                 for n, t in self.trackers.items()},
                    "jobs": {j: jip.status.state for j, jip in self.jobs.items()},
                    "cost_model": self.cost_model.snapshot()}

    # -- JobTracker process (hbmr/mapred/jtprocess.py): the node's driver side --------
    def rpc_wait_job(self, jid, timeout=30.0):
        """Long-poll: True once the job is complete (or ``timeout`` passed)."""
        jip = self.check_access(jid, "view")
        return jip.done.wait(max(0.0, min(float(timeout), 60.0)))

    def rpc_wait_job_info(self, jid, timeout=30.0):
        """rpc_wait_job and rpc_job_info in one call: the job's information
        once it is complete, None if ``timeout`` passed first (a driver waiting
        for each iteration job spends one RPC on it, not two)."""
        return self.rpc_job_info(jid) if self.rpc_wait_job(jid, timeout) else None

    def rpc_job_info(self, jid):
        """Everything a driver reads about a job, in one call: status,
        counters, the phase timeline, maps per tracker and the reduce result."""
        jip = self.check_access(jid, "view")
        st = jip.status
        with self.lock:
            per = jip.maps_per_tracker()
        return {"state": st.state, "map_progress": st.map_progress,
                "reduce_progress": st.reduce_progress, "start_time": st.start_time,
                "finish_time": st.finish_time, "failure_info": st.failure_info,
                "counters": jip.fold_counters().to_dict(), "timeline": jip.timeline(),
                "maps_per_tracker": per, "result": jip.result}

    def rpc_wait_for_trackers(self, n, timeout=60.0):
        return self.wait_for_trackers(int(n), float(timeout))

    def rpc_start_expiry(self):
        self.start_expiry_thread()

    def rpc_broadcast_shutdown(self):
        self.broadcast_shutdown()

    def rpc_live_trackers(self, exclude="", window=0.5):
        with self.lock:
            now = time.time()
            return sum(1 for t in self.trackers.values()
                       if t.name != exclude and now - t.last_seen < window)

    def rpc_cost_model(self):
        return self.cost_model.snapshot()

    def rpc_cpu_seconds(self):
        """CPU seconds of this process (a JobTracker process's own cost)."""
        return time.process_time()

    def rpc_thread_cpu(self):
        """CPU seconds per thread of this process, summed over threads whose
        names differ only in digits (RPC handler threads, long-polls): where a
        JobTracker process's CPU goes."""
        import re as _re
        out = {}
        for t in threading.enumerate():
            try:
                sec = time.clock_gettime(time.pthread_getcpuclockid(t.ident))
            except (OSError, AttributeError, TypeError):
                continue
            key = _re.sub(r"\d+", "#", t.name)
            out[key] = out.get(key, 0.0) + sec
        return out

    def broadcast_shutdown(self):
        """Tell every tracker to exit on its next heartbeat."""
        with self.lock:
            self._shutdown_trackers = True
            self._kick()

    def shutdown(self):
        self._stop.set()
        with self.lock:
            self._kick()


def job_result(rj: RunningJob):
    impl = rj._impl
    return getattr(impl, "result", None)


def _history_dir(conf):
    return conf.get("hbmr.history.dir") or conf.get("hadoop.job.history.location")
