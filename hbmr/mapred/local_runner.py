"""LocalJobRunner: runs a whole job in-process
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/LocalJobRunner.java:72-260).

Maps run one after another (or on ``mapred.local.map.tasks.maximum`` threads),
then the reducers; the map outputs are local files, so the "shuffle" is a
direct read.  Selected by ``mapred.job.tracker=local`` — BASELINE config 1
(WordCount, CPU-only mappers) runs here.
"""
from __future__ import annotations

import concurrent.futures as cf
import itertools
import logging
import os
import shutil
import tempfile
import threading
import time

from ..utils.reflection import new_instance
from . import counters as C
from .ids import JobID, TaskAttemptID, TaskID
from .jobclient import FAILED, RUNNING, SUCCEEDED, RunningJob, _Waitable
from .child import use_child_process
from .task import MapOutputLocation, MapTask, ReduceTask

log = logging.getLogger("hbmr.local")

_job_seq = itertools.count(1)


class TaskReport:
    def __init__(self, tid, progress, state, start, finish, counters, run_on_gpu=False,
                 gpu_device_id=-1, tracker=""):
        self.task_id = tid
        self.progress = progress
        self.state = state
        self.start_time = start
        self.finish_time = finish
        self.counters = counters
        self.run_on_gpu = run_on_gpu
        self.gpu_device_id = gpu_device_id
        self.tracker = tracker

    def getRunOnGPU(self):  # noqa: N802
        return self.run_on_gpu

    def getGPUDeviceId(self):  # noqa: N802
        return self.gpu_device_id

    def getTaskID(self):  # noqa: N802
        return self.task_id

    def getStartTime(self):  # noqa: N802
        return self.start_time

    def getFinishTime(self):  # noqa: N802
        return self.finish_time


class _LocalJob(_Waitable):
    def __init__(self, job_id, conf, runner):
        super().__init__(job_id)
        self.conf = conf
        self.runner = runner
        self.killed = threading.Event()
        self.map_reports: list[TaskReport] = []
        self.reduce_reports: list[TaskReport] = []

    def kill(self):
        self.killed.set()

    def task_reports(self, is_map=True):
        return list(self.map_reports if is_map else self.reduce_reports)


_POOLS: dict = {}
_POOLS_LOCK = threading.Lock()


def _local_children(job):
    """A warm pool of child processes shared by this process's local jobs
    (the LocalJobRunner's parallel maps, ``mapred.task.isolation=process``):
    children are started once and kept across jobs with the same child
    environment — each task carries its own conf and work directory — and
    leave after ``hbmr.task.child.idle.ms`` idle.  Starting 8 interpreters per
    job cost more than the maps of a 64 MB WordCount (219 MB/s with 8 map
    processes against 509 serial in round 5).  Returns (manager, pool key)."""
    from .child import ChildManager
    from .jobconf import JobConf
    env = (job.get("mapred.child.env") or "", job.get_int("mapred.child.ulimit", 0))
    key = f"local:{hash(env) & 0xFFFFFFFF:08x}"
    with _POOLS_LOCK:
        mgr = _POOLS.get(key)
        if mgr is None:
            conf = JobConf()
            conf.set("mapred.child.env", env[0])
            conf.set_int("mapred.child.ulimit", env[1])
            conf.set_int("mapred.job.reuse.jvm.num.tasks", -1)
            conf.set_int("hbmr.task.child.idle.ms", job.get_int("hbmr.task.child.idle.ms", 5000))
            mgr = _POOLS[key] = (ChildManager("local-pool", tempfile.mkdtemp(prefix="hbmr-lpool-"),
                                              conf), conf)
            if len(_POOLS) == 1:
                import atexit
                atexit.register(_shutdown_pools)
    return _PooledChildren(*mgr), key


class _PooledChildren:
    """run_task on the pool with the pool's spawn conf (unlimited reuse)."""

    def __init__(self, mgr, spawn_conf):
        self.mgr, self.spawn_conf = mgr, spawn_conf

    def run_task(self, key, job, payload, reporter, kill_event):
        return self.mgr.run_task(key, job, payload, reporter, kill_event,
                                 spawn_conf=self.spawn_conf)


def _shutdown_pools():
    with _POOLS_LOCK:
        pools = list(_POOLS.values())
        _POOLS.clear()
    for mgr, _conf in pools:
        mgr.shutdown()


class LocalJobRunner:
    def __init__(self, conf=None):
        self.conf = conf
        self.jt_id = "local" + time.strftime("%Y%m%d%H%M")

    def submit_job(self, job) -> RunningJob:
        jid = JobID(self.jt_id, next(_job_seq))
        lj = _LocalJob(jid, job, self)
        t = threading.Thread(target=self._run, args=(lj,), name=f"LocalJob-{jid}", daemon=True)
        t.start()
        return RunningJob(jid, lj, job)

    def _run(self, lj: _LocalJob):
        job = lj.conf
        st = lj._status
        st.state = RUNNING
        local_root = tempfile.mkdtemp(prefix=f"hbmr-{lj._status.job_id}-",
                                      dir=job.get("hbmr.local.scratch") or None)
        committer_cls = job.get_output_committer()
        committer = committer_cls() if isinstance(committer_cls, type) else committer_cls
        try:
            from ..filecache import TrackerCacheManager
            TrackerCacheManager(local_root).localize(str(st.job_id), job)
            informat = new_instance(job.get_input_format(), job)
            outfmt = new_instance(job.get_output_format(), job)
            outfmt.checkOutputSpecs(None, job)
            splits = informat.getSplits(job, job.get_num_map_tasks())
            R = job.get_num_reduce_tasks()
            committer.setup_job(job)
            st.setup_progress = 1.0
            jid = st.job_id
            outputs = [None] * len(splits)
            maps = []
            for i, sp in enumerate(splits):
                aid = TaskAttemptID(TaskID(jid, True, i), 0)
                maps.append(MapTask(job, aid, i, sp))
            nthreads = max(1, job.get_int("mapred.local.map.tasks.maximum", 1))
            # parallel local maps in child processes (past the GIL) when asked for
            children = None
            pool_key = str(jid)
            if nthreads > 1 and use_child_process(job):
                children, pool_key = _local_children(job)
                conf_dict = job.to_dict()

            def run_map(i):
                if lj.killed.is_set():
                    raise RuntimeError("job killed")
                t = maps[i]
                work = os.path.join(local_root, str(t.attempt_id))
                if children is not None:
                    sp = t.split
                    payload = {"attempt_id": str(t.attempt_id), "is_map": True, "partition": i,
                               "split": {"kind": "class",
                                         "cls": f"{type(sp).__module__}:{type(sp).__qualname__}",
                                         "data": sp.serialize().hex()},
                               "conf": conf_dict, "work_dir": work, "progress_interval": 1.0}
                    t.start_time = time.time()
                    outputs[i] = children.run_task(pool_key, job, payload, t.reporter,
                                                   threading.Event())
                    t.finish_time = time.time()
                else:
                    outputs[i] = t.run(work)
                lj.map_reports.append(TaskReport(t.attempt_id.task, 1.0, SUCCEEDED, t.start_time,
                                                 t.finish_time, t.reporter.counters))
                lj._counters.incr_all(t.reporter.counters)
                st.map_progress = len(lj.map_reports) / max(1, len(maps))

            if nthreads == 1:
                for i in range(len(maps)):
                    run_map(i)
            else:
                with cf.ThreadPoolExecutor(nthreads) as ex:
                    list(ex.map(run_map, range(len(maps))))
            lj._counters.incr(C.JOB_GROUP, C.TOTAL_LAUNCHED_MAPS, len(maps))
            lj._counters.incr(C.JOB_GROUP, C.CPU_MAP_TASKS, len(maps))
            st.map_progress = 1.0
            for r in range(R):
                if lj.killed.is_set():
                    raise RuntimeError("job killed")
                aid = TaskAttemptID(TaskID(jid, False, r), 0)
                rt = ReduceTask(job, aid, r, len(maps))
                for m, path in zip(maps, outputs):
                    rt.add_map_output(MapOutputLocation(m.attempt_id, path))
                rt.run(os.path.join(local_root, str(aid)))
                lj.reduce_reports.append(TaskReport(aid.task, 1.0, SUCCEEDED, rt.start_time,
                                                    rt.finish_time, rt.reporter.counters))
                lj._counters.incr_all(rt.reporter.counters)
                st.reduce_progress = (r + 1) / R
            if R:
                lj._counters.incr(C.JOB_GROUP, C.TOTAL_LAUNCHED_REDUCES, R)
            st.reduce_progress = 1.0
            committer.commit_job(job)
            st.cleanup_progress = 1.0
            st.state = SUCCEEDED
        except BaseException as e:  # noqa: BLE001
            log.exception("job %s failed", st.job_id)
            st.failure_info = f"{type(e).__name__}: {e}"
            st.state = FAILED
            try:
                committer.abort_job(job)
            except Exception:
                pass
        finally:
            st.finish_time = time.time()
            shutil.rmtree(local_root, ignore_errors=True)
            lj._done.set()
