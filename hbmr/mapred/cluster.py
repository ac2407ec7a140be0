"""In-process node cluster: one JobTracker plus N TaskTrackers in this process.

The analogue of the reference's MiniMRCluster (src/test/org/apache/hadoop/
mapred/MiniMRCluster.java: JobTracker thread + N TaskTracker threads, each with
its own local dir and fake host name).  Used by tests and by single-process
runs (``mapred.job.tracker=inproc``).  Trackers share an
:class:`~hbmr.parallel.collectives.InProcessComm` so collective reduces run
the same code as the multi-process RCCL path.
"""
from __future__ import annotations

import logging
import tempfile

from ..parallel.collectives import InProcessComm, SoloComm
from .jobclient import RunningJob
from .jobconf import JobConf, as_jobconf
from .jobtracker import JobTracker
from .tasktracker import TaskTracker

log = logging.getLogger("hbmr.cluster")

_default = None


class LocalCluster:
    def __init__(self, conf=None, num_trackers=1, gpus=None, cpu_slots=None, reduce_slots=None,
                 gpu_slots_per_device=None, local_dir=None, hosts=None):
        """gpus: list per tracker of device ids, e.g. [[0], [1]]; None = CPU only.
        hosts: optional fake host name per tracker (rack-awareness tests)."""
        self.conf = as_jobconf(conf or JobConf())
        self.local_dir = local_dir or tempfile.mkdtemp(prefix="hbmr-cluster-")
        # like MiniMRCluster, each cluster gets its own mapred.system.dir unless the
        # caller named one: the stale-job sweep of a starting JobTracker must never
        # see another live cluster's job files
        if self.conf.get_raw("mapred.system.dir") == "${hadoop.tmp.dir}/mapred/system":
            self.conf.set("mapred.system.dir", f"{self.local_dir}/system")
        self.jt = JobTracker(self.conf)
        comms = InProcessComm.group(num_trackers) if num_trackers > 1 else [SoloComm()]
        gpus = gpus or [[] for _ in range(num_trackers)]
        self.trackers = []
        for i in range(num_trackers):
            tt = TaskTracker(self.conf, self.jt, name=f"tracker_{i}", rank=i,
                             world_size=num_trackers, gpu_devices=gpus[i], cpu_slots=cpu_slots,
                             reduce_slots=reduce_slots, gpu_slots_per_device=gpu_slots_per_device,
                             comm=comms[i], local_dir=f"{self.local_dir}/tt{i}",
                             host=hosts[i] if hosts else None)
            tt.all_trackers_local = True
            self.trackers.append(tt)
        for tt in self.trackers:
            tt.start()
        if not self.jt.wait_for_trackers(num_trackers, timeout=60):
            raise RuntimeError("trackers failed to register")
        self.jt.start_expiry_thread()

    def submit_job(self, job) -> RunningJob:
        rj = self.jt.submit_job(as_jobconf(job))
        return rj

    def job_result(self, rj: RunningJob, tracker=0):
        return self.trackers[tracker].job_result(rj.getID())

    def restart_jobtracker(self, conf=None):
        """Replace the JobTracker with a fresh one (MiniMRCluster.stopJobTracker +
        startJobTracker, as TestJobTrackerRestart does); the trackers keep running,
        are told to re-initialise and register again.  With
        mapred.jobtracker.restart.recover the new JT re-submits unfinished jobs."""
        old = self.jt
        old.shutdown()
        self.jt = JobTracker(as_jobconf(conf or self.conf))
        for tt in self.trackers:
            tt.jt = self.jt
            tt.notify_jobtracker()
        self.jt.start_expiry_thread()
        return self.jt

    def shutdown(self):
        for tt in self.trackers:
            tt.stop()
        self.jt.shutdown()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.shutdown()


def default_cluster(conf):
    global _default
    if _default is None:
        _default = LocalCluster(conf)
    return _default
