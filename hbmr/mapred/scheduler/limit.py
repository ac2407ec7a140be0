"""LimitTasksPerJobTaskScheduler, GPU-aware.

The reference's variant of the FIFO scheduler caps the number of running tasks
of every job at ``mapred.jobtracker.scheduler.maxRunningTasksPerJob``
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/
LimitTasksPerJobTaskScheduler.java:38-200) and treats GPU slots as generic map
slots (:145).  Here the cap applies on top of the hybrid CPU/GPU
placement of :class:`HybridTaskScheduler`; ``hbmr.scheduler.maxRunningGpuTasksPerJob``
optionally caps the GPU attempts of a job separately, so one job cannot take
every GPU slot of the cluster.
"""
from __future__ import annotations

from .hybrid import HybridTaskScheduler


class LimitTasksPerJobTaskScheduler(HybridTaskScheduler):
    def __init__(self, jt, conf):
        super().__init__(jt, conf)
        lim = conf.get_int("mapred.jobtracker.scheduler.maxRunningTasksPerJob", 1 << 30)
        self.max_running = lim if lim > 0 else 1 << 30
        glim = conf.get_int("hbmr.scheduler.maxRunningGpuTasksPerJob", 0)
        self.max_gpu = glim if glim > 0 else 1 << 30

    def _running(self, jip):
        reduces = sum(1 for t in jip.reduces if t.is_running())
        return jip.running_maps() + reduces

    def job_limit(self, jip, kind) -> int:
        left = max(0, self.max_running - self._running(jip))
        if kind == "gpu":
            left = min(left, max(0, self.max_gpu - jip.running_maps(on_gpu=True)))
        return left
