"""Job control: run a DAG of jobs with dependencies (hadoop-1.0.3 mapred/
jobcontrol/{Job,JobControl}.java).  A job becomes READY when all the jobs it
depends on succeeded, DEPENDENT_FAILED if any of them failed."""
from __future__ import annotations

import threading
import time

from .jobclient import JobClient

WAITING, READY, RUNNING, SUCCESS, FAILED, DEPENDENT_FAILED = (
    "WAITING", "READY", "RUNNING", "SUCCESS", "FAILED", "DEPENDENT_FAILED")


class ControlledJob:
    def __init__(self, conf, depending=None, name=None):
        self.conf = conf
        self.depending = list(depending or [])
        self.state = WAITING
        self.name = name or conf.get_job_name() or "job"
        self.running = None
        self.message = ""

    def addDependingJob(self, job):  # noqa: N802
        if self.state != WAITING:
            return False
        self.depending.append(job)
        return True

    def getState(self):  # noqa: N802
        return self.state

    def getJobName(self):  # noqa: N802
        return self.name

    def getMessage(self):  # noqa: N802
        return self.message

    def _check(self):
        if self.state == RUNNING:
            rj = self.running
            if rj.isComplete():
                if rj.isSuccessful():
                    self.state = SUCCESS
                else:
                    self.state = FAILED
                    self.message = rj.getFailureInfo()
        elif self.state == WAITING:
            if any(d.state in (FAILED, DEPENDENT_FAILED) for d in self.depending):
                self.state = DEPENDENT_FAILED
                self.message = "depending job failed"
            elif all(d.state == SUCCESS for d in self.depending):
                self.state = READY
        return self.state


Job = ControlledJob


class JobControl:
    """addJob(s), then run() (a thread target): submits READY jobs until stop()
    or allFinished()."""

    def __init__(self, group_name="jobcontrol", cluster=None, poll=0.02):
        self.group = group_name
        self.cluster = cluster
        self.poll = poll
        self.jobs: list[ControlledJob] = []
        self._stop = threading.Event()
        self.lock = threading.Lock()

    def addJob(self, job):  # noqa: N802
        with self.lock:
            self.jobs.append(job)
        return job.name

    def addJobs(self, jobs):  # noqa: N802
        for j in jobs:
            self.addJob(j)

    def _in(self, state):
        with self.lock:
            return [j for j in self.jobs if j.state == state]

    def getWaitingJobs(self):  # noqa: N802
        return self._in(WAITING)

    def getRunningJobs(self):  # noqa: N802
        return self._in(RUNNING)

    def getReadyJobs(self):  # noqa: N802
        return self._in(READY)

    def getSuccessfulJobs(self):  # noqa: N802
        return self._in(SUCCESS)

    def getFailedJobs(self):  # noqa: N802
        return self._in(FAILED) + self._in(DEPENDENT_FAILED)

    def allFinished(self):  # noqa: N802
        with self.lock:
            return all(j.state in (SUCCESS, FAILED, DEPENDENT_FAILED) for j in self.jobs)

    def stop(self):
        self._stop.set()

    def run(self):
        while not self._stop.is_set():
            with self.lock:
                jobs = list(self.jobs)
            for j in jobs:
                if j._check() == READY:
                    j.running = JobClient(j.conf, cluster=self.cluster).submitJob(j.conf)
                    j.state = RUNNING
            if self.allFinished():
                break
            time.sleep(self.poll)
