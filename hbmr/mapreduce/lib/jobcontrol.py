"""New-API job control (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapreduce/lib/
jobcontrol/{ControlledJob,JobControl}.java): a DAG of new-API ``Job``s run by
a JobControl thread; a job is submitted when every job it depends on
succeeded and becomes DEPENDENT_FAILED when one of them failed.  Same state
machine as :mod:`hbmr.mapred.jobcontrol` (the old-API twin), over
``Job.submit()`` / ``isComplete()`` / ``isSuccessful()``."""
from __future__ import annotations

import threading
import time

from ...mapred import jobcontrol as _old

State = type("State", (), {s: s for s in ("WAITING", "READY", "RUNNING", "SUCCESS", "FAILED",
                                          "DEPENDENT_FAILED")})


class ControlledJob:
    CREATE_DIR = "mapreduce.jobcontrol.createdir.ifnotexist"

    def __init__(self, job_or_conf, depending=None):
        from ..job import Job
        self.job = job_or_conf if isinstance(job_or_conf, Job) else Job(job_or_conf)
        self.depending = list(depending or [])
        self.state = State.WAITING
        self.message = "just initialized"
        self.control_id = "unassigned"

    # -- accessors (ControlledJob.java) --------------------------------------------------
    def getJob(self):  # noqa: N802
        return self.job

    def getJobName(self):  # noqa: N802
        return self.job.getJobName()

    def setJobName(self, name):  # noqa: N802
        self.job.setJobName(name)

    def getJobID(self):  # noqa: N802
        return self.control_id

    def setJobID(self, i):  # noqa: N802
        self.control_id = i

    def getMapredJobID(self):  # noqa: N802
        return self.job.getJobID() if self.state != State.WAITING and \
            self.state != State.READY else None

    def getJobState(self):  # noqa: N802
        return self.state

    def getMessage(self):  # noqa: N802
        return self.message

    def setMessage(self, m):  # noqa: N802
        self.message = m

    def getDependentJobs(self):  # noqa: N802
        return list(self.depending) or None

    def addDependingJob(self, job):  # noqa: N802
        if self.state != State.WAITING:
            return False
        self.depending.append(job)
        return True

    def isCompleted(self):  # noqa: N802
        return self.state in (State.FAILED, State.DEPENDENT_FAILED, State.SUCCESS)

    def isReady(self):  # noqa: N802
        return self.state == State.READY

    def killJob(self):  # noqa: N802
        self.job.killJob()

    def failJob(self, message):  # noqa: N802
        if self.state == State.RUNNING:
            try:
                self.job.killJob()
            except Exception:  # noqa: BLE001
                pass
        self.state = State.FAILED
        self.message = message

    # -- state machine ---------------------------------------------------------------------
    def _check(self):
        if self.state == State.RUNNING:
            if self.job.isComplete():
                if self.job.isSuccessful():
                    self.state = State.SUCCESS
                else:
                    self.state = State.FAILED
                    self.message = "Job failed!"
        elif self.state == State.WAITING:
            if any(d.state in (State.FAILED, State.DEPENDENT_FAILED) for d in self.depending):
                self.state = State.DEPENDENT_FAILED
                self.message = "depending job failed"
            elif all(d.state == State.SUCCESS for d in self.depending):
                self.state = State.READY
        return self.state

    def submit(self):
        try:
            conf = self.job.getConfiguration()
            if conf.get_boolean(self.CREATE_DIR, False):
                import os
                for p in (conf.get("mapred.input.dir") or "").split(","):
                    if p and "://" not in p:
                        os.makedirs(p, exist_ok=True)
            self.job.submit()
            self.state = State.RUNNING
        except Exception as e:  # noqa: BLE001
            self.state = State.FAILED
            self.message = f"{type(e).__name__}: {e}"


class JobControl(_old.JobControl):
    """addJob(s), then run() as a thread target; submits READY jobs until
    allFinished() or stop()."""

    def __init__(self, group_name="jobcontrol", poll=0.02):
        super().__init__(group_name, poll=poll)
        self._next = 0
        self._lock2 = threading.Lock()

    def addJob(self, job):  # noqa: N802
        with self._lock2:
            self._next += 1
            job.setJobID(f"{self.group}{self._next}")
        with self.lock:
            self.jobs.append(job)
        return job.getJobID()

    def addJobCollection(self, jobs):  # noqa: N802
        for j in jobs:
            self.addJob(j)

    def _in(self, state):
        with self.lock:
            return [j for j in self.jobs if j.state == state]

    def getFailedJobList(self):  # noqa: N802
        return self._in(State.FAILED) + self._in(State.DEPENDENT_FAILED)

    def getSuccessfulJobList(self):  # noqa: N802
        return self._in(State.SUCCESS)

    def getRunningJobList(self):  # noqa: N802
        return self._in(State.RUNNING)

    def getWaitingJobList(self):  # noqa: N802
        return self._in(State.WAITING)

    def getReadyJobsList(self):  # noqa: N802
        return self._in(State.READY)

    def run(self):
        while not self._stop.is_set():
            with self.lock:
                jobs = list(self.jobs)
            for j in jobs:
                if j._check() == State.READY:
                    j.submit()
            if self.allFinished():
                break
            time.sleep(self.poll)
