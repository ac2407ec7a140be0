"""JobClient / RunningJob (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/JobClient.java).

``JobClient.runJob(conf)`` submits and waits (JobClient.java:1259, monitorAndPrintJob
:1281); ``submitJob`` returns a :class:`RunningJob` handle.  ``mapred.job.tracker``
selects the runner exactly as JobClient.init does (JobClient.java:465-476):

* ``local``                    → :class:`hbmr.mapred.local_runner.LocalJobRunner`
                                 (in-process, serial — BASELINE config 1);
* ``inproc`` / a cluster object → the in-process node cluster
                                 (:mod:`hbmr.mapred.cluster`, JobTracker +
                                 TaskTrackers with CPU and GPU slots);
* ``host:port``                → the JobTracker RPC server of a running node.
"""
from __future__ import annotations

import logging
import threading
import time

from .counters import Counters
from .jobconf import JobConf, as_jobconf

log = logging.getLogger("hbmr.jobclient")

PREP, RUNNING, SUCCEEDED, FAILED, KILLED = "PREP", "RUNNING", "SUCCEEDED", "FAILED", "KILLED"


class JobStatus:
    def __init__(self, job_id, state=PREP):
        self.job_id = job_id
        self.state = state
        self.map_progress = 0.0
        self.reduce_progress = 0.0
        self.setup_progress = 0.0
        self.cleanup_progress = 0.0
        self.start_time = time.time()
        self.finish_time = 0.0
        self.failure_info = ""

    def is_complete(self):
        return self.state in (SUCCEEDED, FAILED, KILLED)


class RunningJob:
    """Client-side handle. Backed by a ``job_impl`` exposing status(),
    counters(), kill(), wait(timeout) and task_reports()."""

    def __init__(self, job_id, impl, conf):
        self.job_id = job_id
        self._impl = impl
        self.conf = conf

    def getID(self):  # noqa: N802
        return self.job_id

    getJobID = getID  # noqa: N815

    def getJobName(self):  # noqa: N802
        return self.conf.get_job_name()

    def status(self) -> JobStatus:
        return self._impl.status()

    def mapProgress(self):  # noqa: N802
        return self.status().map_progress

    def reduceProgress(self):  # noqa: N802
        return self.status().reduce_progress

    def isComplete(self):  # noqa: N802
        return self.status().is_complete()

    def isSuccessful(self):  # noqa: N802
        return self.status().state == SUCCEEDED

    def getJobState(self):  # noqa: N802
        return self.status().state

    def waitForCompletion(self, timeout=None):  # noqa: N802
        return self._impl.wait(timeout)

    def killJob(self):  # noqa: N802
        self._impl.kill()

    def getCounters(self) -> Counters:  # noqa: N802
        return self._impl.counters()

    def getTaskReports(self, is_map=True):  # noqa: N802
        return self._impl.task_reports(is_map)

    def getFailureInfo(self):  # noqa: N802
        return self.status().failure_info

    def makespan(self) -> float:
        s = self.status()
        return (s.finish_time or time.time()) - s.start_time


class JobClient:
    def __init__(self, conf=None, cluster=None):
        self.conf = as_jobconf(conf or JobConf())
        self.cluster = cluster
        self._runner = None

    def _get_runner(self):
        if self._runner is not None:
            return self._runner
        if self.cluster is not None:
            self._runner = self.cluster
            return self._runner
        tracker = self.conf.get("mapred.job.tracker", "local")
        if tracker == "local":
            from .local_runner import LocalJobRunner
            self._runner = LocalJobRunner(self.conf)
        elif tracker == "inproc":
            from .cluster import default_cluster
            self._runner = default_cluster(self.conf)
        else:
            from .rpc import JobTrackerClient
            self._runner = JobTrackerClient(tracker, self.conf)
        return self._runner

    def submitJob(self, job) -> RunningJob:  # noqa: N802
        job = as_jobconf(job)
        return self._get_runner().submit_job(job)

    submit_job = submitJob

    @classmethod
    def runJob(cls, job, cluster=None, verbose=True) -> RunningJob:  # noqa: N802
        """Submit, wait, print progress + counters; raise if the job failed."""
        job = as_jobconf(job)
        client = cls(job, cluster=cluster)
        rj = client.submitJob(job)
        if not client.monitor_and_print_job(job, rj, verbose=verbose):
            raise RuntimeError(f"Job failed: {rj.getID()} {rj.getFailureInfo()}")
        return rj

    run_job = runJob

    def monitor_and_print_job(self, job, rj: RunningJob, verbose=True, poll=0.05) -> bool:
        last = None
        while True:
            done = rj.waitForCompletion(timeout=poll)
            st = rj.status()
            report = f" map {int(st.map_progress * 100)}% reduce {int(st.reduce_progress * 100)}%"
            if verbose and report != last:
                log.info(report)
                last = report
            if done or st.is_complete():
                break
        ok = rj.isSuccessful()
        if verbose:
            log.info("Job complete: %s (%s)", rj.getID(), rj.getJobState())
            rj.getCounters().log(log)
        return ok

    monitorAndPrintJob = monitor_and_print_job  # noqa: N815


class _Waitable:
    """Small helper for job implementations: a completion event + status."""

    def __init__(self, job_id):
        self._status = JobStatus(job_id)
        self._done = threading.Event()
        self._counters = Counters()

    def status(self):
        return self._status

    def counters(self):
        return self._counters

    def wait(self, timeout=None):
        return self._done.wait(timeout)
