"""Two-phase task output commit (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/
FileOutputCommitter.java:41-121).

Each attempt writes under ``<out>/_temporary/_<attempt>/``; ``commit_task`` moves
its files into ``<out>`` (only the attempt the JobTracker allows to commit —
speculative duplicates are discarded), ``commit_job`` removes ``_temporary``
and drops the ``_SUCCESS`` marker.
"""
from __future__ import annotations

import os

from .. import fs as F
from .formats import get_output_path

TEMP_DIR = "_temporary"
SUCCEEDED_FILE = "_SUCCESS"


class OutputCommitter:
    def setup_job(self, job):
        pass

    def commit_job(self, job):
        pass

    def abort_job(self, job, state="FAILED"):
        pass

    def setup_task(self, job, attempt):
        pass

    def needs_task_commit(self, job, attempt) -> bool:
        return False

    def commit_task(self, job, attempt):
        pass

    def abort_task(self, job, attempt):
        pass


class FileOutputCommitter(OutputCommitter):
    def _out(self, job):
        return get_output_path(job)

    def work_path(self, job, attempt) -> str | None:
        out = self._out(job)
        if out is None:
            return None
        return os.path.join(out, TEMP_DIR, f"_{attempt}")

    def setup_job(self, job):
        out = self._out(job)
        if out:
            F.makedirs(os.path.join(out, TEMP_DIR))

    def commit_job(self, job):
        out = self._out(job)
        if not out:
            return
        F.rmtree(os.path.join(out, TEMP_DIR))
        if job.get_boolean("mapreduce.fileoutputcommitter.marksuccessfuljobs", True):
            F.fopen(os.path.join(out, SUCCEEDED_FILE), "wb").close()

    def abort_job(self, job, state="FAILED"):
        out = self._out(job)
        if out:
            F.rmtree(os.path.join(out, TEMP_DIR))

    def setup_task(self, job, attempt):
        # nothing, as in FileOutputCommitter.setupTask (FileOutputCommitter.java
        # :115-119): the attempt's work dir is made on demand by the first writer
        # (every RecordWriter makes its parent directories); a map whose output
        # goes to its local map-output files never creates one, which saves the
        # mkdir here and the listdir in needs_task_commit per map
        pass

    def needs_task_commit(self, job, attempt) -> bool:
        wp = self.work_path(job, attempt)
        return bool(wp) and F.isdir(wp) and bool(F.listdir(wp))

    def commit_task(self, job, attempt):
        wp = self.work_path(job, attempt)
        out = self._out(job)
        if not wp or not F.isdir(wp):
            return
        for rel in F.walk_files(wp):
            dst = os.path.join(out, rel)
            F.makedirs(os.path.dirname(dst))
            F.replace(os.path.join(wp, rel), dst)
        F.rmtree(wp)

    def abort_task(self, job, attempt):
        wp = self.work_path(job, attempt)
        if wp:
            F.rmtree(wp)
