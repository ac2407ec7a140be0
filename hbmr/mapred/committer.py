"""Two-phase task output commit (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/
FileOutputCommitter.java:41-121).

Each attempt writes under ``<out>/_temporary/_<attempt>/``; ``commit_task`` moves
its files into ``<out>`` (only the attempt the JobTracker allows to commit —
speculative duplicates are discarded), ``commit_job`` removes ``_temporary``
and drops the ``_SUCCESS`` marker.
"""
from __future__ import annotations

import os
import shutil

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
            os.makedirs(os.path.join(out, TEMP_DIR), exist_ok=True)

    def commit_job(self, job):
        out = self._out(job)
        if not out:
            return
        shutil.rmtree(os.path.join(out, TEMP_DIR), ignore_errors=True)
        if job.get_boolean("mapreduce.fileoutputcommitter.marksuccessfuljobs", True):
            open(os.path.join(out, SUCCEEDED_FILE), "wb").close()

    def abort_job(self, job, state="FAILED"):
        out = self._out(job)
        if out:
            shutil.rmtree(os.path.join(out, TEMP_DIR), ignore_errors=True)

    def setup_task(self, job, attempt):
        wp = self.work_path(job, attempt)
        if wp:
            os.makedirs(wp, exist_ok=True)

    def needs_task_commit(self, job, attempt) -> bool:
        wp = self.work_path(job, attempt)
        return bool(wp) and os.path.isdir(wp) and bool(os.listdir(wp))

    def commit_task(self, job, attempt):
        wp = self.work_path(job, attempt)
        out = self._out(job)
        if not wp or not os.path.isdir(wp):
            return
        for root, _dirs, files in os.walk(wp):
            rel = os.path.relpath(root, wp)
            dst_dir = out if rel == "." else os.path.join(out, rel)
            os.makedirs(dst_dir, exist_ok=True)
            for f in files:
                os.replace(os.path.join(root, f), os.path.join(dst_dir, f))
        shutil.rmtree(wp, ignore_errors=True)

    def abort_task(self, job, attempt):
        wp = self.work_path(job, attempt)
        if wp:
            shutil.rmtree(wp, ignore_errors=True)
