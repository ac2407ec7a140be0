"""Bad-record skipping (SkipBadRecords).

Reference: hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/SkipBadRecords.java
(configuration keys and defaults, :44-330) with the range narrowing of
SortedRanges / TaskInProgress.getSkipRanges.  After
``mapred.skip.attempts.to.start.skipping`` (2) failed attempts of a task, the
next attempts run in *skipping mode*; records (map) or key groups (reduce)
whose processing fails are skipped and appended to a SequenceFile under
``mapred.skip.out.dir`` (default ``<output>/_logs/skip``), up to
``mapred.skip.map.max.skip.records`` / ``mapred.skip.reduce.max.skip.groups``
(0 = skipping disabled).

Re-design: the reference needs many attempts to binary-search the bad range
because a crashing Pipes/streaming child gives no per-record signal; hbmr's
in-process map/reduce functions raise per record, so a skipping-mode attempt
isolates and skips exactly the failing records in one pass (counters
MAP_SKIPPED_RECORDS, REDUCE_SKIPPED_GROUPS, REDUCE_SKIPPED_RECORDS as in
Task.Counter).
"""
from __future__ import annotations

import os
import threading

from . import counters as C

ATTEMPTS_TO_START_SKIPPING = "mapred.skip.attempts.to.start.skipping"
AUTO_INCR_MAP_PROC_COUNT = "mapred.skip.map.auto.incr.proc.count"
AUTO_INCR_REDUCE_PROC_COUNT = "mapred.skip.reduce.auto.incr.proc.count"
OUT_PATH = "mapred.skip.out.dir"
MAPPER_MAX_SKIP_RECORDS = "mapred.skip.map.max.skip.records"
REDUCER_MAX_SKIP_GROUPS = "mapred.skip.reduce.max.skip.groups"

COUNTER_GROUP = "SkippingTaskCounters"
COUNTER_MAP_PROCESSED_RECORDS = "MapProcessedRecords"
COUNTER_REDUCE_PROCESSED_GROUPS = "ReduceProcessedGroups"


class SkipBadRecords:
    @staticmethod
    def getAttemptsToStartSkipping(conf):  # noqa: N802
        return conf.get_int(ATTEMPTS_TO_START_SKIPPING, 2)

    @staticmethod
    def setAttemptsToStartSkipping(conf, n):  # noqa: N802
        conf.set_int(ATTEMPTS_TO_START_SKIPPING, n)

    @staticmethod
    def getAutoIncrMapperProcCount(conf):  # noqa: N802
        return conf.get_boolean(AUTO_INCR_MAP_PROC_COUNT, True)

    @staticmethod
    def setAutoIncrMapperProcCount(conf, b):  # noqa: N802
        conf.set_boolean(AUTO_INCR_MAP_PROC_COUNT, b)

    @staticmethod
    def getAutoIncrReducerProcCount(conf):  # noqa: N802
        return conf.get_boolean(AUTO_INCR_REDUCE_PROC_COUNT, True)

    @staticmethod
    def setAutoIncrReducerProcCount(conf, b):  # noqa: N802
        conf.set_boolean(AUTO_INCR_REDUCE_PROC_COUNT, b)

    @staticmethod
    def getSkipOutputPath(conf):  # noqa: N802
        p = conf.get(OUT_PATH)
        if p == "none":
            return None
        if p:
            return p
        out = conf.get("mapred.output.dir")
        return os.path.join(out, "_logs", "skip") if out else None

    @staticmethod
    def setSkipOutputPath(conf, path):  # noqa: N802
        conf.set(OUT_PATH, "none" if path is None else str(path))

    @staticmethod
    def getMapperMaxSkipRecords(conf):  # noqa: N802
        return conf.get_int(MAPPER_MAX_SKIP_RECORDS, 0)

    @staticmethod
    def setMapperMaxSkipRecords(conf, n):  # noqa: N802
        conf.set_int(MAPPER_MAX_SKIP_RECORDS, n)

    @staticmethod
    def getReducerMaxSkipGroups(conf):  # noqa: N802
        return conf.get_int(REDUCER_MAX_SKIP_GROUPS, 0)

    @staticmethod
    def setReducerMaxSkipGroups(conf, n):  # noqa: N802
        conf.set_int(REDUCER_MAX_SKIP_GROUPS, n)


def _attempt_number(job):
    tid = job.get("mapred.task.id") or ""
    try:
        return int(tid.rsplit("_", 1)[1])
    except (IndexError, ValueError):
        return 0


def skipping_limit(job, is_map) -> int:
    """Max records/groups this attempt may skip (0 = not in skipping mode)."""
    lim = (SkipBadRecords.getMapperMaxSkipRecords(job) if is_map
           else SkipBadRecords.getReducerMaxSkipGroups(job))
    if lim <= 0:
        return 0
    if _attempt_number(job) < SkipBadRecords.getAttemptsToStartSkipping(job):
        return 0
    return lim


class SkipLog:
    """Appends skipped records to <skip dir>/<attempt> (a SequenceFile)."""

    def __init__(self, job, key_class, value_class):
        self.job = job
        self.kc, self.vc = key_class, value_class
        self.w = None
        self.n = 0
        self._lock = threading.Lock()

    def add(self, key, value):
        with self._lock:
            self.n += 1
            d = SkipBadRecords.getSkipOutputPath(self.job)
            if d is None or key is None:
                return
            try:
                if self.w is None:
                    from ..io import sequencefile as SF
                    os.makedirs(d, exist_ok=True)
                    self.w = SF.Writer(os.path.join(d, self.job.get("mapred.task.id", "task")),
                                       type(key), type(value))
                self.w.append(key, value)
            except (OSError, TypeError, AttributeError, NotImplementedError):
                pass   # skipped-record logging is best effort

    def close(self):
        if self.w is not None:
            self.w.close()
            self.w = None


def record_skip(reporter, is_map, n_records=1):
    if is_map:
        reporter.incrCounter(C.TASK_GROUP, "MAP_SKIPPED_RECORDS", n_records)
    else:
        reporter.incrCounter(C.TASK_GROUP, "REDUCE_SKIPPED_GROUPS", 1)
        reporter.incrCounter(C.TASK_GROUP, "REDUCE_SKIPPED_RECORDS", n_records)
