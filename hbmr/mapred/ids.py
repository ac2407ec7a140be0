"""Job/task/attempt identifiers with Hadoop's string forms
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/{JobID,TaskID,TaskAttemptID}.java):

    job_<jtIdentifier>_<0001>
    task_<jtIdentifier>_<0001>_m_<000007>
    attempt_<jtIdentifier>_<0001>_m_<000007>_<0>
"""
from __future__ import annotations

import re
from dataclasses import dataclass


@dataclass(frozen=True, order=True)
class JobID:
    jt: str
    id: int

    def __post_init__(self):
        object.__setattr__(self, "_s", f"job_{self.jt}_{self.id:04d}")

    def __str__(self):
        return self._s

    @classmethod
    def for_name(cls, s: str) -> "JobID":
        m = re.fullmatch(r"job_(.+)_(\d+)", s)
        if not m:
            raise ValueError(f"bad JobID {s!r}")
        return cls(m.group(1), int(m.group(2)))

    forName = for_name  # noqa: N815


@dataclass(frozen=True, order=True)
class TaskID:
    job: JobID
    is_map: bool
    id: int

    def __post_init__(self):
        object.__setattr__(self, "_s", f"task_{self.job.jt}_{self.job.id:04d}_"
                                       f"{'m' if self.is_map else 'r'}_{self.id:06d}")

    def __str__(self):
        return self._s

    @classmethod
    def for_name(cls, s: str) -> "TaskID":
        m = re.fullmatch(r"task_(.+)_(\d+)_([mr])_(\d+)", s)
        if not m:
            raise ValueError(f"bad TaskID {s!r}")
        return cls(JobID(m.group(1), int(m.group(2))), m.group(3) == "m", int(m.group(4)))

    def isMap(self):  # noqa: N802
        return self.is_map


@dataclass(frozen=True, order=True)
class TaskAttemptID:
    task: TaskID
    id: int

    def __post_init__(self):
        object.__setattr__(self, "_s", "attempt" + str(self.task)[4:] + f"_{self.id}")

    def __str__(self):
        return self._s

    @property
    def job(self):
        return self.task.job

    @property
    def is_map(self):
        return self.task.is_map

    @classmethod
    def for_name(cls, s: str) -> "TaskAttemptID":
        m = re.fullmatch(r"attempt_(.+)_(\d+)_([mr])_(\d+)_(\d+)", s)
        if not m:
            raise ValueError(f"bad TaskAttemptID {s!r}")
        return cls(TaskID(JobID(m.group(1), int(m.group(2))), m.group(3) == "m",
                          int(m.group(4))), int(m.group(5)))
