"""Job/task/attempt identifiers with Hadoop's string forms
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/{JobID,TaskID,TaskAttemptID}.java):

    job_<jtIdentifier>_<0001>
    task_<jtIdentifier>_<0001>_m_<000007>
    attempt_<jtIdentifier>_<0001>_m_<000007>_<0>
"""
from __future__ import annotations

import re


class _ID:
    """Immutable id with value semantics (eq / order / hash by its fields) and
    its Hadoop string form computed once; plain slots instead of a frozen
    dataclass (ids are built per task and attempt on the scheduling path)."""
    __slots__ = ()

    def _key(self):
        raise NotImplementedError

    def __eq__(self, o):
        return type(o) is type(self) and self._key() == o._key()

    def __lt__(self, o):
        return self._key() < o._key()

    def __le__(self, o):
        return self._key() <= o._key()

    def __gt__(self, o):
        return self._key() > o._key()

    def __ge__(self, o):
        return self._key() >= o._key()

    def __hash__(self):
        return hash(self._s)

    def __str__(self):
        return self._s

    def __setattr__(self, k, v):
        raise AttributeError(f"{type(self).__name__} is immutable")

    def __reduce__(self):
        return (type(self), self._key())


class JobID(_ID):
    __slots__ = ("jt", "id", "_s")

    def __init__(self, jt: str, id: int):  # noqa: A002
        object.__setattr__(self, "jt", jt)
        object.__setattr__(self, "id", id)
        object.__setattr__(self, "_s", f"job_{jt}_{id:04d}")

    def _key(self):
        return (self.jt, self.id)

    def __repr__(self):
        return f"JobID(jt={self.jt!r}, id={self.id!r})"

    @classmethod
    def for_name(cls, s: str) -> "JobID":
        m = re.fullmatch(r"job_(.+)_(\d+)", s)
        if not m:
            raise ValueError(f"bad JobID {s!r}")
        return cls(m.group(1), int(m.group(2)))

    forName = for_name  # noqa: N815


class TaskID(_ID):
    __slots__ = ("job", "is_map", "id", "_s")

    def __init__(self, job: JobID, is_map: bool, id: int, s: str | None = None):  # noqa: A002
        # ``s``: the string form when the caller has it (a job's TIPs are
        # built from one prefix)
        _set = object.__setattr__
        _set(self, "job", job)
        _set(self, "is_map", is_map)
        _set(self, "id", id)
        _set(self, "_s", s or f"task_{job.jt}_{job.id:04d}_{'m' if is_map else 'r'}_{id:06d}")

    def _key(self):
        return (self.job, self.is_map, self.id)

    def __repr__(self):
        return f"TaskID(job={self.job!r}, is_map={self.is_map!r}, id={self.id!r})"

    @classmethod
    def for_name(cls, s: str) -> "TaskID":
        m = re.fullmatch(r"task_(.+)_(\d+)_([mr])_(\d+)", s)
        if not m:
            raise ValueError(f"bad TaskID {s!r}")
        return cls(JobID(m.group(1), int(m.group(2))), m.group(3) == "m", int(m.group(4)))

    def isMap(self):  # noqa: N802
        return self.is_map


class TaskAttemptID(_ID):
    __slots__ = ("task", "id", "_s")

    def __init__(self, task: TaskID, id: int):  # noqa: A002
        object.__setattr__(self, "task", task)
        object.__setattr__(self, "id", id)
        object.__setattr__(self, "_s", "attempt" + task._s[4:] + f"_{id}")

    def _key(self):
        return (self.task, self.id)

    def __repr__(self):
        return f"TaskAttemptID(task={self.task!r}, id={self.id!r})"

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
