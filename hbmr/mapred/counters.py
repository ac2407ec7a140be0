"""Counters (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/Counters.java) with
the framework counter groups of Task.Counter (Task.java:73-90), JobInProgress
counters and the hbmr GPU/CPU placement counters."""
from __future__ import annotations

import threading

TASK_GROUP = "org.apache.hadoop.mapred.Task$Counter"
JOB_GROUP = "org.apache.hadoop.mapred.JobInProgress$Counter"
FS_GROUP = "FileSystemCounters"
GPU_GROUP = "hbmr.GpuCounters"

# Task$Counter names
MAP_INPUT_RECORDS = "MAP_INPUT_RECORDS"
MAP_OUTPUT_RECORDS = "MAP_OUTPUT_RECORDS"
MAP_OUTPUT_BYTES = "MAP_OUTPUT_BYTES"
MAP_INPUT_BYTES = "MAP_INPUT_BYTES"
MAP_SKIPPED_RECORDS = "MAP_SKIPPED_RECORDS"
COMBINE_INPUT_RECORDS = "COMBINE_INPUT_RECORDS"
COMBINE_OUTPUT_RECORDS = "COMBINE_OUTPUT_RECORDS"
REDUCE_INPUT_GROUPS = "REDUCE_INPUT_GROUPS"
REDUCE_SHUFFLE_BYTES = "REDUCE_SHUFFLE_BYTES"
REDUCE_INPUT_RECORDS = "REDUCE_INPUT_RECORDS"
REDUCE_OUTPUT_RECORDS = "REDUCE_OUTPUT_RECORDS"
REDUCE_SKIPPED_GROUPS = "REDUCE_SKIPPED_GROUPS"
REDUCE_SKIPPED_RECORDS = "REDUCE_SKIPPED_RECORDS"
SPILLED_RECORDS = "SPILLED_RECORDS"
SPLIT_RAW_BYTES = "SPLIT_RAW_BYTES"
CPU_MILLISECONDS = "CPU_MILLISECONDS"

# JobInProgress$Counter names
TOTAL_LAUNCHED_MAPS = "TOTAL_LAUNCHED_MAPS"
TOTAL_LAUNCHED_REDUCES = "TOTAL_LAUNCHED_REDUCES"
NUM_FAILED_MAPS = "NUM_FAILED_MAPS"
NUM_FAILED_REDUCES = "NUM_FAILED_REDUCES"
NUM_KILLED_MAPS = "NUM_KILLED_MAPS"
DATA_LOCAL_MAPS = "DATA_LOCAL_MAPS"
RACK_LOCAL_MAPS = "RACK_LOCAL_MAPS"
OTHER_LOCAL_MAPS = "OTHER_LOCAL_MAPS"
SLOTS_MILLIS_MAPS = "SLOTS_MILLIS_MAPS"
SLOTS_MILLIS_REDUCES = "SLOTS_MILLIS_REDUCES"

# FileSystemCounters
FILE_BYTES_READ = "FILE_BYTES_READ"
FILE_BYTES_WRITTEN = "FILE_BYTES_WRITTEN"

# hbmr GPU placement counters (the fork's finishedCPU/GPUMapTasks, JobInProgress.java:114-115)
CPU_MAP_TASKS = "CPU_MAP_TASKS"
GPU_MAP_TASKS = "GPU_MAP_TASKS"
GPU_KERNEL_MS = "GPU_KERNEL_MS"
GPU_H2D_BYTES = "GPU_H2D_BYTES"
GPU_D2H_BYTES = "GPU_D2H_BYTES"
GPU_SPLIT_CACHE_HITS = "GPU_SPLIT_CACHE_HITS"
GPU_SPLIT_CACHE_MISSES = "GPU_SPLIT_CACHE_MISSES"
COLLECTIVE_BYTES = "COLLECTIVE_BYTES"


class Counter:
    __slots__ = ("name", "display_name", "value")

    def __init__(self, name, display_name=None, value=0):
        self.name = name
        self.display_name = display_name or name
        self.value = value

    def increment(self, amount=1):
        self.value += amount

    def getValue(self):  # noqa: N802
        return self.value

    getCounter = getValue  # noqa: N815

    def __repr__(self):
        return f"{self.name}={self.value}"


class Group:
    def __init__(self, name, display_name=None):
        self.name = name
        self.display_name = display_name or name
        self.counters: dict[str, Counter] = {}

    def get(self, name) -> Counter:
        c = self.counters.get(name)
        if c is None:
            c = self.counters[name] = Counter(name)
        return c

    getCounterForName = get  # noqa: N815

    def __iter__(self):
        return iter(self.counters.values())

    def getCounter(self, name):  # noqa: N802
        c = self.counters.get(name)
        return c.value if c else 0


class Counters:
    def __init__(self):
        self.groups: dict[str, Group] = {}
        self._lock = threading.Lock()

    def group(self, name) -> Group:
        g = self.groups.get(name)
        if g is None:
            g = self.groups[name] = Group(name)
        return g

    getGroup = group  # noqa: N815

    def find_counter(self, group, name) -> Counter:
        return self.group(group).get(name)

    findCounter = find_counter  # noqa: N815

    def incr(self, group, name, amount=1):
        with self._lock:
            self.group(group).get(name).increment(amount)

    incrCounter = incr  # noqa: N815

    def get(self, group, name) -> int:
        g = self.groups.get(group)
        return g.getCounter(name) if g else 0

    def incr_all(self, other: "Counters"):
        with self._lock:
            for gname, g in other.groups.items():
                mine = self.group(gname)
                for c in g:
                    mine.get(c.name).increment(c.value)

    incrAllCounters = incr_all  # noqa: N815

    def incr_dicts(self, dicts):
        """Add counters given as ``{group: {name: value}}`` dicts (the wire
        form), without building a Counters object per dict."""
        with self._lock:
            groups = self.groups
            for d in dicts:
                if not d:
                    continue
                for gname, cs in d.items():
                    g = groups.get(gname)
                    if g is None:
                        g = groups[gname] = Group(gname)
                    gc = g.counters
                    for n, v in cs.items():
                        c = gc.get(n)
                        if c is None:
                            gc[n] = Counter(n, value=v)
                        else:
                            c.value += v

    def to_dict(self) -> dict:
        return {g: {c.name: c.value for c in grp} for g, grp in self.groups.items()}

    @classmethod
    def from_dict(cls, d: dict) -> "Counters":
        out = cls()
        for g, cs in (d or {}).items():
            for n, v in cs.items():
                out.group(g).get(n).value = v
        return out

    def __iter__(self):
        return iter(self.groups.values())

    def size(self):
        return sum(len(g.counters) for g in self.groups.values())

    def log(self, logger):
        logger.info("Counters: %d", self.size())
        for g in self:
            logger.info("  %s", g.display_name)
            for c in g:
                logger.info("    %s=%d", c.display_name, c.value)

    def __repr__(self):
        return f"Counters({self.to_dict()})"
