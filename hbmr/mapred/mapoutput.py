"""Map outputs kept in the TaskTracker process's memory.

A map's sorted output is ``file.out`` + ``file.out.index`` under the attempt's
local dir (MapTask.java:1440-1621), served to reduces by the TaskTracker that
ran it (TaskTracker.MapOutputServlet).  Here, when every reduce of the job
reads its inputs in this same process (an in-process JobTracker — LocalCluster
— and no child-process tasks), a small map output (one spill, at most
``hbmr.map.output.memory.max.bytes``) is not written at all: its IFile bytes
and index stay in this store under the path the file would have had, and
MapOutputLocation.read_partition looks here first.  That drops the per-map
mkdir / open / write / close / rename / re-open of the local files, which is
most of a small map's cost on a slow local file system.

Fault semantics are those of the files: both live as long as the tracker that
holds them (a dead tracker's map outputs are re-executed either way).  Entries
go when the job is purged from the tracker (KillJobAction); the store is capped
(``hbmr.map.output.memory.total.bytes``) and a map whose output does not fit
writes its files as usual.
"""
from __future__ import annotations

import threading


class MemoryMapOutputs:
    def __init__(self, cap_bytes: int = 256 << 20):
        self.cap = cap_bytes
        self._d: dict[str, tuple[bytes, object]] = {}
        self._bytes = 0
        self._lock = threading.Lock()

    def put(self, path: str, data: bytes, index, cap: int | None = None) -> bool:
        """Hold ``data`` (the IFile segments) and its SpillRecord under
        ``path``; False (nothing held) if that would pass the cap."""
        n = len(data)
        with self._lock:
            limit = self.cap if cap is None else cap
            old = self._d.get(path)
            have = self._bytes - (len(old[0]) if old is not None else 0)
            if have + n > limit:
                return False
            self._d[path] = (data, index)
            self._bytes = have + n
        return True

    def get(self, path: str):
        return self._d.get(path)

    def drop_prefix(self, prefix: str) -> int:
        """Forget every output under ``prefix`` (a job's local dir)."""
        with self._lock:
            gone = [p for p in self._d if p.startswith(prefix)]
            for p in gone:
                self._bytes -= len(self._d.pop(p)[0])
        return len(gone)

    @property
    def bytes(self) -> int:
        return self._bytes

    def __len__(self):
        return len(self._d)


STORE = MemoryMapOutputs()

MAX_KEY = "hbmr.map.output.memory.max.bytes"
TOTAL_KEY = "hbmr.map.output.memory.total.bytes"
