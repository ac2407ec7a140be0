"""Device busy-time accounting for GPU map batches.

A batch of map tasks runs on one slot stream between two timing events; the
slots of a device are several streams, so batches of different slots overlap
on the device, and a staged batch's stream first waits for the gate of the job
it depends on (hbmr/gpu/gates.py).  The time the cost model should learn per
task (the GPU side of the reference's map-time estimate,
hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/JobInProgress.java:527-565)
is the device time the batch *adds*: the part of its interval that no other
charged batch already covers, from the moment its kernels could start.

:class:`BusyTimeline` keeps the union of charged intervals per device and
charges each new interval its uncovered length, whatever order the slot
completers report in — so the charges of a device's batches sum exactly to
the length of the union (the device's busy time), with no per-batch floor
(round 4 charged ``max(uncovered, elapsed / slots)``, which over-counted by
~1.6x against the kernel trace)."""
from __future__ import annotations

import bisect
import threading


class BusyTimeline:
    """Union of busy intervals [start, end) on one device (milliseconds on
    any common clock).  ``charge`` returns the part of a new interval that the
    union did not cover yet and adds the interval to it."""

    def __init__(self, keep: int = 256):
        self._starts: list[float] = []
        self._ends: list[float] = []
        self._keep = keep
        self._lock = threading.Lock()
        self.total = 0.0           # length of the union so far (charged in all)

    def charge(self, start: float, end: float) -> float:
        if end <= start:
            return 0.0
        with self._lock:
            st, en = self._starts, self._ends
            # merged intervals overlapping or touching [start, end]
            i = bisect.bisect_left(en, start)
            j = bisect.bisect_right(st, end)
            covered = 0.0
            for k in range(i, j):
                covered += max(0.0, min(end, en[k]) - max(start, st[k]))
            new_s = min(start, st[i]) if i < j else start
            new_e = max(end, en[j - 1]) if i < j else end
            st[i:j] = [new_s]
            en[i:j] = [new_e]
            if len(st) > self._keep:
                # the oldest intervals are final: a batch that old has reported
                del st[: len(st) - self._keep]
                del en[: len(en) - self._keep]
            add = (end - start) - covered
            self.total += add
            return add


def batch_interval(ev0_ms: float, elapsed_ms: float, gate_ms=()) -> tuple[float, float]:
    """[start, end) of a batch on the device clock: its start event at
    ``ev0_ms``, ``elapsed_ms`` to its end event, and the times its stream's
    gate events fired (``gate_ms``): time the stream spent waiting for a gate
    is not the batch's (its start is the latest of the start event and the
    gates)."""
    end = ev0_ms + elapsed_ms
    start = max([ev0_ms, *gate_ms])
    return min(start, end), end
