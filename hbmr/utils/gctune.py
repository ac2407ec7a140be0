"""Garbage-collector settings for the long-running control-plane processes
(JobTracker, TaskTracker, GPU worker).

Each iteration job allocates thousands of short-lived objects (TIPs, attempts,
statuses, messages).  With CPython's defaults (thresholds 700/10/10) a
K-Means bench run did ~8 gen-0 and ~0.75 gen-1 collections per job plus a
full collection every ~15 jobs that scanned every object of the process —
torch's modules included — for ~60 ms with the GIL held: jitter of a whole
job's length at one GPU.  ``tune()`` moves the objects that exist after
start-up (imports, configuration, the cluster's fixed state) into the
permanent generation (``gc.freeze``) so collections no longer scan them, and
raises the gen-0 threshold so collections come less often.  Reference
cycles are still collected.

``HBMR_GC_THRESHOLD=a,b,c`` overrides the thresholds; ``HBMR_GC_TUNE=0``
leaves the collector alone."""
from __future__ import annotations

import gc
import os

DEFAULT = (20000, 20, 20)


def tune():
    if os.environ.get("HBMR_GC_TUNE", "1") == "0":
        return
    th = DEFAULT
    env = os.environ.get("HBMR_GC_THRESHOLD")
    if env:
        try:
            th = tuple(int(x) for x in env.split(","))[:3]
        except ValueError:
            pass
    gc.collect()
    gc.freeze()
    gc.set_threshold(*th)
