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


_MALLOC_TUNED = False


def tune_malloc():
    """glibc malloc: serve allocations below 64 MiB from the heap and keep up
    to 256 MiB of freed heap (M_MMAP_THRESHOLD / M_TRIM_THRESHOLD).  A Pipes
    map's output arrives as one ~1 MB value (a K-Means partials block at
    k = 1024) per map: with the defaults each such buffer could be a fresh
    mmap — its pages faulted in and zeroed on every map — in the uplink
    thread that serialises the maps of a device (a 1 MB socket read plus its
    copy took 0.39 ms with the defaults, 0.32 ms after; tools/gpu/r6_c3.sh).
    ``HBMR_MALLOC_TUNE=0`` leaves malloc alone."""
    global _MALLOC_TUNED
    if _MALLOC_TUNED or os.environ.get("HBMR_MALLOC_TUNE", "1") == "0":
        return
    _MALLOC_TUNED = True
    try:
        import ctypes
        libc = ctypes.CDLL("libc.so.6")
        libc.mallopt(-3, 64 << 20)     # M_MMAP_THRESHOLD
        libc.mallopt(-1, 256 << 20)    # M_TRIM_THRESHOLD
    except (OSError, AttributeError):
        pass


def tune():
    tune_malloc()
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
