"""Device-ordered hand-off between chained split jobs (pre-staged iterations).

A job W that depends on job J (``hbmr.job.depends.on``; e.g. K-Means iteration
i+1 on iteration i) needs J's reduce result — for K-Means the new centroid
image, which J's collective reduce leaves resident on every GPU.  The
reference can only start W after J has finished as a whole: a JobControl
driver polls J, then submits W, whose tasks reach a TaskTracker on its next
heartbeat (≥ 3 s apart, MRConstants.java:28; JobControl.java polls every 5 s).

Here the JobTracker *stages* W while J runs: W's GPU map attempts are launched
to the trackers early, marked with ``gate = J``.  The device runtime holds
them (:class:`Gates`) until J's reduce on that tracker has **enqueued** its
result on the device and opened the gate with a device event; the held maps
then go onto the slot streams behind a ``wait_event`` on that event.  So the
next iteration's assign kernels follow the previous reduce's update kernel in
device order, with no host round trip (JobTracker → tracker → worker) in
between; the JobTracker still records every attempt and only *completes* W
after J succeeded (JobTracker._finish_job).
"""
from __future__ import annotations

import threading


class Gates:
    """Held runs per gate job, and the gates already opened (job id → device
    event, or None when the result is ready on the host)."""

    def __init__(self, keep: int = 256):
        self._lock = threading.Lock()
        self._held: dict = {}
        self._open: dict = {}
        self._epoch: dict = {}      # job id → times its gate was closed
        self._keep = keep

    def admit(self, runs):
        """Runs that may be launched now (each with ``run.wait`` set to the
        event of its open gate, if any); gated runs of unopened gates are held."""
        now = []
        with self._lock:
            for r in runs:
                g = getattr(r.spec, "gate", None)
                if g is None:
                    now.append(r)
                elif g in self._open:
                    r.wait = self._open[g]
                    now.append(r)
                else:
                    self._held.setdefault(g, []).append(r)
        return now

    def epoch(self, job_id) -> int:
        """Taken by a reduce attempt when it starts; its ``open`` is ignored if
        the gate was closed since (a killed attempt of a restarted gang)."""
        with self._lock:
            return self._epoch.get(job_id, 0)

    def open(self, job_id, event=None, epoch=None):
        """Job ``job_id``'s result is enqueued (``event`` marks it on the
        device): returns the runs that were held for it, each with ``wait``."""
        with self._lock:
            if epoch is not None and epoch != self._epoch.get(job_id, 0):
                return []
            self._open.pop(job_id, None)
            self._open[job_id] = event
            while len(self._open) > self._keep:
                self._open.pop(next(iter(self._open)))
            held = self._held.pop(job_id, [])
        for r in held:
            r.wait = event
        return held

    def close(self, job_id):
        """Job ``job_id``'s reduce is re-run (its gang failed after opening
        the gate): runs gated on it are held again until the new reduce opens."""
        with self._lock:
            self._open.pop(job_id, None)
            self._epoch[job_id] = self._epoch.get(job_id, 0) + 1
            while len(self._epoch) > self._keep:
                self._epoch.pop(next(iter(self._epoch)))

    def is_open(self, job_id) -> bool:
        with self._lock:
            return job_id in self._open

    def held_count(self) -> int:
        with self._lock:
            return sum(len(v) for v in self._held.values())

    def drop(self, job_id):
        """Forget held runs of job ``job_id`` (killed / purged) — returns them."""
        out = []
        with self._lock:
            for g, rs in list(self._held.items()):
                keep = [r for r in rs if r.spec.job_id != job_id]
                out += [r for r in rs if r.spec.job_id == job_id]
                if keep:
                    self._held[g] = keep
                else:
                    del self._held[g]
        return out
