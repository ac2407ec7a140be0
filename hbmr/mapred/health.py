"""Node health checking for a TaskTracker, extended to its GPUs.

Reference: NodeHealthCheckerService (hadoop-1.0.3/src/mapred/org/apache/hadoop/
mapred/NodeHealthCheckerService.java:42-380) runs the admin script
``mapred.healthChecker.script.path`` every ``mapred.healthChecker.interval`` ms
with ``mapred.healthChecker.script.args``; a line of output starting with
``ERROR`` marks the node unhealthy (the report is sent in the heartbeat and the
JobTracker stops giving the tracker tasks, JobTracker.java:3447-3460); a script
that times out (``mapred.healthChecker.script.timeout``) also marks it
unhealthy; a non-zero exit code alone does not.

GPU extension (no counterpart in the reference, where a dead GPU showed up only
as failing Pipes children): every check also probes each GPU of the tracker
(``runtime.probe(d)``: repeated device-level task errors, or a failed device
query).  A bad GPU is withdrawn from the heartbeat's device list — its slots
disappear from the cluster's GPU capacity — while the node itself stays
healthy and keeps its CPU and healthy-GPU slots.
"""
from __future__ import annotations

import logging
import subprocess
import threading
import time

log = logging.getLogger("hbmr.health")


class NodeHealthChecker:
    def __init__(self, conf, gpu_runtime=None):
        self.script = conf.get("mapred.healthChecker.script.path")
        self.interval = conf.get_int("mapred.healthChecker.interval", 60000) / 1000.0
        self.timeout = conf.get_int("mapred.healthChecker.script.timeout", 600000) / 1000.0
        self.args = conf.get_strings("mapred.healthChecker.script.args") or []
        self.runtime = gpu_runtime
        self.healthy = True
        self.report = ""
        self.bad_devices: dict[int, str] = {}
        self.last_check = 0.0
        self._running = False
        self._lock = threading.Lock()

    @property
    def enabled(self):
        return bool(self.script) or (self.runtime is not None and hasattr(self.runtime, "probe"))

    def check_now(self):
        healthy, report = True, ""
        if self.script:
            try:
                p = subprocess.run([self.script, *self.args], capture_output=True, text=True,
                                   timeout=self.timeout, check=False)
                for line in p.stdout.splitlines():
                    if line.startswith("ERROR"):
                        healthy, report = False, p.stdout.strip()[:2000]
                        break
            except subprocess.TimeoutExpired:
                healthy, report = False, "Node health script timed out"
            except OSError as e:
                # a missing / unrunnable script is the admin's problem, not the node's
                log.warning("health script %s could not run: %s", self.script, e)
        bad = {}
        if self.runtime is not None and hasattr(self.runtime, "probe"):
            for d in list(getattr(self.runtime, "devices", {})):
                why = self.runtime.probe(d)
                if why:
                    bad[d] = why
        with self._lock:
            if bad != self.bad_devices and bad:
                log.warning("GPU(s) marked unhealthy: %s", bad)
            self.healthy, self.report, self.bad_devices = healthy, report, bad
            self.last_check = time.time()

    def maybe_check(self, now=None):
        """Called from the heartbeat loop; the check itself runs on a side
        thread so a slow script never delays a heartbeat."""
        now = now or time.time()
        if not self.enabled or now - self.last_check < self.interval:
            return
        with self._lock:
            if self._running:
                return
            self._running = True
            self.last_check = now

        def run():
            try:
                self.check_now()
            finally:
                with self._lock:
                    self._running = False
        threading.Thread(target=run, name="health-check", daemon=True).start()

    def filter_gpus(self, gpus):
        """Drop unhealthy devices from a heartbeat's GPU status list."""
        with self._lock:
            bad = set(self.bad_devices)
        return [g for g in gpus if g["device"] not in bad] if bad else gpus

    def health_report(self):
        with self._lock:
            parts = [self.report] if self.report else []
            parts += [f"gpu{d}: {w}" for d, w in sorted(self.bad_devices.items())]
            return self.healthy, "; ".join(parts)
