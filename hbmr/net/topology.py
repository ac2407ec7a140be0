"""Host → rack resolution (DNSToSwitchMapping).

Re-design of the reference's rack awareness: ``ScriptBasedMapping`` runs the
executable named by ``topology.script.file.name`` with up to
``topology.script.number.args`` host names as arguments and reads one rack path
per host from its stdout (hadoop-1.0.3/src/core/org/apache/hadoop/net/
ScriptBasedMapping.java:125-170); unknown hosts map to ``/default-rack``
(NetworkTopology.DEFAULT_RACK).  The JobTracker resolves each tracker once
(JobTracker.java:2708 resolveAndAddToTopology) and the scheduler prefers a
rack-local split before an off-rack one (JobInProgress.java:1537
obtainNewNodeOrRackLocalMapTask — the level the GPU fork dropped).

hbmr additions: a static table ``hbmr.topology.table`` ("host=/rack,...") for
clusters without a script, and a cache so a script runs once per host.
"""
from __future__ import annotations

import logging
import subprocess
import threading

log = logging.getLogger("hbmr.net")

DEFAULT_RACK = "/default-rack"


class Topology:
    def __init__(self, conf=None):
        self.script = conf.get("topology.script.file.name") if conf is not None else None
        self.max_args = max(1, conf.get_int("topology.script.number.args", 100)) if conf else 100
        self.table: dict[str, str] = {}
        spec = conf.get("hbmr.topology.table", "") if conf is not None else ""
        for item in (spec or "").split(","):
            if "=" in item:
                h, r = item.split("=", 1)
                self.table[h.strip()] = _norm(r.strip())
        self._cache: dict[str, str] = {}
        self._lock = threading.Lock()

    def resolve(self, hosts) -> list[str]:
        hosts = list(hosts)
        with self._lock:
            todo = [h for h in dict.fromkeys(hosts) if h not in self._cache]
            for h in list(todo):
                if h in self.table:
                    self._cache[h] = self.table[h]
                    todo.remove(h)
            if todo:
                if self.script:
                    for i in range(0, len(todo), self.max_args):
                        chunk = todo[i:i + self.max_args]
                        for h, r in zip(chunk, self._run_script(chunk)):
                            self._cache[h] = r
                else:
                    for h in todo:
                        self._cache[h] = DEFAULT_RACK
            return [self._cache[h] for h in hosts]

    def rack(self, host: str) -> str:
        return self.resolve([host])[0]

    def _run_script(self, hosts):
        try:
            out = subprocess.run([self.script, *hosts], capture_output=True, text=True,
                                 timeout=30, check=False).stdout.split()
        except (OSError, subprocess.SubprocessError) as e:
            log.warning("topology script %s failed: %s", self.script, e)
            out = []
        if len(out) != len(hosts):
            log.warning("topology script returned %d racks for %d hosts", len(out), len(hosts))
            return [DEFAULT_RACK] * len(hosts)
        return [_norm(r) for r in out]


def _norm(rack: str) -> str:
    rack = rack.strip() or DEFAULT_RACK
    return rack if rack.startswith("/") else "/" + rack
