"""Metrics registry with Prometheus exposition and a file sink — the role of
hadoop-1.0.3 metrics2 (JobTrackerMetricsSource.java:33, TaskTrackerMetricsSource,
conf/hadoop-metrics2.properties file sink), SURVEY.md §5 "Metrics".

Counters and gauges are keyed by (name, sorted label pairs); incrementing is a
dict update under the GIL (no lock on the hot path).  ``prometheus_text()``
renders the text exposition format served at the web UI's ``/metrics``;
:class:`FileSink` appends a JSON snapshot every period
(``hbmr.metrics.file`` / ``hbmr.metrics.period.s``).
"""
from __future__ import annotations

import json
import threading
import time
import weakref


class Registry:
    def __init__(self):
        self.counters: dict = {}
        self.gauges: dict = {}
        self.help: dict = {}
        self.gauge_fns: list = []   # callables returning [(name, labels, value)]

    @staticmethod
    def _key(name, labels):
        return name, tuple(sorted((labels or {}).items()))

    def inc(self, name, amount=1, help="", **labels):  # noqa: A002
        k = self._key(name, labels)
        self.counters[k] = self.counters.get(k, 0) + amount
        if help and name not in self.help:
            self.help[name] = help

    def set(self, name, value, help="", **labels):  # noqa: A002
        self.gauges[self._key(name, labels)] = value
        if help and name not in self.help:
            self.help[name] = help

    def register_gauges(self, fn):
        """fn() -> iterable of (name, labels dict, value), sampled at scrape time.
        Bound methods are held weakly (a stopped daemon drops out)."""
        ref = weakref.WeakMethod(fn) if hasattr(fn, "__self__") else (lambda: fn)
        self.gauge_fns = [r for r in self.gauge_fns if r() is not None] + [ref]

    def _sampled(self):
        out = dict(self.gauges)
        for ref in list(self.gauge_fns):
            fn = ref()
            if fn is None:
                continue
            try:
                for name, labels, value in fn():
                    out[self._key(name, labels)] = value
            except Exception:  # noqa: BLE001
                pass
        return out

    def snapshot(self) -> dict:
        def flat(d):
            res = {}
            for (name, labels), v in d.items():
                key = name + ("{" + ",".join(f"{k}={v_}" for k, v_ in labels) + "}"
                              if labels else "")
                res[key] = v
            return res
        return {"ts": time.time(), "counters": flat(self.counters), "gauges": flat(self._sampled())}

    def prometheus_text(self) -> str:
        lines = []
        for kind, d in (("counter", self.counters), ("gauge", self._sampled())):
            names = sorted({k[0] for k in d})
            for name in names:
                if name in self.help:
                    lines.append(f"# HELP {name} {self.help[name]}")
                lines.append(f"# TYPE {name} {kind}")
                for (n, labels), v in sorted(d.items()):
                    if n != name:
                        continue
                    lab = "{" + ",".join(f'{k}="{v_}"' for k, v_ in labels) + "}" if labels else ""
                    lines.append(f"{name}{lab} {float(v)}")
        return "\n".join(lines) + "\n"


METRICS = Registry()


class FileSink:
    def __init__(self, registry: Registry, path: str, period: float = 10.0):
        self.reg, self.path, self.period = registry, path, period
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._loop, daemon=True, name="metrics-sink")

    def start(self):
        self.thread.start()
        return self

    def _loop(self):
        while not self._stop.wait(self.period):
            self.flush()

    def flush(self):
        with open(self.path, "a") as f:
            f.write(json.dumps(self.reg.snapshot()) + "\n")

    def stop(self):
        self._stop.set()
        self.flush()
