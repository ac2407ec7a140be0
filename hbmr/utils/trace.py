"""Structured event tracing for the control plane and the GPU runtime.

A process-wide, lock-free-ish (list.append under the GIL) event recorder with
near-zero cost when disabled (call sites test ``TRACE.on``).  Events are
(ts_ns, thread, phase, name, dur_ns, args):

* ``TRACE.instant(name, **args)``       point event
* ``with TRACE.span(name, **args):``    duration event
* ``TRACE.complete(name, t0_ns, t1_ns, **args)``  duration measured elsewhere
  (e.g. a GPU batch bracketed by HIP events, on a ``gpuN/slotM`` track)

Exports: JSON lines (one event per line — the per-task event log of SURVEY.md
§5) and the Chrome trace-event format (open in Perfetto / chrome://tracing):
CPU and GPU tracks side by side, map tasks coloured by where they ran.

Enable with ``HBMR_TRACE=1`` (or ``=path.json`` to dump at exit), or
``hbmr.trace.enabled=true`` in a daemon's configuration.  The reference's
equivalent is scattered ``LOG.info("DEBUG: ...")`` timing lines
(PipesGPUMapRunner.java:110-112, MapTask.java:443-451,
JobQueueTaskScheduler.java:150-161) plus JobHistory.
"""
from __future__ import annotations

import atexit
import json
import os
import threading
import time
from contextlib import contextmanager

_now = time.perf_counter_ns
# perf_counter has an arbitrary origin; anchor it to the wall clock once
_WALL0 = time.time_ns()
_PERF0 = _now()


def wall_ns(perf_ns: int) -> int:
    return _WALL0 + (perf_ns - _PERF0)


class _Roctx:
    """roctx markers (``HBMR_ROCTX=1``): every traced instant becomes a
    roctxMark and every span a roctxRangePush/Pop, so a ``rocprofv3
    --marker-trace`` timeline shows the control plane's events beside the
    kernels (libroctx64 from the ROCm install; silently off if absent)."""

    def __init__(self):
        self.lib = None
        if os.environ.get("HBMR_ROCTX") != "1":
            return
        import ctypes
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                self.lib = lib
                return
            except (OSError, AttributeError):
                continue

    def mark(self, name, args):
        self.lib.roctxMarkA(_label(name, args))

    def push(self, name, args):
        self.lib.roctxRangePushA(_label(name, args))

    def pop(self):
        self.lib.roctxRangePop()


def _label(name, args):
    if not args:
        return name.encode()
    return (name + " " + " ".join(f"{k}={v}" for k, v in args.items()))[:200].encode()


class Tracer:
    def __init__(self):
        self.on = False
        self.events: list = []
        self.max_events = 2_000_000
        self._dump_path = None
        self.roctx = _Roctx()
        if self.roctx.lib is not None:
            self.on = True

    def enable(self, dump_path: str | None = None):
        self.on = True
        if dump_path and self._dump_path is None:
            self._dump_path = dump_path
            atexit.register(self._dump_at_exit)

    def disable(self):
        self.on = False

    def clear(self):
        self.events = []

    # -- recording ------------------------------------------------------------------------
    def instant(self, name, **args):
        if self.on and len(self.events) < self.max_events:
            self.events.append((_now(), threading.current_thread().name, "i", name, 0, args))
            if self.roctx.lib is not None:
                self.roctx.mark(name, args)

    def complete(self, name, t0_ns, t1_ns, track=None, **args):
        if self.on and len(self.events) < self.max_events:
            self.events.append((t0_ns, track or threading.current_thread().name, "X", name,
                                max(0, t1_ns - t0_ns), args))

    @contextmanager
    def span(self, name, **args):
        if not self.on:
            yield
            return
        t0 = _now()
        rx = self.roctx.lib is not None
        if rx:
            self.roctx.push(name, args)
        try:
            yield
        finally:
            if rx:
                self.roctx.pop()
            self.complete(name, t0, _now(), **args)

    # -- queries --------------------------------------------------------------------------
    def find(self, name=None, since_ns=0):
        return [e for e in self.events if (name is None or e[3] == name) and e[0] >= since_ns]

    # -- export ---------------------------------------------------------------------------
    def to_jsonl(self, path):
        with open(path, "w") as f:
            for ts, th, ph, name, dur, args in self.events:
                rec = {"ts_us": wall_ns(ts) / 1e3, "mono_ns": ts, "thread": th, "ph": ph,
                       "name": name}
                if ph == "X":
                    rec["dur_us"] = dur / 1e3
                if args:
                    rec["args"] = args
                f.write(json.dumps(rec, default=str) + "\n")

    def to_chrome(self, path):
        tids: dict = {}
        out = []
        pid = os.getpid()
        for ts, th, ph, name, dur, args in self.events:
            tid = tids.setdefault(th, len(tids) + 1)
            ev = {"name": name, "ph": ph, "ts": wall_ns(ts) / 1e3, "pid": pid, "tid": tid}
            if ph == "X":
                ev["dur"] = dur / 1e3
            else:
                ev["s"] = "t"
            if args:
                ev["args"] = {k: (v if isinstance(v, (int, float, str, bool)) else str(v))
                              for k, v in args.items()}
                where = args.get("where")
                if where is not None:
                    # GPU map tasks green (the reference's TaskGraphServlet
                    # #00DD00), CPU map tasks blue (#AAAAFF)
                    ev["cname"] = "good" if str(where).startswith(("cuda", "gpu", "simgpu")) \
                        else "rail_idle"
            out.append(ev)
        for th, tid in tids.items():
            out.append({"name": "thread_name", "ph": "M", "pid": pid, "tid": tid,
                        "args": {"name": th}})
        with open(path, "w") as f:
            json.dump({"traceEvents": out, "displayTimeUnit": "ms"}, f)

    def _dump_at_exit(self):
        try:
            p = self._dump_path
            if p.endswith(".jsonl"):
                self.to_jsonl(p)
            else:
                self.to_chrome(p)
        except Exception:  # noqa: BLE001
            pass


TRACE = Tracer()

_env = os.environ.get("HBMR_TRACE", "")
if _env and _env != "0":
    # "{rank}" / "{pid}" in the path keep the dumps of a multi-process node
    # (ranks, GPU worker processes) apart
    TRACE.enable(None if _env == "1" else _env.replace("{rank}", os.environ.get("RANK", "0"))
                 .replace("{pid}", str(os.getpid())))


def configure(conf):
    """Daemons call this with their configuration (hbmr.trace.enabled / .file)."""
    if conf.get_boolean("hbmr.trace.enabled", False):
        TRACE.enable(conf.get("hbmr.trace.file"))
