"""One persistent Pipes child per (GPU executable, device), serving the map
tasks of that device as a FIFO with several RUN_MAPs in flight.

The reference runs a GPU map as a Pipes child of its own
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/pipes/PipesGPUMapRunner.java
:66-118 builds an Application per attempt and waits for it; Application.java
:130-215 starts the binary; HadoopPipes.cc:1093-1146 is the child's task
loop).  Per map that costs a process start (or, with hbmr.pipes.child.reuse,
a socket round trip between one map's DONE and the next RUN_MAP) on top of a
device map of ~0.1 ms.  Here the map attempts of one device share one child:
each attempt's thread appends its task (SET_JOB_CONF with the attempt's own
conf — once per job for apps that declare hbmr.pipes.gpu.mux.shared.conf —
then RUN_MAP) to the child's command stream without waiting for the previous map,
up to ``hbmr.pipes.gpu.queue.depth`` maps in flight, and the uplink reader
hands the child's messages to the head of the FIFO — the child runs its maps
back to back (its runtime reads the next command as soon as a map is DONE),
and the device state it keeps (HBM-resident splits, the job's centroid
image) serves every one of them.

Used by PipesGPUMapRunner for child-read input (hadoop.pipes.java.recordreader
false) with ``hbmr.pipes.gpu.mux`` (default true)."""
from __future__ import annotations

import collections
import logging
import threading

from ..utils.trace import TRACE
from .application import Application, OutputHandler

log = logging.getLogger("hbmr.pipes")

MUX = "hbmr.pipes.gpu.mux"
DEPTH = "hbmr.pipes.gpu.queue.depth"
# an app that reads only job-level keys from its JobConf may take the conf
# once per job; by default every attempt's own conf (its mapred.task.id,
# partition, work output dir, input file ...) goes down with its RUN_MAP, as
# the reference's per-attempt Application gives each child its own
# (PipesGPUMapRunner.java:66-79)
SHARED_CONF = "hbmr.pipes.gpu.mux.shared.conf"
TASK_KEYS = ("mapred.task.id", "mapred.tip.id", "mapred.task.partition", "mapred.task.is.map",
             "mapred.work.output.dir", "mapred.output.dir", "map.input.file",
             "map.input.start", "map.input.length")


def _job_key(job):
    """The job an attempt's conf belongs to (from its mapred.task.id)."""
    tid = job.get("mapred.task.id") or ""
    parts = tid.split("_")
    if len(parts) >= 3 and parts[0] == "attempt":
        return "_".join(parts[1:3])
    return job.get("mapred.job.id") or id(job)


class _Ticket:
    """One map's place in the child's FIFO."""

    def __init__(self, handler, job_id):
        self.handler = handler
        self.job_id = job_id


class _FifoHandler:
    """The uplink's handler: every message goes to the task at the head of
    the FIFO; DONE completes it and moves on to the next."""

    def __init__(self, mux):
        self.mux = mux
        # authentication happens before any task
        self.boot = OutputHandler(None, None, None, None)

    def _head(self):
        q = self.mux.fifo
        return q[0].handler if q else self.boot

    def output(self, k, v):
        self._head().output(k, v)

    def partitioned_output(self, part, k, v):
        self._head().partitioned_output(part, k, v)

    def status(self, msg):
        self._head().status(msg)

    def progress(self, p):
        self._head().progress(p)

    def register_counter(self, cid, group, name):
        self._head().register_counter(cid, group, name)

    def increment_counter(self, cid, amount):
        self._head().increment_counter(cid, amount)

    def authenticate(self, digest):
        self.boot.authenticate(digest)

    def done(self):
        if TRACE.on:
            TRACE.instant("pipes.mux.done")
        with self.mux.cond:
            t = self.mux.fifo.popleft() if self.mux.fifo else None
            self.mux.cond.notify_all()
        (t.handler if t is not None else self.boot).done()

    def failed(self, e):
        with self.mux.cond:
            pending = list(self.mux.fifo)
            self.mux.fifo.clear()
            self.mux.dead = e
            self.mux.cond.notify_all()
        for t in pending:
            t.handler.failed(e)
        self.boot.failed(e)


class _Pending:
    """The handler of a map sent to the child ahead of its task thread
    (MuxChild.prelaunch): the child's messages for it are kept until the
    thread attaches its own OutputHandler, then replayed in order and
    forwarded from there on."""

    def __init__(self):
        self.lock = threading.Lock()
        self.target = None
        self.buf: list = []

    def _call(self, name, *args):
        with self.lock:
            t = self.target
            if t is None:
                self.buf.append((name, args))
                return
        getattr(t, name)(*args)

    def output(self, k, v):
        self._call("output", k, v)

    def partitioned_output(self, part, k, v):
        self._call("partitioned_output", part, k, v)

    def status(self, msg):
        self._call("status", msg)

    def progress(self, p):
        self._call("progress", p)

    def register_counter(self, cid, group, name):
        self._call("register_counter", cid, group, name)

    def increment_counter(self, cid, amount):
        self._call("increment_counter", cid, amount)

    def done(self):
        self._call("done")

    def failed(self, e):
        self._call("failed", e)

    def attach(self, handler):
        # (under the lock: a message arriving meanwhile waits for the replay)
        with self.lock:
            for name, args in self.buf:
                getattr(handler, name)(*args)
            self.buf = []
            self.target = handler


class MuxChild:
    """A reused GPU Pipes child shared by the map attempts of one device."""

    def __init__(self, job, executable, device, work_dir, depth):
        self.depth = max(1, depth)
        self.fifo: collections.deque = collections.deque()
        self.cond = threading.Condition()
        self.dead = None
        self.send_lock = threading.Lock()
        self.conf_job = None
        self.maps = 0
        # the child is started like any reused Pipes child, then its uplink
        # is switched to the FIFO dispatcher
        job.set_boolean("hbmr.pipes.child.reuse", True)
        self.app = Application(job, None, None, None, None, executable, run_on_gpu=True,
                               gpu_device_id=device, work_dir=work_dir, reuse=True)
        # (the Application's start sent this attempt's conf)
        self.conf_job = _job_key(job) if job.get_boolean(SHARED_CONF, False) else \
            (_job_key(job),) + tuple(job.get(k) for k in TASK_KEYS)
        self.dispatch = _FifoHandler(self)
        self.app.uplink.handler = self.dispatch

    def alive(self):
        return self.dead is None and self.app.alive()

    def submit(self, job, collector, reporter, key_class, value_class, partitioner, split,
               num_reduces):
        """Queue one map (blocks while ``depth`` maps are in flight)."""
        h = OutputHandler(collector, reporter, key_class, value_class, partitioner)
        if TRACE.on:
            TRACE.instant("pipes.mux.submit")
        with self.send_lock:
            # the depth check and the FIFO append in one critical section (and
            # under send_lock, so the FIFO order is the command order): two
            # attempts can no longer both pass a full FIFO's check
            with self.cond:
                while len(self.fifo) >= self.depth and self.dead is None:
                    self.cond.wait()
                if self.dead is not None:
                    raise RuntimeError(f"pipes child failed: {self.dead}")
                t = _Ticket(h, _job_key(job))
                self.fifo.append(t)
            # the child's task loop keeps the last SET_JOB_CONF: it is resent
            # whenever the conf the child would see differs (every attempt has
            # its own task keys) unless the app shares one conf per job
            jid = t.job_id
            key = jid if job.get_boolean(SHARED_CONF, False) else \
                (jid,) + tuple(job.get(k) for k in TASK_KEYS)
            try:
                if key != self.conf_job:
                    job.set_boolean("hbmr.pipes.child.reuse", True)
                    self.app.downlink.set_job_conf(job)
                    self.conf_job = key
                    if TRACE.on:
                        TRACE.instant("pipes.mux.conf_sent")
                self.app.downlink.run_map(split, num_reduces, False)
            except OSError as e:
                # the child is gone (its uplink reader fails the FIFO): say why
                with self.cond:
                    if t in self.fifo:
                        self.fifo.remove(t)
                    self.dead = self.dead or e
                    self.cond.notify_all()
                raise RuntimeError(f"pipes child failed: {e}; {self.app._stderr_tail()}") from e
            self.maps += 1
            if TRACE.on:
                TRACE.instant("pipes.mux.run_map_sent", fifo=len(self.fifo))
        return t

    def prelaunch(self, job, split, num_reduces):
        """Send a map to the child now, before its task thread exists (the
        TaskTracker, for every attempt of a bulk launch): the child starts
        on it while the threads set their tasks up (config 2's 8 maps were
        ~0.3 ms of Python each, one after another under the GIL, ahead of
        their RUN_MAPs).  Its messages are held by a _Pending handler until
        PipesGPUMapRunner attaches its own.  None (nothing sent) when the
        FIFO is full: that map takes the ordinary submit path."""
        h = _Pending()
        with self.send_lock:
            with self.cond:
                if len(self.fifo) >= self.depth or self.dead is not None:
                    return None
                t = _Ticket(h, _job_key(job))
                self.fifo.append(t)
            jid = t.job_id
            key = jid if job.get_boolean(SHARED_CONF, False) else \
                (jid,) + tuple(job.get(k) for k in TASK_KEYS)
            try:
                if key != self.conf_job:
                    job.set_boolean("hbmr.pipes.child.reuse", True)
                    self.app.downlink.set_job_conf(job)
                    self.conf_job = key
                self.app.downlink.run_map(split, num_reduces, False)
                self.app.downlink.flush()
            except OSError as e:
                with self.cond:
                    if t in self.fifo:
                        self.fifo.remove(t)
                    self.dead = self.dead or e
                    self.cond.notify_all()
                return None
            self.maps += 1
        if TRACE.on:
            TRACE.instant("pipes.mux.prelaunched")
        return t

    def wait(self, ticket):
        try:
            ticket.handler.wait_for_finish()
        except BaseException as e:
            raise RuntimeError(f"pipes child failed: {e}; {self.app._stderr_tail()}") from e

    def close(self):
        try:
            self.app.close_child()
        except Exception:  # noqa: BLE001
            pass


class MuxRegistry:
    """The live MuxChild per (executable, device) of this process."""

    def __init__(self):
        self._lock = threading.Lock()
        self._children: dict = {}

    def get(self, job, executable, device, work_dir, depth):
        key = (executable, device)
        with self._lock:
            m = self._children.get(key)
            if m is not None and not m.alive():
                m.close()
                m = None
            if m is None:
                wd = work_dir() if callable(work_dir) else work_dir
                m = self._children[key] = MuxChild(job, executable, device, wd, depth)
            return m

    def close_all(self):
        with self._lock:
            ms = list(self._children.values())
            self._children.clear()
        for m in ms:
            m.close()


REGISTRY = MuxRegistry()

# attempt id -> (MuxChild, ticket) of the maps sent ahead of their threads
PRELAUNCHED: dict = {}
PRELAUNCH = "hbmr.pipes.gpu.prelaunch"
