"""Launch and drive one Pipes child process (hadoop-1.0.3/src/mapred/org/apache/
hadoop/mapred/pipes/Application.java + OutputHandler.java).

The parent opens a loopback server socket, exports its port as
``hadoop.pipes.command.port``, writes the job token to a private file named by
``hadoop.pipes.shared.secret.location``, starts the executable, accepts its
connection and authenticates it with an HMAC-SHA1 challenge.  A GPU attempt's
executable gets the scheduler-chosen device both as ``argv[1]`` (the fork's
convention, Application.java:178-181) and as ``HBMR_GPU_DEVICE`` — and unlike
the fork (PipesGPUMapRunner.java:64-79 hard-wired device 0) the
id really is the one the JobTracker assigned.
"""
from __future__ import annotations

import logging
import os
import secrets
import socket
import subprocess
import tempfile
import threading

from ..mapred import counters as C
from . import protocol as _protocol
from .protocol import DownwardProtocol, UplinkReader, create_digest, from_wire

log = logging.getLogger("hbmr.pipes")


class OutputHandler:
    """Upward-message sink: forwards output to the collector, progress/status to
    the reporter, child counters to the task's counters."""

    def __init__(self, collector, reporter, key_class, value_class, partitioner=None):
        self.collector = collector
        self.reporter = reporter
        self.kcls = key_class
        self.vcls = value_class
        self.partitioner = partitioner
        self.counters: dict[int, tuple] = {}
        self.done_event = threading.Event()
        self.auth_event = threading.Event()
        self.auth_digest = None
        self.error = None
        self.progress_value = 0.0
        self.records = 0
        # a map's output buffer takes the frames as they are (MapOutputBuffer.
        # raw_sink): no Writable built and re-serialised per record
        rs = getattr(collector, "raw_sink", None) if _protocol.RAW_FRAMES else None
        self.sink = rs() if rs is not None else None

    def output(self, k, v):
        if self.sink is not None:
            self.sink(k, v, None)
        else:
            if v.__class__ is memoryview:      # a large value read in place
                v = bytes(v)
            self.collector.collect(from_wire(k, self.kcls), from_wire(v, self.vcls))
        self.records += 1

    def partitioned_output(self, part, k, v):
        if self.sink is not None:
            self.sink(k, v, part)
            self.records += 1
            return
        if self.partitioner is not None:
            self.partitioner.set_next(part)
        self.output(k, v)

    def status(self, msg):
        if self.reporter is not None:
            self.reporter.setStatus(msg)

    def progress(self, p):
        self.progress_value = p
        if self.reporter is not None:
            self.reporter.progress()

    def done(self):
        self.done_event.set()
        self.auth_event.set()

    def register_counter(self, cid, group, name):
        self.counters[cid] = (group, name)

    def increment_counter(self, cid, amount):
        g = self.counters.get(cid)
        if g is not None and self.reporter is not None:
            self.reporter.incrCounter(g[0], g[1], amount)

    def authenticate(self, digest):
        self.auth_digest = digest
        self.auth_event.set()

    def failed(self, e):
        self.error = e
        self.done_event.set()
        self.auth_event.set()

    def wait_for_finish(self, timeout=None):
        self.done_event.wait(timeout)
        if self.error is not None:
            raise self.error
        return True


class Application:
    def __init__(self, job, collector, reporter, key_class, value_class, executable: str,
                 run_on_gpu: bool = False, gpu_device_id: int = -1, partitioner=None,
                 work_dir: str | None = None, reuse: bool = False):
        if not executable:
            raise ValueError("no Pipes executable configured (hadoop.pipes.executable / "
                             "hadoop.pipes.gpu.executable)")
        self.job = job
        self.server = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.server.bind(("127.0.0.1", 0))
        self.server.listen(16)
        port = self.server.getsockname()[1]
        self.work_dir = work_dir or tempfile.mkdtemp(prefix="hbmr-pipes-")
        os.makedirs(self.work_dir, exist_ok=True)
        password = secrets.token_hex(32).encode()
        self.secret_file = os.path.join(self.work_dir, "jobTokenPassword")
        fd = os.open(self.secret_file, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "wb") as f:
            f.write(password)
        env = dict(os.environ)
        env["hadoop.pipes.command.port"] = str(port)
        env["hadoop.pipes.shared.secret.location"] = self.secret_file
        cmd = [executable]
        if run_on_gpu:
            env["HBMR_GPU_DEVICE"] = str(gpu_device_id)
            cmd.append(str(gpu_device_id))
        else:
            env.pop("HBMR_GPU_DEVICE", None)
        self.stdout = open(os.path.join(self.work_dir, "stdout"), "wb")
        self.stderr = open(os.path.join(self.work_dir, "stderr"), "wb")
        log.info("launching pipes child: %s", " ".join(cmd))
        self.proc = subprocess.Popen(cmd, env=env, stdout=self.stdout, stderr=self.stderr,
                                     cwd=self.work_dir)
        self.server.settimeout(1.0)
        client = None
        while client is None:
            try:
                client, _ = self.server.accept()
            except socket.timeout:
                if self.proc.poll() is not None:
                    raise RuntimeError(f"pipes child exited with {self.proc.returncode} before "
                                       f"connecting: {self._stderr_tail()}")
        client.settimeout(None)
        client.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.client = client
        self.reuse = reuse
        self.handler = OutputHandler(collector, reporter, key_class, value_class, partitioner)
        self.downlink = DownwardProtocol(client)
        self.uplink = UplinkReader(client, self.handler, reuse=reuse)
        self.uplink.start()
        challenge = secrets.token_hex(16)
        digest = create_digest(password, challenge)
        self.downlink.authenticate(digest, challenge)
        self.handler.auth_event.wait(60)
        if self.handler.error is not None:
            raise RuntimeError(f"pipes child failed during authentication: {self.handler.error}; "
                               f"{self._stderr_tail()}")
        if self.handler.auth_digest != create_digest(password, digest):
            raise RuntimeError("pipes child failed authentication")
        self.downlink.start()
        self.downlink.set_job_conf(job)

    def _stderr_tail(self):
        try:
            self.stderr.flush()
            with open(os.path.join(self.work_dir, "stderr"), "rb") as f:
                return f.read()[-2000:].decode(errors="replace")
        except OSError:
            return ""

    def alive(self):
        return self.proc.poll() is None and self.uplink.is_alive()

    def begin_task(self, job, collector, reporter, key_class, value_class, partitioner=None):
        """Next task on a reused child: its own output handler, its task conf."""
        self.handler = OutputHandler(collector, reporter, key_class, value_class, partitioner)
        self.uplink.handler = self.handler
        self.job = job
        self.downlink.set_job_conf(job)

    def wait_for_finish(self):
        try:
            self.handler.wait_for_finish()
        except BaseException as e:
            rc = self.proc.wait(timeout=30)
            raise RuntimeError(f"pipes child failed (exit {rc}): {e}; {self._stderr_tail()}") \
                from e
        if self.reuse:
            return True          # the child waits for its next task
        rc = self.proc.wait()
        if rc != 0:
            raise RuntimeError(f"pipes child exited with {rc}: {self._stderr_tail()}")
        return True

    def abort(self, e=None):
        try:
            self.downlink.abort()
        finally:
            if self.proc.poll() is None:
                self.proc.kill()
                self.proc.wait()

    def cleanup(self):
        for c in (self.downlink, ):
            c.close()
        for s in (self.client, self.server):
            try:
                s.close()
            except OSError:
                pass
        self.stdout.close()
        self.stderr.close()
        try:
            os.remove(self.secret_file)
        except OSError:
            pass

    def close_child(self, timeout=10.0):
        """End a reused child: CLOSE while it waits for a task, then reap it."""
        try:
            self.downlink.end_of_input()
            self.downlink.flush()
        except OSError:
            pass
        try:
            self.proc.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            self.proc.kill()
            self.proc.wait()
        self.cleanup()

    def incr_records(self, reporter, n):
        if reporter is not None:
            reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, n)


class ChildPool:
    """Idle reusable Pipes children (``hbmr.pipes.child.reuse``), keyed by
    (executable, device, map|reduce): the Pipes analogue of the JvmManager's
    JVM reuse (JvmManager.java:119-413).  A GPU binary that stays up keeps its
    HIP context, device buffers and HBM-resident splits for the next task.
    Idle children are closed after ``hbmr.pipes.child.idle.s`` seconds."""

    def __init__(self, idle_s: float = 30.0):
        self.idle_s = idle_s
        self._idle: dict = {}
        self._lock = threading.Lock()
        self._reaper = None

    def acquire(self, key, split=None):
        """An idle child for ``key``: one that already mapped ``split`` (its
        serialized bytes) if any — a GPU binary keeps the split resident —
        else the most recently idle."""
        with self._lock:
            lst = self._idle.get(key) or []
            if split:
                for i in range(len(lst) - 1, -1, -1):
                    app = lst[i][0]
                    if split in getattr(app, "splits_seen", ()) and app.alive():
                        del lst[i]
                        return app
            while lst:
                app, _t = lst.pop()
                if app.alive():
                    return app
                app.cleanup()
        return None

    def release(self, key, app, idle_s=None, split=None):
        import time
        if not app.alive():
            app.cleanup()
            return
        if split:
            seen = getattr(app, "splits_seen", None)
            if seen is None:
                seen = app.splits_seen = set()
            if len(seen) < 4096:
                seen.add(split)
        with self._lock:
            self._idle.setdefault(key, []).append((app, time.time()))
            if idle_s is not None:
                self.idle_s = idle_s
            if self._reaper is None:
                self._reaper = threading.Thread(target=self._reap, daemon=True,
                                                name="pipes-child-reaper")
                self._reaper.start()

    def _reap(self):
        import time
        while True:
            time.sleep(min(5.0, max(0.5, self.idle_s / 4)))
            now = time.time()
            stale = []
            with self._lock:
                for key, lst in list(self._idle.items()):
                    keep = [(a, t) for a, t in lst if now - t < self.idle_s and a.alive()]
                    stale += [a for a, t in lst if (a, t) not in keep]
                    self._idle[key] = keep
            for a in stale:
                a.close_child()

    def close_all(self):
        with self._lock:
            apps = [a for lst in self._idle.values() for a, _ in lst]
            self._idle.clear()
        for a in apps:
            a.close_child()

    def size(self):
        with self._lock:
            return sum(len(v) for v in self._idle.values())


POOL = ChildPool()
