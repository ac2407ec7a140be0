"""Task child processes: process isolation and process reuse for classic tasks.

The reference runs every map/reduce attempt in a child JVM that the
TaskTracker forks through TaskRunner/JvmManager/TaskController and that pulls
its task over the umbilical RPC (TaskRunner.run, TaskRunner.java:188;
JvmManager.launchJvm/spawnNewJvm/runChild, JvmManager.java:119, 413, 485;
Child.main/getTask/task.run, Child.java:69, 172, 255; umbilical protocol
TaskUmbilicalProtocol.java:74-181), optionally reusing one JVM for several
tasks of a job (``mapred.job.reuse.jvm.num.tasks``, JvmManager), killing
children that outgrow their memory limit (TaskMemoryManagerThread.java:39,
``mapred.job.{map,reduce}.memory.mb``) and capturing each attempt's
stdout/stderr under ``userlogs/<attempt>`` (TaskLog).

hbmr's default is in-process execution (a persistent tracker process per GPU,
tasks on threads: no per-task launch cost, the "map-task invocation overhead"
of Shirahata et al.).  ``hbmr.task.child.process=true`` (or
``mapred.task.isolation=process``) runs classic CPU tasks in child Python
processes instead — needed for user map/reduce code that holds the GIL or may
crash.  Split-level GPU jobs always stay in the tracker, whose HBM split cache
and HIP context they depend on.

Design:
* :class:`ChildManager` (JvmManager): per-job pools of idle children; a child
  serves up to ``mapred.job.reuse.jvm.num.tasks`` tasks (``-1`` = unlimited,
  default 1 = fresh process per task, like the reference).
* The umbilical is a private socketpair inherited by the child (so no port
  and no token to guard, unlike the reference's RPC umbilical): child → parent
  messages are ``status`` (progress, status
  string, counters; every ``hbmr.task.progress.interval.ms``, default 1000 —
  the reference's 3 s PROGRESS_INTERVAL, Task.java:498), ``done`` and
  ``failed``; parent → child are ``task`` and ``exit``.
* Kill = SIGKILL of the child (a child cannot be trusted to honour a flag);
  a child that exits mid-task fails the attempt with its exit status, as
  "Task process exit with nonzero status of N" does in the reference.
* ``mapred.child.env`` ("A=1,B=2") is exported into the child,
  ``mapred.child.ulimit`` (KB) becomes RLIMIT_AS.
"""
from __future__ import annotations

import logging
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import traceback
from multiprocessing.connection import Connection

log = logging.getLogger("hbmr.child")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def use_child_process(conf) -> bool:
    if conf.get_boolean("hbmr.task.child.process", False):
        return True
    return (conf.get("mapred.task.isolation") or "").lower() == "process"


class ChildDied(RuntimeError):
    pass


class _Child:
    """One live child process (a JvmRunner)."""

    def __init__(self, mgr, job_id, conn, proc, max_tasks):
        self.mgr = mgr
        self.job_id = job_id
        self.conn = conn
        self.proc = proc
        self.pid = proc.pid
        self.max_tasks = max_tasks
        self.tasks_run = 0
        self.busy_attempt = None
        self.memory_limit_mb = 0
        self.killed_reason = None
        self.idle_since = 0.0

    def alive(self):
        return self.proc.poll() is None

    def kill(self, reason=None):
        if reason and self.killed_reason is None:
            self.killed_reason = reason
        try:
            os.killpg(self.proc.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            try:
                self.proc.kill()
            except ProcessLookupError:
                pass
        try:
            self.proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            pass
        try:
            self.conn.close()
        except OSError:
            pass

    def rss_mb(self):
        """Resident memory of the child's process tree (ProcfsBasedProcessTree)."""
        try:
            import psutil
            p = psutil.Process(self.pid)
            procs = [p] + p.children(recursive=True)
            total = 0
            for q in procs:
                try:
                    total += q.memory_info().rss
                except psutil.Error:
                    pass
            return total / (1 << 20)
        except Exception:  # noqa: BLE001
            return 0.0


class ChildManager:
    """JvmManager for one tracker."""

    def __init__(self, tracker_name, local_dir, conf):
        self.tracker_name = tracker_name
        self.local_dir = local_dir
        self._idle: dict[str, list[_Child]] = {}
        self._busy: set[_Child] = set()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.spawned = 0
        self.monitor_interval = min(1.0, conf.get_int(
            "mapred.tasktracker.taskmemorymanager.monitoring-interval", 5000) / 1000.0)
        # a reused child of a job that sends no more tasks exits after this
        self.idle_timeout = conf.get_int("hbmr.task.child.idle.ms", 5000) / 1000.0
        self._mon = threading.Thread(target=self._monitor, daemon=True,
                                     name=f"{tracker_name}-taskmem")
        self._mon.start()

    # -- process pool ------------------------------------------------------------------
    def _spawn(self, job_id, conf):
        env = dict(os.environ)
        # the child sees the tracker's import path (the reference puts the job
        # jar and its lib/ on the child classpath, TaskRunner.java:378-471)
        paths = [ROOT] + [p for p in sys.path if p and os.path.isdir(p)]
        if env.get("PYTHONPATH"):
            paths.append(env["PYTHONPATH"])
        env["PYTHONPATH"] = os.pathsep.join(dict.fromkeys(paths))
        for kv in (conf.get("mapred.child.env") or "").split(","):
            if "=" in kv:
                k, v = kv.split("=", 1)
                env[k.strip()] = v.strip().replace("$" + k.strip(), env.get(k.strip(), ""))
        ulimit = conf.get_int("mapred.child.ulimit", 0)
        if ulimit > 0:
            env["HBMR_CHILD_ULIMIT_KB"] = str(ulimit)
        # the umbilical: one end of a private socketpair, inherited by fd
        parent_sock, child_sock = socket.socketpair()
        env["HBMR_UMBILICAL_FD"] = str(child_sock.fileno())
        cmd = [sys.executable, "-m", "hbmr.mapred.child"]
        try:
            proc = subprocess.Popen(cmd, env=env, cwd=self.local_dir, stdin=subprocess.DEVNULL,
                                    pass_fds=(child_sock.fileno(),), start_new_session=True)
        finally:
            child_sock.close()
        conn = Connection(parent_sock.detach())
        if not conn.poll(60):
            proc.kill()
            conn.close()
            raise ChildDied("child did not report in within 60 s")
        try:
            hello = conn.recv()
        except (EOFError, OSError) as e:
            proc.kill()
            raise ChildDied(f"child exited during start-up (status {proc.wait()})") from e
        if hello[0] != "hello" or hello[1] != proc.pid:
            proc.kill()
            raise ChildDied(f"unexpected child handshake {hello!r}")
        self.spawned += 1
        reuse = conf.get_int("mapred.job.reuse.jvm.num.tasks", 1)
        return _Child(self, job_id, conn, proc, reuse)

    def acquire(self, job_id, conf) -> _Child:
        with self._lock:
            pool = self._idle.get(job_id, [])
            while pool:
                ch = pool.pop()
                if ch.alive():
                    self._busy.add(ch)
                    return ch
        ch = self._spawn(job_id, conf)
        with self._lock:
            self._busy.add(ch)
        return ch

    def release(self, ch: _Child, reusable: bool):
        with self._lock:
            self._busy.discard(ch)
            ch.busy_attempt = None
            if reusable and ch.alive() and (ch.max_tasks < 0 or ch.tasks_run < ch.max_tasks) \
                    and not self._stop.is_set():
                ch.idle_since = time.time()
                self._idle.setdefault(ch.job_id, []).append(ch)
                return
        self._retire(ch)

    def _retire(self, ch):
        """Tell a child to exit; reap it off the task's critical path."""
        try:
            ch.conn.send(("exit",))
        except OSError:
            pass

        def _reap():
            try:
                ch.proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                ch.kill()
            try:
                ch.conn.close()
            except OSError:
                pass
        threading.Thread(target=_reap, daemon=True, name=f"reap-{ch.pid}").start()

    def job_done(self, job_id):
        with self._lock:
            pool = self._idle.pop(job_id, [])
        for ch in pool:
            self._retire(ch)

    def shutdown(self):
        self._stop.set()
        with self._lock:
            idle = [c for p in self._idle.values() for c in p]
            busy = list(self._busy)
            self._idle.clear()
        for ch in idle:
            self._retire(ch)
        for ch in busy:
            ch.kill("tracker shutting down")

    # -- TaskMemoryManagerThread ---------------------------------------------------------
    def _monitor(self):
        while not self._stop.wait(self.monitor_interval):
            now = time.time()
            stale = []
            with self._lock:
                for job, pool in list(self._idle.items()):
                    keep = [c for c in pool if now - c.idle_since < self.idle_timeout]
                    stale += [c for c in pool if now - c.idle_since >= self.idle_timeout]
                    if keep:
                        self._idle[job] = keep
                    else:
                        del self._idle[job]
                busy = [c for c in self._busy if c.memory_limit_mb > 0 and c.busy_attempt]
            for ch in stale:
                self._retire(ch)
            for ch in busy:
                rss = ch.rss_mb()
                if rss > ch.memory_limit_mb:
                    msg = (f"Task {ch.busy_attempt} is running beyond memory-limits. Current "
                           f"usage : {rss:.0f}MB. Limit : {ch.memory_limit_mb}MB. Killing task.")
                    log.warning(msg)
                    ch.kill(msg)

    # -- one attempt ------------------------------------------------------------------------
    def run_task(self, job_id, conf, payload, reporter, kill_event, progress_cb=None,
                 spawn_conf=None):
        """Run one attempt in a child; returns the task's result (map output path or
        None).  Mirrors counters/status/progress into ``reporter`` as they arrive.
        Raises on failure (ChildDied when the process died or was killed).
        ``spawn_conf``: the conf a new child starts from (environment, reuse
        count), if not the task's own (a pool shared by several jobs)."""
        ch = self.acquire(job_id, spawn_conf if spawn_conf is not None else conf)
        ch.busy_attempt = payload["attempt_id"]
        key = "mapred.job.map.memory.mb" if payload["is_map"] else "mapred.job.reduce.memory.mb"
        ch.memory_limit_mb = max(0, conf.get_int(key, -1))
        ch.tasks_run += 1
        reusable = False
        try:
            ch.conn.send(("task", payload))
            while True:
                if kill_event.is_set():
                    ch.kill("killed")
                    raise ChildDied("task killed")
                try:
                    ready = ch.conn.poll(0.05)
                except (OSError, EOFError):
                    ready = True
                if not ready:
                    if not ch.alive():
                        raise ChildDied(ch.killed_reason or
                                        f"Task process exit with nonzero status of "
                                        f"{ch.proc.returncode}.")
                    continue
                try:
                    msg = ch.conn.recv()
                except (EOFError, OSError):
                    try:
                        ch.proc.wait(timeout=5)
                    except subprocess.TimeoutExpired:
                        pass
                    raise ChildDied(ch.killed_reason or
                                    f"Task process exit with nonzero status of "
                                    f"{ch.proc.returncode}.") from None
                kind = msg[0]
                if kind == "status":
                    _, prog, status, counters, last = msg
                    _mirror(reporter, prog, status, counters, last)
                    if progress_cb is not None:
                        progress_cb(prog)
                elif kind == "done":
                    _, result, counters = msg
                    _mirror(reporter, 1.0, reporter.status, counters, time.time())
                    reusable = True
                    return result
                elif kind == "failed":
                    _, diag, counters = msg
                    _mirror(reporter, reporter.progress_value, reporter.status, counters,
                            time.time())
                    reusable = True
                    raise RuntimeError(diag)
        finally:
            self.release(ch, reusable)


def _mirror(reporter, prog, status, counters, last_progress):
    """Copy a child's report.  Only the child's own progress time moves
    ``last_progress``: a periodic report of a task that made no progress is the
    reference's ping, which does not hold off mapred.task.timeout."""
    from .counters import Counters
    reporter.counters = Counters.from_dict(counters)
    reporter.status = status
    reporter.progress_value = float(prog)
    reporter.last_progress = max(reporter.last_progress, float(last_progress))


# ----------------------------------------------------------------------------- child side
def _redirect_logs(log_dir):
    """Per-attempt stdout/stderr (TaskLog userlogs/<attempt>/{stdout,stderr})."""
    os.makedirs(log_dir, exist_ok=True)
    sys.stdout.flush()
    sys.stderr.flush()
    for fd, name in ((1, "stdout"), (2, "stderr")):
        f = os.open(os.path.join(log_dir, name), os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        os.dup2(f, fd)
        os.close(f)


def _run_one(conn, payload, interval):
    from .ids import TaskAttemptID
    from .jobconf import JobConf
    from .profiling import run_profiled
    from .task import MapOutputLocation, MapTask, ReduceTask

    conf = JobConf()
    for k, v in payload["conf"].items():
        conf.set(k, v)
    aid = TaskAttemptID.for_name(payload["attempt_id"])
    if payload["is_map"]:
        from .tasktracker import _split_from_dict
        task = MapTask(conf, aid, payload["partition"], _split_from_dict(payload["split"]))
        task.setRunOnGPU(payload.get("run_on_gpu", False))
        task.setGPUDeviceId(payload.get("gpu_device_id", -1))
    else:
        task = ReduceTask(conf, aid, payload["partition"], payload["num_maps"])
        for map_aid, path in payload["map_outputs"]:
            task.add_map_output(MapOutputLocation(map_aid, path))
    rep = task.reporter
    send_lock = threading.Lock()
    stop = threading.Event()

    def _pinger():   # Task.TaskReporter's progress thread (Task.java:554, 654-700)
        while not stop.wait(interval):
            with send_lock:
                conn.send(("status", rep.progress_value, rep.status, rep.counters.to_dict(),
                           rep.last_progress))

    th = threading.Thread(target=_pinger, daemon=True)
    th.start()
    try:
        result = run_profiled(conf, payload["attempt_id"], payload["is_map"],
                              payload["partition"], task.run, payload["work_dir"])
        stop.set()
        with send_lock:
            conn.send(("done", result, rep.counters.to_dict()))
    except BaseException as e:  # noqa: BLE001
        stop.set()
        with send_lock:
            conn.send(("failed", f"{type(e).__name__}: {e}\n{traceback.format_exc()[-2000:]}",
                       rep.counters.to_dict()))
    th.join(timeout=1)


def child_main():
    """Child.main: connect to the tracker's umbilical, then serve tasks until told
    to exit (or the tracker goes away)."""
    ulimit = int(os.environ.get("HBMR_CHILD_ULIMIT_KB", "0"))
    if ulimit > 0:
        import resource
        resource.setrlimit(resource.RLIMIT_AS, (ulimit * 1024, ulimit * 1024))
    conn = Connection(int(os.environ.pop("HBMR_UMBILICAL_FD")))
    conn.send(("hello", os.getpid()))
    while True:
        try:
            msg = conn.recv()
        except (EOFError, OSError):
            break
        if msg[0] == "exit":
            break
        if msg[0] == "task":
            payload = msg[1]
            if payload.get("log_dir"):
                _redirect_logs(payload["log_dir"])
            _run_one(conn, payload, payload.get("progress_interval", 1.0))
    conn.close()


if __name__ == "__main__":
    child_main()
