"""The JobTracker in a process of its own (``hbmr.jobtracker.process``).

The reference ran its JobTracker as a daemon JVM of its own
(hadoop-1.0.3/bin/hadoop-daemon.sh start jobtracker; JobTracker.main,
JobTracker.java:4380-4420), apart from every TaskTracker and from the job
client.  On one MI355X node hbmr's rank 0 would otherwise host the
JobTracker, its RPC handlers for the other ranks' trackers, its own
TaskTracker and the job driver under ONE interpreter lock: the per-job control
work of all N trackers then competes with rank 0's tracker and driver for it.
Here rank 0 starts this process (a child, before anything touches the GPU;
the JobTracker never does), every tracker — rank 0's included — talks to it
over the msgpack RPC, and the driver submits and waits through
:class:`RemoteJobTracker`: one long-poll per job wait and one call for a
finished job's status, counters, timeline and result.

Started as ``python -m hbmr.mapred.jtprocess``: the job configuration arrives
as JSON on stdin, the RPC port goes back as ``PORT <n>`` on stdout; the
process exits after ``rpc_stop`` (or when its parent's pipe closes).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time

from .jobclient import JobStatus, RunningJob
from .counters import Counters
from .rpc import JT_PROCESS_METHODS, RpcClient, RpcServer, _conf_secret


# --------------------------------------------------------------------------- server side
def serve(conf_dict: dict, out=sys.stdout) -> int:
    from .jobconf import JobConf
    from .jobtracker import JobTracker
    conf = JobConf()
    for k, v in conf_dict.items():
        conf.set(k, v)
    # every RPC handler thread is woken by a socket read: with CPython's
    # default 5 ms switch interval a woken handler waits that long for the
    # interpreter behind another one's bookkeeping (as in the trackers)
    si = conf.get_float("hbmr.python.switchinterval.ms", 0.2)
    if si > 0:
        sys.setswitchinterval(si / 1e3)
    jt = JobTracker(conf)
    stopped = threading.Event()

    def rpc_stop():
        jt.shutdown()
        stopped.set()
    jt.rpc_stop = rpc_stop
    srv = RpcServer(jt, JT_PROCESS_METHODS, secret=_conf_secret(conf)).start()
    out.write(f"PORT {srv.port}\n")
    out.flush()
    # the parent's end of stdin closes when it exits: do not outlive it
    threading.Thread(target=lambda: (sys.stdin.read(), stopped.set()), daemon=True,
                     name="jt-parent-watch").start()
    stopped.wait()
    time.sleep(0.05)            # the rpc_stop reply leaves before the server goes
    srv.stop()
    return 0


def main() -> int:
    line = sys.stdin.readline()
    conf_dict = json.loads(line) if line.strip() else {}
    from ..utils.gctune import tune
    from ..utils.sampler import dump_profiles, maybe_profile_threads, maybe_start
    tune()
    cprof = maybe_profile_threads()     # HBMR_CPROFILE / HBMR_SAMPLE_PROF cover this process
    sampler = maybe_start()
    from ..utils.phaseprof import maybe_install
    maybe_install()                     # HBMR_PHASE_PROF: per-method thread CPU
    try:
        return serve(conf_dict)
    finally:
        if cprof:
            dump_profiles(cprof)
        if sampler is not None:
            sampler.dump()


# --------------------------------------------------------------------------- client side
class _CostModelView:
    def __init__(self, rpc):
        self.rpc = rpc

    def snapshot(self):
        return self.rpc.call("rpc_cost_model")


class _JobView:
    """What a driver reads from a finished job's JobInProgress (timeline,
    maps per tracker), from the one rpc_job_info answer."""

    def __init__(self, info):
        self._info = info
        self.result = info.get("result")

    def timeline(self):
        return self._info.get("timeline") or {}

    def maps_per_tracker(self):
        return dict(self._info.get("maps_per_tracker") or {})


class _ProcJobHandle:
    """RunningJob backend for a job of a JobTracker process: waits long-poll,
    and a complete job's information is fetched once and cached."""

    def __init__(self, rpc, jid):
        self.rpc = rpc
        self.jid = jid
        self._info = None

    def _fetch(self, info=None):
        if info is None:
            info = self.rpc.call("rpc_job_info", self.jid)
        st = JobStatus(self.jid, info["state"])
        for k in ("map_progress", "reduce_progress", "start_time", "finish_time",
                  "failure_info"):
            setattr(st, k, info[k])
        if st.is_complete():
            self._info = (info, st)
        return info, st

    def _get(self):
        return self._info if self._info is not None else self._fetch()

    def status(self):
        return self._get()[1]

    def counters(self):
        return Counters.from_dict(self._get()[0]["counters"])

    def wait(self, timeout=None):
        if self._info is not None:
            return True
        deadline = None if timeout is None else time.time() + timeout
        while True:
            left = 60.0 if deadline is None else max(0.0, deadline - time.time())
            info = self.rpc.call("rpc_wait_job_info", self.jid, min(left, 60.0))
            if info is not None:
                self._fetch(info)
                return True
            if deadline is not None and time.time() >= deadline:
                return False

    def kill(self):
        self.rpc.call("rpc_kill_job", self.jid)

    def task_reports(self, is_map=True):
        return self.rpc.call("rpc_task_reports", self.jid, is_map)

    @property
    def result(self):
        info = self._get()[0]
        return info.get("result")

    @property
    def jip(self):
        """A finished job's JobInProgress view (None while it runs)."""
        if self._info is None:
            return None
        return _JobView(self._info[0])


class RemoteJobTracker:
    """The node's handle on its JobTracker process: job submission and waits
    for the driver, bring-up and shutdown for the node."""

    def __init__(self, conf):
        env = dict(os.environ, HBMR_JT_PROCESS="1")
        # the package root on the child's path whatever the caller's cwd
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH")
                                    else "")
        self.proc = subprocess.Popen([sys.executable, "-m", "hbmr.mapred.jtprocess"],
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                     env=env, text=True, cwd=root)
        self.proc.stdin.write(json.dumps(conf.to_dict()) + "\n")
        self.proc.stdin.flush()
        line = self.proc.stdout.readline()
        if not line.startswith("PORT "):
            self.proc.kill()
            raise RuntimeError(f"JobTracker process did not start: {line!r}")
        self.port = int(line.split()[1])
        self.address = f"127.0.0.1:{self.port}"
        self.rpc = RpcClient(self.address, secret=_conf_secret(conf))
        self.cost_model = _CostModelView(self.rpc)
        self.remote = True

    def submit_job(self, job):
        jid = self.rpc.call("rpc_submit_job", job.to_dict())
        return RunningJob(jid, _ProcJobHandle(self.rpc, jid), job)

    def wait_for_trackers(self, n, timeout=60.0):
        return bool(self.rpc.call("rpc_wait_for_trackers", n, timeout))

    def start_expiry_thread(self):
        self.rpc.call("rpc_start_expiry")

    def broadcast_shutdown(self):
        self.rpc.call("rpc_broadcast_shutdown")

    def live_trackers(self, exclude="", window=0.5):
        return int(self.rpc.call("rpc_live_trackers", exclude, window))

    def cpu_seconds(self):
        return float(self.rpc.call("rpc_cpu_seconds"))

    def thread_cpu(self):
        return dict(self.rpc.call("rpc_thread_cpu"))

    def shutdown(self):
        try:
            self.rpc.call("rpc_stop")
        except Exception:  # noqa: BLE001
            pass
        self.rpc.close()
        try:
            self.proc.stdin.close()
            self.proc.wait(timeout=10)
        except Exception:  # noqa: BLE001
            self.proc.kill()
            self.proc.wait()


if __name__ == "__main__":
    sys.exit(main())
