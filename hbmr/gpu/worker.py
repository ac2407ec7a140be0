"""Per-GPU worker process: the device side of a TaskTracker, isolated.

The reference never ran GPU code inside its daemons: a GPU map task was a
Pipes binary in a child process of a child JVM, so a crashed GPU program was
an ordinary failed attempt (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/
pipes/Application.java:274-290; child JVMs via JvmManager.java:413-485).  It
paid for that with a process launch per task.  Here one *persistent* worker
process per tracker owns the HIP context, the HBM split cache, the per-job map
outputs and the collective communicator (RCCL among the workers of all
ranks) — launched once, reused by every task of every job (the analogue of
``mapred.job.reuse.jvm.num.tasks = -1``) — while the TaskTracker (and the
JobTracker on rank 0) never touch the GPU.  A HIP fault kills the worker:
its attempts fail, its held map outputs are reported lost, and the tracker
starts a fresh worker (see :mod:`hbmr.gpu.remote`).

Inside the worker the very same runtime code runs as in a tracker: the GPU
slot runtime (:class:`~hbmr.gpu.runtime.GpuRuntime`, or the simulated one)
and the split-task executor (:mod:`hbmr.gpu.splitexec`), against
:class:`WorkerHost`, a tracker facade whose ``_finish`` / ``finish_bulk``
queue reports that ``notify_jobtracker`` ships to the tracker in one frame.

Wire: 4-byte big-endian length + pickle, over a socketpair inherited from the
tracker (parent and child only; nothing else can connect).

  tracker -> worker: ("init", dict) ("job", jid, conf) ("maps", jid, [spec])
                     ("cpu", spec) ("reduce", spec) ("kill", aid) ("drop", jid)
                     ("probe", device) ("stop",)
  worker -> tracker: ("ready", [device status], pid, {devices, GPU_MAX_HW_QUEUES})
                     ("batch", [("done", status) | ("bulk", aids, dt, out, ctrs)],
                      cache_added, cache_removed)
                     ("probe", device, reason-or-None)

Started as ``python -m hbmr.gpu.worker <fd>``.
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import os
import pickle
import random
import socket
import struct
import sys
import threading
import time

from ..utils.trace import TRACE

_LEN = struct.Struct(">I")
log = logging.getLogger("hbmr.gpu.worker")


# --------------------------------------------------------------------------- framing
def send_msg(sock, obj, lock=None):
    data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    frame = _LEN.pack(len(data)) + data
    if lock is None:
        sock.sendall(frame)
    else:
        with lock:
            sock.sendall(frame)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            return None
        got += k
    return bytes(buf)


def recv_msg(sock):
    """Next message, or None at EOF (the peer is gone)."""
    hdr = _recv_exact(sock, 4)
    if hdr is None:
        return None
    (n,) = _LEN.unpack(hdr)
    body = _recv_exact(sock, n)
    if body is None:
        return None
    return pickle.loads(body)


# --------------------------------------------------------------------------- tracker facade
class WorkerHost:
    """The 'tracker' the device runtime and split tasks see inside the worker."""

    def __init__(self, sock, init, comm):
        from ..mapred.jobconf import JobConf
        from .split_cache import SplitCache
        self.sock = sock
        self.send_lock = threading.Lock()
        self.conf = JobConf()
        for k, v in init["conf"].items():
            self.conf.set(k, v)
        self.name = init["name"]
        self.rank = init["rank"]
        self.world_size = init["world"]
        self.cpu_threads = init["cpu_threads"]
        self.split_cache = SplitCache()
        self.comm = comm
        self.fault_p = self.conf.get_float("hbmr.faultinject.probability", 0.0)
        # crash injection: the worker process exits (os._exit) when it starts an
        # attempt whose id contains this text (tests of crash isolation)
        self.exit_on = self.conf.get("hbmr.faultinject.worker.exit.attempt") or ""
        self.exit_p = self.conf.get_float("hbmr.faultinject.worker.exit.probability", 0.0)
        self._rng = random.Random(self.rank * 7919 + 29 + init.get("generation", 0))
        self.jobs: dict = {}
        self.runs: dict = {}
        self._out: list = []
        self._lock = threading.Lock()
        self.tasks_done = 0

    # -- what GpuRuntime / splitexec call -----------------------------------------------
    def _maybe_inject_crash(self, run):
        aid = run.spec.attempt_id
        if (self.exit_on and self.exit_on in aid) or \
                (self.exit_p > 0 and self._rng.random() < self.exit_p):
            # a simulated device crash: the whole process goes, like a HIP fault
            os._exit(70)

    def _maybe_inject_fault(self, run):
        self._maybe_inject_crash(run)
        if self.fault_p > 0 and self._rng.random() < self.fault_p:
            raise RuntimeError(f"injected fault (hbmr.faultinject.probability={self.fault_p})")

    def _finish(self, run, state, diag="", output=None, device_time=0.0, wake=True):
        from ..mapred import protocol as P
        if state != P.SUCCEEDED and run.spec.is_map and run.job is not None:
            run.job.note_failed(run.spec.attempt_id)
        st = run.status
        st.state = state
        st.finish_time = time.time()
        st.diagnostic = diag
        if run.task is not None:
            st.counters = run.task.reporter.counters.to_dict()
        if output is not None:
            st.output = output
        st.device_time = device_time
        if state == P.SUCCEEDED:
            st.progress = 1.0
        with self._lock:
            self.runs.pop(st.attempt_id, None)
            self._out.append(("done", st.to_dict()))
        self.tasks_done += 1
        if wake:
            self.notify_jobtracker()

    def finish_bulk(self, runs, device_time, output, counters=None):
        if counters is None:
            from .runtime import _merge_counters
            counters = _merge_counters(runs).to_dict()
        aids = [r.spec.attempt_id for r in runs]
        with self._lock:
            for a in aids:
                self.runs.pop(a, None)
            self._out.append(("bulk", aids, device_time, output, counters))
        self.tasks_done += len(runs)

    def notify_jobtracker(self):
        added, removed = self.split_cache.drain_changes()
        with self._lock:
            out, self._out = self._out, []
        if out or added or removed:
            send_msg(self.sock, ("batch", out, added, removed), self.send_lock)

    def wakeup(self, _name=None, _seq=None):
        self.notify_jobtracker()


# --------------------------------------------------------------------------- comm
def _make_comm(init):
    """Collectives among the workers of all ranks (world > 1): a process group
    of their own, rendezvousing in the node's store under this generation's
    prefix, so a restarted gang never meets a dead member's keys."""
    from ..parallel.collectives import SoloComm, TorchComm
    spec = init.get("comm")
    if not spec or spec["world"] <= 1:
        return SoloComm()
    import datetime

    import torch.distributed as dist
    store = dist.TCPStore(spec["host"], spec["port"], is_master=False,
                          timeout=datetime.timedelta(seconds=spec.get("timeout", 600)))
    ps = dist.PrefixStore(f"hbmr/gpuworker/g{init.get('generation', 0)}/", store)
    kw = {}
    if spec["backend"] == "nccl":
        import torch
        kw["device_id"] = torch.device("cuda", init["devices"][0])
    dist.init_process_group(spec["backend"], store=ps, rank=spec["rank"],
                            world_size=spec["world"],
                            timeout=datetime.timedelta(seconds=spec.get("timeout", 600)), **kw)
    cpu_group = dist.new_group(backend="gloo") if spec["backend"] != "gloo" else None
    return TorchComm(group=None, cpu_group=cpu_group)


def _watch(host, runtime, every):
    """HBMR_STACKDUMP_S: the worker's view every that many seconds (stderr):
    attempts it holds, staged runs behind gates, device queues, busy slots."""
    def loop():
        while True:
            time.sleep(every)
            try:
                devs = getattr(runtime, "devices", {})
                q = {d: (dv.q.qsize(), sum(s.inflight for s in dv.slots))
                     for d, dv in devs.items()}
                print(f"worker-watch: runs={len(host.runs)} jobs={len(host.jobs)} "
                      f"gated={runtime.gates.held_count()} queue/inflight={q}",
                      file=sys.stderr, flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"worker-watch: {e!r}", file=sys.stderr, flush=True)
    threading.Thread(target=loop, daemon=True, name="hbmr-workerwatch").start()


# --------------------------------------------------------------------------- main loop
def serve(sock):
    msg = recv_msg(sock)
    if msg is None or msg[0] != "init":
        return 2
    init = msg[1]
    logging.basicConfig(level=init.get("log_level", logging.WARNING),
                        format=f"%(asctime)s worker[{init['name']}] %(name)s %(levelname)s "
                               f"%(message)s")
    sys.setswitchinterval(init.get("switchinterval", 0.0002))
    import torch

    from ..mapred import protocol as P
    from ..mapred.tasktracker import JobState, _Flag, _Running
    from .splitexec import run_split_cpu_map, run_split_reduce
    devices = init["devices"]
    simulate = init.get("simulate", False)
    nthr = int(init["conf"].get("hbmr.worker.torch.threads", "0") or 0)
    if nthr > 0:
        torch.set_num_threads(nthr)
    if not simulate:
        torch.cuda.set_device(devices[0])
    comm = _make_comm(init)
    host = WorkerHost(sock, init, comm)
    if simulate:
        from .simulated import SimulatedGpuRuntime as Rt
    else:
        from .runtime import GpuRuntime as Rt
        from ..ops import _lib
        _lib.load()      # fail loudly now, not in the first task
    runtime = Rt(host, devices, init["slots"])
    host.gpu_runtime = runtime      # the reduce opens gates of staged maps on it
    runtime.start()
    if os.environ.get("HBMR_STACKDUMP_S"):
        _watch(host, runtime, float(os.environ["HBMR_STACKDUMP_S"]))
    dev = None if simulate else runtime.torch_device(devices[0])
    cpu_pool = cf.ThreadPoolExecutor(max(1, init.get("cpu_slots", 1)),
                                     thread_name_prefix="worker-cpu")
    status = [g.__dict__ for g in runtime.device_status()]
    from ..utils.gctune import tune
    tune()      # torch and the runtime into the permanent GC generation
    send_msg(sock, ("ready", status, os.getpid(),
                    {"devices": list(devices),
                     "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}),
             host.send_lock)

    def _unknown_job(runs):
        # the tracker sent attempts of a job this worker does not hold (it was
        # dropped): fail them instead of taking the serve loop down with a KeyError
        for r in runs:
            host._finish(r, P.FAILED, f"job {r.spec.job_id} unknown to the GPU worker",
                         wake=False)
        host.notify_jobtracker()
        return []

    def _run(d, kill=None):
        spec = P.TaskSpec.from_dict(d)
        st = P.TaskStatus(spec.attempt_id, spec.is_map, P.RUNNING, 0.0, spec.run_on_gpu,
                          spec.gpu_device_id, time.time())
        r = _Running(spec, st, host.jobs.get(spec.job_id), kill or _Flag())
        if r.job is None:
            _unknown_job([r])
            return None
        with host._lock:
            host.runs[spec.attempt_id] = r
        return r

    def _runs_compact(jid, common, tasks):
        is_map, on_gpu, dev_id, nm, nr, coll, gate = common
        js = host.jobs.get(jid)
        now = time.time()
        out = []
        for aid, part, split in tasks:
            spec = P.TaskSpec(aid, jid, is_map, part, on_gpu, dev_id, split, nm, nr, [], coll,
                              gate=gate)
            st = P.TaskStatus(aid, is_map, P.RUNNING, 0.0, on_gpu, dev_id, now)
            out.append(_Running(spec, st, js, _Flag()))
        if js is None:
            return _unknown_job(out)
        with host._lock:
            for r in out:
                host.runs[r.spec.attempt_id] = r
        return out

    while True:
        msg = recv_msg(sock)
        if msg is None:
            break                       # the tracker is gone
        typ = msg[0]
        if TRACE.on:
            TRACE.instant("wk.recv", kind=typ)
        if typ == "maps_c":
            runtime.submit_many(_runs_compact(msg[1], msg[2], msg[3]))
        elif typ == "maps":
            runtime.submit_many([r for r in (_run(d) for d in msg[2]) if r is not None])
        elif typ == "job":
            jid, conf_dict = msg[1], msg[2]
            if jid not in host.jobs:
                from ..mapred.jobconf import JobConf
                conf = JobConf()
                for k, v in conf_dict.items():
                    conf.set(k, v)
                host.jobs[jid] = JobState(jid, conf)
                if TRACE.on:
                    TRACE.instant("wk.job_ready")
        elif typ == "cpu":
            r = _run(msg[1], threading.Event())
            if r is not None:
                cpu_pool.submit(run_split_cpu_map, host, r)
        elif typ == "reduce":
            def _reduce(r):
                run_split_reduce(host, r, dev)
                if r.status.state == P.SUCCEEDED:
                    # the job is done on this worker; after a FAILED reduce the
                    # JobTracker re-runs maps / the reduce of the same job here
                    host.jobs.pop(r.spec.job_id, None)
            r = _run(msg[1], threading.Event())
            if r is not None:
                # own thread: an early ("expect") reduce waits for maps held
                # behind an earlier job's reduce, which a bounded pool could starve
                threading.Thread(target=_reduce, args=(r,), daemon=True,
                                 name=f"worker-red-{r.spec.attempt_id[-12:]}").start()
        elif typ == "kill":
            with host._lock:
                r = host.runs.get(msg[1])
            if r is not None:
                r.kill.set()
                if r.task is not None and getattr(r.task, "kill_event", None) is not None:
                    r.task.kill_event.set()
        elif typ == "drop":
            host.jobs.pop(msg[1], None)
            for r in runtime.drop_held(msg[1]) if hasattr(runtime, "drop_held") else ():
                host._finish(r, P.KILLED, "job purged", wake=False)
        elif typ == "close_gate":
            if hasattr(runtime, "close_gate"):
                runtime.close_gate(msg[1])
        elif typ == "probe":
            reason = runtime.probe(msg[1]) if hasattr(runtime, "probe") else None
            send_msg(sock, ("probe", msg[1], reason), host.send_lock)
        elif typ == "stop":
            break
    runtime.stop()
    try:
        if not simulate:
            torch.cuda.synchronize()
    except Exception:  # noqa: BLE001
        pass
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    from ..utils.sampler import dump_profiles, maybe_arm_stackdump, maybe_profile_threads, \
        maybe_start
    maybe_arm_stackdump()
    # the bench's control-plane profilers (HBMR_CPROFILE / HBMR_SAMPLE_PROF)
    # cover the worker too: its per-map bookkeeping is on the job's critical path
    cprof = maybe_profile_threads()
    sampler = maybe_start()
    sock = socket.socket(fileno=int(argv[0]))
    try:
        rc = serve(sock)
    finally:
        try:
            sock.close()
        except OSError:
            pass
        if cprof:
            dump_profiles(cprof)
        if sampler is not None:
            sampler.dump()
    sys.stdout.flush()
    sys.stderr.flush()
    if os.environ.get("HBMR_WORKER_CLEAN_EXIT") or \
            any(k.startswith("ROCPROF") for k in os.environ):
        # a normal exit, so a profiler's exit handlers write this process's
        # trace.  Threads still inside HIP calls while the interpreter and the
        # HIP runtime tear down ended the worker in std::terminate under the
        # tracer: let them drain first (reduce threads, pools), bounded.
        deadline = time.time() + 10.0
        for t in threading.enumerate():
            if t is not threading.current_thread() and t.is_alive():
                t.join(timeout=max(0.0, deadline - time.time()))
        try:
            import torch
            if torch.cuda.is_initialized():
                torch.cuda.synchronize()
        except Exception:  # noqa: BLE001
            pass
        sys.exit(rc)
    # skip interpreter teardown of the HIP runtime / process group (the parent
    # only needs the exit status; the grid has drained in serve())
    os._exit(rc)


if __name__ == "__main__":
    main()
