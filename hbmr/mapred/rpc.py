"""Length-prefixed msgpack RPC over TCP — the control plane between processes.

Replaces Hadoop IPC (hadoop-1.0.3/src/core/org/apache/hadoop/ipc/{RPC,Server,
Client}.java, Writable-serialised calls with listener/reader/handler/responder
threads) for the only remote interfaces hbmr needs on one node: the
InterTrackerProtocol (heartbeat / wakeup) and the JobSubmissionProtocol
(submit / status / kill).  Frames: 4-byte big-endian length + msgpack
``{"m": method, "a": args, "k": kwargs}`` → ``{"r": result}`` or ``{"e": error}``.
Sockets use TCP_NODELAY; clients keep one connection per thread so a
long-polling heartbeat never blocks a concurrent wakeup.
"""
from __future__ import annotations

import logging
import socket
import socketserver
import struct
import threading

import msgpack

log = logging.getLogger("hbmr.rpc")

_LEN = struct.Struct(">I")


def _send(sock, obj):
    data = msgpack.packb(obj, use_bin_type=True)
    sock.sendall(_LEN.pack(len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("connection closed")
        buf += chunk
    return bytes(buf)


def _recv(sock):
    (n,) = _LEN.unpack(_recv_exact(sock, 4))
    return msgpack.unpackb(_recv_exact(sock, n), raw=False, strict_map_key=False)


class RpcServer:
    def __init__(self, target, methods, host="0.0.0.0", port=0):
        self.target = target
        self.methods = set(methods)
        outer = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                s = self.request
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                while True:
                    try:
                        req = _recv(s)
                    except (ConnectionError, OSError):
                        return
                    m = req.get("m")
                    try:
                        if m not in outer.methods:
                            raise AttributeError(f"no RPC method {m!r}")
                        res = getattr(outer.target, m)(*req.get("a", ()), **req.get("k", {}))
                        _send(s, {"r": res})
                    except Exception as e:  # noqa: BLE001
                        log.debug("rpc %s failed", m, exc_info=True)
                        try:
                            _send(s, {"e": f"{type(e).__name__}: {e}"})
                        except OSError:
                            return

        class Server(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self.server = Server((host, port), Handler)
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True,
                                       name="rpc-server")

    @property
    def port(self):
        return self.server.server_address[1]

    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self.server.shutdown()
        self.server.server_close()


class RpcError(RuntimeError):
    pass


class RpcClient:
    def __init__(self, address: str, timeout: float = 600.0):
        host, port = address.rsplit(":", 1)
        self.addr = (host, int(port))
        self.timeout = timeout
        self._tl = threading.local()

    def _sock(self):
        s = getattr(self._tl, "sock", None)
        if s is None:
            s = socket.create_connection(self.addr, timeout=self.timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._tl.sock = s
        return s

    def call(self, method, *args, **kwargs):
        for attempt in range(2):
            s = self._sock()
            try:
                _send(s, {"m": method, "a": list(args), "k": kwargs})
                resp = _recv(s)
                break
            except (ConnectionError, OSError):
                self._tl.sock = None
                try:
                    s.close()
                except OSError:
                    pass
                if attempt:
                    raise
        if "e" in resp:
            raise RpcError(resp["e"])
        return resp.get("r")

    def close(self):
        s = getattr(self._tl, "sock", None)
        if s is not None:
            s.close()
            self._tl.sock = None


JT_METHODS = ("heartbeat", "wakeup", "rpc_submit_job", "rpc_job_status", "rpc_kill_job",
              "rpc_job_result", "rpc_cluster_status", "rpc_list_jobs", "rpc_task_reports")


class JobTrackerProxy:
    """TaskTracker/JobClient-side stub of a remote JobTracker."""

    def __init__(self, address):
        self.rpc = RpcClient(address)
        self.address = address

    def heartbeat(self, status, initial=False, accept_new_tasks=True, block=0.0):
        return self.rpc.call("heartbeat", status, initial=initial,
                             accept_new_tasks=accept_new_tasks, block=block)

    def wakeup(self, tracker_name):
        return self.rpc.call("wakeup", tracker_name)


class _RemoteJob:
    def __init__(self, rpc, jid):
        self.rpc = rpc
        self.jid = jid

    def status(self):
        from .jobclient import JobStatus
        d = self.rpc.call("rpc_job_status", self.jid)
        st = JobStatus(self.jid, d["state"])
        st.__dict__.update(d)
        return st

    def counters(self):
        from .counters import Counters
        return Counters.from_dict(self.rpc.call("rpc_job_status", self.jid)["counters"])

    def wait(self, timeout=None):
        import time
        t0 = time.time()
        while True:
            if self.status().is_complete():
                return True
            if timeout is not None and time.time() - t0 >= timeout:
                return False
            time.sleep(0.01)

    def kill(self):
        self.rpc.call("rpc_kill_job", self.jid)

    def task_reports(self, is_map=True):
        return []

    @property
    def result(self):
        return self.rpc.call("rpc_job_result", self.jid)


class JobTrackerClient:
    """JobClient runner for ``mapred.job.tracker=host:port``."""

    def __init__(self, address, conf=None):
        self.rpc = RpcClient(address)

    def submit_job(self, job):
        from .jobclient import RunningJob
        jid = self.rpc.call("rpc_submit_job", job.to_dict())
        return RunningJob(jid, _RemoteJob(self.rpc, jid), job)
