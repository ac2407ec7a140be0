"""Length-prefixed msgpack RPC over TCP — the control plane between processes.

Replaces Hadoop IPC (hadoop-1.0.3/src/core/org/apache/hadoop/ipc/{RPC,Server,
Client}.java, Writable-serialised calls with listener/reader/handler/responder
threads) for the only remote interfaces hbmr needs on one node: the
InterTrackerProtocol (heartbeat / wakeup) and the JobSubmissionProtocol
(submit / status / kill).  Frames: 4-byte big-endian length + msgpack
``{"m": method, "a": args, "k": kwargs}`` → ``{"r": result}`` or ``{"e": error}``.
Sockets use TCP_NODELAY; clients keep one connection per thread so a
long-polling heartbeat never blocks a concurrent wakeup.

Authentication (hbmr.security): every call carries the caller's user name
(Hadoop "simple" auth), which the server installs as the current
UserGroupInformation while the method runs (ACL checks use it).  A server
given a cluster secret (``hbmr.rpc.secret`` / ``HBMR_RPC_SECRET``) first sends
a random challenge and only serves connections that answer
HMAC-SHA256(secret, challenge ‖ user); the user is then taken from the
authenticated handshake, not from the calls.
"""
from __future__ import annotations

import hmac
import json
import logging
import os
import secrets as _secrets
import socket
import socketserver
import struct
import threading
import time

import msgpack

log = logging.getLogger("hbmr.rpc")

_LEN = struct.Struct(">I")

# per-method (calls, seconds in the handler incl. the reply) of this process's
# RPC servers; on with HBMR_SAMPLE_PROF (reported by hbmr.utils.sampler)
# HBMR_RPC_TRACE=prefix: one JSON line per served call (time, method, the
# tracker, its reports and bulk completions, the kinds of action returned) in
# prefix_<pid>.jsonl — the control plane's message flow, call by call
_TR = (open(f"{os.environ['HBMR_RPC_TRACE']}_{os.getpid()}.jsonl", "w", buffering=1)
       if os.environ.get("HBMR_RPC_TRACE") else None)


def _trace(m, req, res):
    args = req.get("a") or [None]
    st = args[0]
    info = {}
    if isinstance(st, dict) and "tracker_name" in st:
        info = {"tracker": st["tracker_name"], "kw": req.get("k", {}),
                "reports": [[r.get("attempt_id"), r.get("state")]
                            for r in st.get("task_reports") or ()],
                "bulk": [len(b["attempts"]) for b in st.get("bulk_reports") or ()]}
    elif args[0] is not None:
        info = {"args": [a for a in args if isinstance(a, (str, int, float, bool))]}
    if isinstance(res, dict) and "actions" in res:
        info["actions"] = [[x.get("type"), x.get("job_id") or
                            (x.get("task") or {}).get("attempt_id")] for x in res["actions"]]
    _TR.write(json.dumps([round(time.time(), 5), m, info]) + "\n")


RPC_STATS: dict | None = {} if os.environ.get("HBMR_SAMPLE_PROF") else None


def _send(sock, obj):
    data = msgpack.packb(obj, use_bin_type=True)
    sock.sendall(_LEN.pack(len(data)) + data)


def _recv_exact(sock, n):
    data = sock.recv(n)             # the common case: all of it in one read
    if len(data) == n:
        return data
    if not data:
        raise ConnectionError("connection closed")
    buf = bytearray(data)
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("connection closed")
        buf += chunk
    return bytes(buf)


# HBMR_RPC_DUMP=path: the raw request frames this process serves, appended
# to path_<pid>.bin (4-byte length + msgpack each) — payload sizes and decode
# costs of the control plane's real messages, offline (tools/rpc_payloads.py)
_DUMP = (open(f"{os.environ['HBMR_RPC_DUMP']}_{os.getpid()}.bin", "ab")
         if os.environ.get("HBMR_RPC_DUMP") else None)


def _recv_buffered(f):
    """One message from a connection's buffered reader (the length word and
    the body usually arrive in one recv)."""
    head = f.read(4)
    if len(head) < 4:
        raise ConnectionError("connection closed")
    (n,) = _LEN.unpack(head)
    body = f.read(n)
    if len(body) < n:
        raise ConnectionError("connection closed")
    if _DUMP is not None:
        _DUMP.write(head + body)
    return msgpack.unpackb(body, raw=False, strict_map_key=False)


def _recv(sock):
    (n,) = _LEN.unpack(_recv_exact(sock, 4))
    return msgpack.unpackb(_recv_exact(sock, n), raw=False, strict_map_key=False)


_ENV = object()


def _conf_secret(conf):
    from ..security import rpc_secret
    return rpc_secret(conf)


def _secret(v):
    if v is _ENV:
        from ..security import rpc_secret
        return rpc_secret(None)
    return v.encode() if isinstance(v, str) else v


class RpcServer:
    def __init__(self, target, methods, host="0.0.0.0", port=0, secret=_ENV):
        from ..security import UserGroupInformation, rpc_response
        self.target = target
        self.methods = set(methods)
        self.secret = _secret(secret)
        outer = self

        class Handler(socketserver.BaseRequestHandler):
            def _authenticate(self, s):
                nonce = _secrets.token_bytes(16)
                _send(s, {"challenge": nonce})
                auth = _recv(s)
                user = str(auth.get("user", "")) if isinstance(auth, dict) else ""
                want = rpc_response(outer.secret, nonce, user)
                if not (isinstance(auth, dict) and isinstance(auth.get("auth"), str) and
                        hmac.compare_digest(auth["auth"], want)):
                    _send(s, {"e": "AccessControlException: RPC authentication failed"})
                    return None
                _send(s, {"r": "ok"})
                return user

            def handle(self):
                s = self.request
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                authed = None
                if outer.secret:
                    try:
                        authed = self._authenticate(s)
                    except (ConnectionError, OSError, ValueError):
                        return
                    if authed is None:
                        return
                # requests and replies alternate on a connection, so a
                # buffered reader cannot read past the next request
                rf = s.makefile("rb", buffering=1 << 16)
                ugis = {}
                while True:
                    try:
                        req = _recv_buffered(rf)
                    except (ConnectionError, OSError, ValueError):
                        return
                    m = req.get("m")
                    user = authed or req.get("u")
                    try:
                        if m not in outer.methods:
                            raise AttributeError(f"no RPC method {m!r}")
                        # (thread CPU, not wall: a long-poll's wait is not cost)
                        t0 = time.thread_time() if RPC_STATS is not None else 0.0
                        if user:
                            # doAs: the caller's identity on this thread's stack
                            ugi = ugis.get(user)
                            if ugi is None:
                                ugi = ugis[user] = UserGroupInformation.create_remote_user(user)
                            with ugi.do_as():
                                res = getattr(outer.target, m)(*req.get("a", ()),
                                                               **req.get("k", {}))
                        else:
                            res = getattr(outer.target, m)(*req.get("a", ()),
                                                           **req.get("k", {}))
                        _send(s, {"r": res})
                        if _TR is not None:
                            _trace(m, req, res)
                        if RPC_STATS is not None:
                            if isinstance(res, dict) and "actions" in res:
                                # heartbeat / report: by the kinds of action returned
                                m = m + ":" + ("+".join(sorted({a.get("type", "?") for a in
                                                                res["actions"]})) or "-")
                            st = RPC_STATS.setdefault(m, [0, 0.0])
                            st[0] += 1
                            st[1] += time.thread_time() - t0
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
    def __init__(self, address: str, timeout: float = 600.0, secret=_ENV):
        host, port = address.rsplit(":", 1)
        self.addr = (host, int(port))
        self.timeout = timeout
        self.secret = _secret(secret)
        self._tl = threading.local()

    def _sock(self):
        s = getattr(self._tl, "sock", None)
        if s is not None and self.secret:
            from ..security import UserGroupInformation
            if getattr(self._tl, "user", None) != UserGroupInformation.get_current_user().user:
                s.close()   # the handshake bound another identity: reconnect
                s = self._tl.sock = None
        if s is None:
            s = socket.create_connection(self.addr, timeout=self.timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            if self.secret:
                self._handshake(s)
            self._tl.sock = s
        return s

    def _handshake(self, s):
        from ..security import UserGroupInformation, rpc_response
        hello = _recv(s)
        if "challenge" not in hello:
            raise RpcError(f"server did not start the RPC handshake: {hello}")
        user = UserGroupInformation.get_current_user().user
        self._tl.user = user
        _send(s, {"user": user, "auth": rpc_response(self.secret, hello["challenge"], user)})
        resp = _recv(s)
        if "e" in resp:
            s.close()
            raise RpcError(resp["e"])

    def call(self, method, *args, **kwargs):
        from ..security import UserGroupInformation
        user = UserGroupInformation.get_current_user().user
        for attempt in range(2):
            s = self._sock()
            try:
                _send(s, {"m": method, "a": list(args), "k": kwargs, "u": user})
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
        if "challenge" in resp:
            self.close()
            raise RpcError("server requires RPC authentication (set hbmr.rpc.secret)")
        return resp.get("r")

    def close(self):
        s = getattr(self._tl, "sock", None)
        if s is not None:
            s.close()
            self._tl.sock = None


JT_METHODS = ("heartbeat", "wakeup", "report", "resend", "map_completion_events", "rpc_submit_job",
              "rpc_job_status", "rpc_kill_job", "rpc_job_result", "rpc_cluster_status",
              "rpc_list_jobs", "rpc_task_reports", "rpc_wait_job", "rpc_job_info",
              "rpc_wait_job_info")
# served by a JobTracker process to the node that started it (hbmr/mapred/jtprocess.py)
JT_PROCESS_METHODS = JT_METHODS + ("rpc_wait_for_trackers", "rpc_start_expiry",
                                   "rpc_broadcast_shutdown", "rpc_live_trackers",
                                   "rpc_cost_model", "rpc_cpu_seconds", "rpc_thread_cpu",
                                   "rpc_stop")


class JobTrackerProxy:
    """TaskTracker/JobClient-side stub of a remote JobTracker."""

    def __init__(self, address, conf=None):
        self.rpc = RpcClient(address, secret=_conf_secret(conf))
        self.address = address

    def heartbeat(self, status, initial=False, accept_new_tasks=True, block=0.0):
        return self.rpc.call("heartbeat", status, initial=initial,
                             accept_new_tasks=accept_new_tasks, block=block)

    def wakeup(self, tracker_name, seq=None):
        return self.rpc.call("wakeup", tracker_name, seq)

    def resend(self, tracker_name, after_seq):
        return self.rpc.call("resend", tracker_name, after_seq)

    def report(self, status, assign=False):
        return self.rpc.call("report", status, assign)

    def map_completion_events(self, job_id, start=0, wait=0.0):
        return self.rpc.call("map_completion_events", job_id, start, wait)


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
        self.rpc = RpcClient(address, secret=_conf_secret(conf))

    def submit_job(self, job):
        from .jobclient import RunningJob
        jid = self.rpc.call("rpc_submit_job", job.to_dict())
        return RunningJob(jid, _RemoteJob(self.rpc, jid), job)
