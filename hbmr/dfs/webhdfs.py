"""WebHDFS: the HDFS REST API and the ``webhdfs://`` FileSystem over it.

Server — the NameNode's ``/webhdfs/v1/<path>?op=...`` resource and the
DataNodes' (hadoop-1.0.3/src/hdfs/org/apache/hadoop/hdfs/server/namenode/web/
resources/NamenodeWebHdfsMethods.java, .../datanode/web/resources/
DatanodeWebHdfsMethods.java).  Namespace operations answer at the NameNode;
data operations (OPEN, CREATE, APPEND, GETFILECHECKSUM) answer with a
307 redirect to the HTTP endpoint of a DataNode (the one holding the first
block read, or a live node chosen for the write — the write then lands its
first replica there), where the bytes move.  JSON bodies carry JsonUtil.java's
field names (FileStatus / FileStatuses / ContentSummary / FileChecksum /
LocatedBlocks / boolean / long / Path / Token) and errors are
``{"RemoteException": {exception, javaClassName, message}}`` with
ExceptionHandler.java's status mapping (404 FileNotFound, 401 security, 400
bad argument, 403 other IOExceptions).  Authentication is ``user.name``
(simple auth) or a ``delegation`` token this server issued
(GETDELEGATIONTOKEN / RENEW / CANCEL); ``doas`` for another user is refused
unless ``hadoop.proxyuser.<user>.users`` lists it.

Client — WebHdfsFileSystem.java: ``webhdfs://host:port/path`` with the
FileSystem API the MapReduce layer uses (status, listing, globbing, create,
open with seek as re-opened offset reads (OffsetUrlInputStream), rename,
delete, mkdirs, replication, owner/permission/times, content summary,
checksum, block locations, home directory, delegation tokens), registered in
:mod:`hbmr.fs` so jobs read and write ``webhdfs://`` paths.
"""
from __future__ import annotations

import base64
import fnmatch
import hashlib
import hmac
import http.client
import io
import json
import os
import secrets
import tempfile
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ..fs import FileStatus, hidden
from ..security import AccessControlException
from .client import DistributedFileSystem, namenode_for

PREFIX = "/webhdfs/v1"
SCHEME = "webhdfs"

GET_OPS = {"OPEN", "GETFILESTATUS", "LISTSTATUS", "GETCONTENTSUMMARY", "GETFILECHECKSUM",
           "GETHOMEDIRECTORY", "GETDELEGATIONTOKEN", "GET_BLOCK_LOCATIONS"}
PUT_OPS = {"CREATE", "MKDIRS", "RENAME", "SETREPLICATION", "SETOWNER", "SETPERMISSION",
           "SETTIMES", "RENEWDELEGATIONTOKEN", "CANCELDELEGATIONTOKEN"}
POST_OPS = {"APPEND"}
DELETE_OPS = {"DELETE"}
REDIRECT_OPS = {"OPEN", "CREATE", "APPEND", "GETFILECHECKSUM"}


class Unauthorized(Exception):
    """SecurityException / AuthorizationException → 401."""


# Python exception → (Java simple name, Java class name, HTTP status)
def _java(e):
    if isinstance(e, Unauthorized):
        return "SecurityException", "java.lang.SecurityException", 401
    if isinstance(e, FileNotFoundError):
        return "FileNotFoundException", "java.io.FileNotFoundException", 404
    if isinstance(e, AccessControlException):
        return ("AccessControlException",
                "org.apache.hadoop.security.AccessControlException", 403)
    if isinstance(e, FileExistsError):
        return ("FileAlreadyExistsException",
                "org.apache.hadoop.fs.FileAlreadyExistsException", 403)
    if isinstance(e, NotImplementedError):
        return "UnsupportedOperationException", "java.lang.UnsupportedOperationException", 400
    if isinstance(e, (ValueError, KeyError)):
        return "IllegalArgumentException", "java.lang.IllegalArgumentException", 400
    if isinstance(e, OSError):
        return "IOException", "java.io.IOException", 403
    return "RuntimeException", "java.lang.RuntimeException", 500


_FROM_JAVA = {"FileNotFoundException": FileNotFoundError,
              "AccessControlException": AccessControlException,
              "FileAlreadyExistsException": FileExistsError,
              "IllegalArgumentException": ValueError,
              "UnsupportedOperationException": NotImplementedError,
              "SecurityException": PermissionError,
              "AuthorizationException": PermissionError}


# -- JSON (JsonUtil.java) -----------------------------------------------------------------
def status_json(d, name=""):
    return {"pathSuffix": name, "type": "DIRECTORY" if d["is_dir"] else "FILE",
            "length": int(d["length"]), "owner": d.get("owner", ""), "group": d.get("group", ""),
            "permission": format(int(d.get("permission", 0o755)), "o"),
            "accessTime": int(d.get("atime", 0) * 1000),
            "modificationTime": int(d["mtime"] * 1000),
            "blockSize": int(d["block_size"] or 0), "replication": int(d["replication"] or 0)}


def located_blocks_json(nn, path, blocks, info):
    dns = {d["id"]: d for d in nn.datanode_report()}
    out = []
    for b in blocks:
        locs = [{"name": dns.get(i, {}).get("host", i), "hostName": dns.get(i, {}).get("host", i),
                 "storageID": i, "networkLocation": dns.get(i, {}).get("rack", "/default-rack"),
                 "capacity": dns.get(i, {}).get("capacity", 0),
                 "dfsUsed": dns.get(i, {}).get("used", 0), "adminState": "NORMAL"}
                for i in b["dns"]]
        out.append({"block": {"blockId": b["block"], "numBytes": b["length"],
                              "generationStamp": 0},
                    "startOffset": b["offset"], "isCorrupt": False, "locations": locs,
                    "blockToken": {"urlString": ""}})
    return {"LocatedBlocks": {"fileLength": int(info["length"]),
                              "isUnderConstruction": bool(info.get("under_construction")),
                              "locatedBlocks": out}}


# -- delegation tokens -----------------------------------------------------------------------
class TokenManager:
    """DelegationTokenSecretManager in miniature: HMAC-signed tokens with an
    owner, renewer, expiry (renew interval) and max lifetime; cancel revokes."""

    def __init__(self, renew_ms=24 * 3600 * 1000, max_ms=7 * 24 * 3600 * 1000):
        self.key = secrets.token_bytes(32)
        self.renew_ms, self.max_ms = renew_ms, max_ms
        self.live: dict[int, dict] = {}
        self.seq = 0
        self.lock = threading.Lock()

    def _sign(self, body: bytes) -> str:
        return base64.urlsafe_b64encode(hmac.new(self.key, body, hashlib.sha256).digest()[:18]) \
            .decode()

    def issue(self, owner, renewer):
        now = int(time.time() * 1000)
        with self.lock:
            self.seq += 1
            ident = {"owner": owner, "renewer": renewer or owner, "issue": now,
                     "max": now + self.max_ms, "seq": self.seq}
            self.live[self.seq] = {"ident": ident, "expiry": now + self.renew_ms}
        body = json.dumps(ident, sort_keys=True).encode()
        return base64.urlsafe_b64encode(body).decode() + "." + self._sign(body)

    def _ident(self, token: str):
        try:
            b64, sig = token.rsplit(".", 1)
            body = base64.urlsafe_b64decode(b64.encode())
        except Exception as e:  # noqa: BLE001
            raise Unauthorized(f"malformed delegation token: {e}") from None
        if not hmac.compare_digest(sig, self._sign(body)):
            raise Unauthorized("delegation token signature mismatch")
        return json.loads(body)

    def verify(self, token: str) -> str:
        ident = self._ident(token)
        with self.lock:
            rec = self.live.get(ident["seq"])
            if rec is None:
                raise Unauthorized("delegation token can't be found in cache")
            if rec["expiry"] < time.time() * 1000:
                raise Unauthorized("delegation token is expired")
        return ident["owner"]

    def renew(self, token: str, user: str) -> int:
        ident = self._ident(token)
        if user != ident["renewer"]:
            raise AccessControlException(f"{user} tries to renew a token with renewer "
                                         f"{ident['renewer']}")
        with self.lock:
            rec = self.live.get(ident["seq"])
            if rec is None:
                raise Unauthorized("delegation token can't be found in cache")
            rec["expiry"] = min(ident["max"], int(time.time() * 1000) + self.renew_ms)
            return rec["expiry"]

    def cancel(self, token: str, user: str):
        ident = self._ident(token)
        if user not in (ident["owner"], ident["renewer"]):
            raise AccessControlException(f"{user} is not authorized to cancel the token")
        with self.lock:
            if self.live.pop(ident["seq"], None) is None:
                raise Unauthorized("delegation token can't be found in cache")


# -- server ----------------------------------------------------------------------------------
def _params(query: str) -> dict:
    # parameter names are case-insensitive (ParamFilter.java), values are not
    return {k.lower(): v[-1] for k, v in urllib.parse.parse_qs(query, keep_blank_values=True)
            .items()}


def _bool(v, default=False):
    if v is None or v == "":
        return default
    if v.lower() in ("true", "false"):
        return v.lower() == "true"
    raise ValueError(f"Invalid value for boolean parameter: {v!r}")


def _int(v, default=None, name="value"):
    if v is None or v == "" or v.lower() == "null":
        return default
    try:
        return int(v)
    except ValueError:
        raise ValueError(f"Invalid value for webhdfs parameter \"{name}\": {v!r}") from None


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "hbmr-webhdfs"
    web: "WebHdfsServer" = None
    dn_host: str | None = None       # None: the NameNode endpoint

    def log_message(self, *a):  # quiet
        pass

    # -- plumbing
    def _send(self, code, body=b"", ctype="application/json", headers=()):
        if isinstance(body, (dict, list)):
            body = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        for k, v in headers:
            self.send_header(k, v)
        self.end_headers()
        if body and self.command != "HEAD":
            self.wfile.write(body)

    def _error(self, e):
        simple, java, code = _java(e)
        msg = str(e) or simple
        self._send(code, {"RemoteException": {"exception": simple, "javaClassName": java,
                                              "message": msg}})

    def _body(self) -> bytes:
        n = int(self.headers.get("Content-Length") or 0)
        return self.rfile.read(n) if n else b""

    def _dispatch(self, method):
        try:
            url = urllib.parse.urlsplit(self.path)
            if not url.path.startswith(PREFIX):
                raise FileNotFoundError(f"no resource {url.path}")
            path = urllib.parse.unquote(url.path[len(PREFIX):]) or "/"
            if not path.startswith("/"):
                raise ValueError(f"bad path {path!r}")
            q = _params(url.query)
            op = (q.get("op") or "").upper()
            allowed = {"GET": GET_OPS, "PUT": PUT_OPS, "POST": POST_OPS,
                       "DELETE": DELETE_OPS}[method]
            if op not in allowed:
                raise ValueError(f"Invalid value for webhdfs parameter \"op\": "
                                 f"{q.get('op')!r} is not a {method} operation")
            user = self.web.authenticate(q)
            if self.dn_host is None:
                self.web.namenode_op(self, method, op, path, q, user)
            else:
                self.web.datanode_op(self, op, path, q, user)
        except Exception as e:  # noqa: BLE001 — every failure is a RemoteException reply
            if method in ("PUT", "POST"):
                try:
                    self._body()
                except Exception:  # noqa: BLE001
                    pass
            self._error(e)

    def do_GET(self):  # noqa: N802
        self._dispatch("GET")

    def do_PUT(self):  # noqa: N802
        self._dispatch("PUT")

    def do_POST(self):  # noqa: N802
        self._dispatch("POST")

    def do_DELETE(self):  # noqa: N802
        self._dispatch("DELETE")


class WebHdfsServer:
    """HTTP endpoints of one DFS (``authority`` as for hdfs://): the NameNode's
    and one per DataNode host, each a threading HTTP server on ``host``."""

    def __init__(self, authority, conf=None, host="127.0.0.1", port=0):
        self.authority = authority
        self.conf = conf
        self.host = host
        self.nn = namenode_for(authority)
        self.tokens = TokenManager()
        self._servers = []
        self.nn_httpd = self._serve(None, port)
        self.dn_httpd: dict[str, ThreadingHTTPServer] = {}
        for d in self.nn.datanode_report():
            self._datanode_server(d["host"])

    def _serve(self, dn_host, port=0):
        handler = type("WebHdfsHandler", (_Handler,), {"web": self, "dn_host": dn_host})
        httpd = ThreadingHTTPServer((self.host, port), handler)
        httpd.daemon_threads = True
        threading.Thread(target=httpd.serve_forever, args=(0.05,), daemon=True,
                         name=f"webhdfs-{dn_host or 'nn'}").start()
        self._servers.append(httpd)
        return httpd

    def _datanode_server(self, dn_host):
        s = self.dn_httpd.get(dn_host)
        if s is None:
            s = self.dn_httpd[dn_host] = self._serve(dn_host)
        return s

    @property
    def address(self):
        return f"{self.host}:{self.nn_httpd.server_address[1]}"

    @property
    def uri(self):
        return f"{SCHEME}://{self.address}"

    def shutdown(self):
        for s in self._servers:
            s.shutdown()
            s.server_close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.shutdown()

    # -- auth (AuthFilter / UserProvider; simple auth + delegation tokens)
    def authenticate(self, q) -> str:
        tok = q.get("delegation")
        if tok:
            user = self.tokens.verify(tok)
        else:
            user = q.get("user.name") or ""
            if not user:
                import getpass
                user = getpass.getuser()
        doas = q.get("doas")
        if doas and doas != user:
            allowed = (self.conf.get(f"hadoop.proxyuser.{user}.users", "")
                       if self.conf is not None else "")
            if allowed != "*" and doas not in [u.strip() for u in allowed.split(",")]:
                raise Unauthorized(f"User: {user} is not allowed to impersonate {doas}")
            user = doas
        return user

    def _fs(self, dn_host=None):
        return DistributedFileSystem(self.authority, self.conf, host=dn_host)

    def _redirect(self, h, op, path, q, dn_host):
        s = self._datanode_server(dn_host)
        q = dict(q)
        q["op"] = op
        loc = (f"http://{self.host}:{s.server_address[1]}{PREFIX}"
               f"{urllib.parse.quote(path)}?{urllib.parse.urlencode(q)}")
        h._send(307, b"", "application/octet-stream", [("Location", loc)])

    def _pick_datanode(self, path=None, offset=0):
        """Host of the first replica of the block at ``offset`` (reads), else a
        live DataNode (writes) — NamenodeWebHdfsMethods.chooseDatanode."""
        if path is not None:
            for b in self.nn.get_block_locations(path, offset, 1):
                if b["hosts"]:
                    return b["hosts"][0]
        live = [d["host"] for d in self.nn.datanode_report() if d["alive"]]
        if not live:
            raise IOError("no live DataNodes")
        return live[secrets.randbelow(len(live))]

    # -- NameNode resource
    def namenode_op(self, h, method, op, path, q, user):
        nn = self.nn
        if op == "GETFILESTATUS":
            d = nn.get_file_info(path)
            if d is None:
                raise FileNotFoundError(f"File does not exist: {path}")
            return h._send(200, {"FileStatus": status_json(d)})
        if op == "LISTSTATUS":
            d = nn.get_file_info(path)
            if d is None:
                raise FileNotFoundError(f"File {path} does not exist.")
            items = nn.list_status(path)
            return h._send(200, {"FileStatuses": {"FileStatus": [
                status_json(x, "" if not d["is_dir"] else os.path.basename(x["path"]))
                for x in items]}})
        if op == "GETCONTENTSUMMARY":
            return h._send(200, {"ContentSummary": nn.get_content_summary(path)})
        if op == "GETHOMEDIRECTORY":
            return h._send(200, {"Path": f"/user/{user}"})
        if op == "GET_BLOCK_LOCATIONS":
            info = nn.get_file_info(path)
            if info is None or info["is_dir"]:
                raise FileNotFoundError(f"File does not exist: {path}")
            off = _int(q.get("offset"), 0, "offset")
            ln = _int(q.get("length"), None, "length")
            return h._send(200, located_blocks_json(nn, path,
                                                    nn.get_block_locations(path, off, ln), info))
        if op == "GETDELEGATIONTOKEN":
            return h._send(200, {"Token": {"urlString": self.tokens.issue(user,
                                                                          q.get("renewer"))}})
        if op == "RENEWDELEGATIONTOKEN":
            return h._send(200, {"long": self.tokens.renew(q.get("token") or "", user)})
        if op == "CANCELDELEGATIONTOKEN":
            self.tokens.cancel(q.get("token") or "", user)
            return h._send(200, b"", "application/octet-stream")
        if op == "MKDIRS":
            perm = int(q["permission"], 8) if q.get("permission") else None
            return h._send(200, {"boolean": bool(nn.mkdirs(path, owner=user, permission=perm))})
        if op == "RENAME":
            dst = q.get("destination")
            if not dst or not dst.startswith("/"):
                raise ValueError(f"Invalid value for webhdfs parameter \"destination\": {dst!r}")
            try:
                ok = bool(nn.rename(path, dst))
            except (FileNotFoundError, FileExistsError):
                ok = False
            return h._send(200, {"boolean": ok})
        if op == "SETREPLICATION":
            r = _int(q.get("replication"), None, "replication")
            if r is None:       # ReplicationParam's default: dfs.replication
                r = self.conf.get_int("dfs.replication", 3) if self.conf is not None else 3
            return h._send(200, {"boolean": bool(nn.set_replication(path, r))})
        if op == "SETOWNER":
            if not q.get("owner") and not q.get("group"):
                raise ValueError("Both owner and group are empty.")
            nn.set_owner(path, q.get("owner") or None, q.get("group") or None)
            return h._send(200, b"", "application/octet-stream")
        if op == "SETPERMISSION":
            perm = int(q["permission"], 8) if q.get("permission") else 0o755
            nn.set_permission(path, perm)
            return h._send(200, b"", "application/octet-stream")
        if op == "SETTIMES":
            mt = _int(q.get("modificationtime"), -1, "modificationtime")
            at = _int(q.get("accesstime"), -1, "accesstime")
            nn.set_times(path, mt / 1000.0 if mt >= 0 else -1, at / 1000.0 if at >= 0 else -1)
            return h._send(200, b"", "application/octet-stream")
        if op == "DELETE":
            rec = _bool(q.get("recursive"), False)
            try:
                ok = bool(nn.delete(path, rec))
            except OSError as e:
                if "non-empty" in str(e):
                    raise IOError(f"{path} is non empty") from None
                raise
            return h._send(200, {"boolean": ok})
        if op in ("OPEN", "GETFILECHECKSUM"):
            info = nn.get_file_info(path)
            if info is None:
                raise FileNotFoundError(f"File does not exist: {path}")
            if info["is_dir"]:
                raise FileNotFoundError(f"Path is not a file: {path}")
            off = _int(q.get("offset"), 0, "offset")
            if off < 0:
                raise ValueError("Invalid value for webhdfs parameter \"offset\": negative")
            return self._redirect(h, op, path, q, self._pick_datanode(path, off))
        if op == "CREATE":
            info = nn.get_file_info(path)
            if info is not None and (info["is_dir"] or not _bool(q.get("overwrite"), False)):
                raise FileExistsError(f"{path} already exists")
            q = dict(q, **{"user.name": user})
            q.pop("delegation", None)
            return self._redirect(h, op, path, q, self._pick_datanode())
        if op == "APPEND":
            info = nn.get_file_info(path)
            if info is None or info["is_dir"]:
                raise FileNotFoundError(f"failed to append to non-existent file {path}")
            q = dict(q, **{"user.name": user})
            q.pop("delegation", None)
            return self._redirect(h, op, path, q, self._pick_datanode(path, 0))
        raise NotImplementedError(f"{op} is not supported")

    # -- DataNode resource
    def datanode_op(self, h, op, path, q, user):
        fs = self._fs(h.dn_host)
        if op == "OPEN":
            off = _int(q.get("offset"), 0, "offset")
            ln = _int(q.get("length"), None, "length")
            info = self.nn.get_file_info(path)
            if info is None or info["is_dir"]:
                raise FileNotFoundError(f"File does not exist: {path}")
            n = max(0, int(info["length"]) - off)
            if ln is not None:
                n = min(n, ln)
            with fs.open(path) as f:
                f.seek(off)
                data = f.read(n) if n else b""
            return h._send(200, data, "application/octet-stream")
        if op == "GETFILECHECKSUM":
            alg, raw = fs.get_file_checksum(path)
            return h._send(200, {"FileChecksum": {"algorithm": alg, "bytes": raw.hex(),
                                                  "length": len(raw)}})
        if op == "CREATE":
            data = h._body()
            perm = int(q["permission"], 8) if q.get("permission") else None
            repl = _int(q.get("replication"), None, "replication")
            bs = _int(q.get("blocksize"), None, "blocksize")
            if self.nn.get_file_info(path) is not None and not _bool(q.get("overwrite"), False):
                raise FileExistsError(f"{path} already exists")
            with fs.create(path, overwrite=True, replication=repl, block_size=bs,
                           permission=perm, owner=user) as f:
                f.write(data)
            return h._send(201, b"", "application/octet-stream",
                           [("Location", f"{SCHEME}://{self.address}{path}")])
        if op == "APPEND":
            data = h._body()
            self._append(fs, path, data, user)
            return h._send(200, b"", "application/octet-stream")
        raise NotImplementedError(f"{op} is not a DataNode operation")

    def _append(self, fs, path, data, user):
        """No block-level append in this NameNode: rewrite the file as old bytes
        + new ones under a temporary name and rename it over the original
        (one writer at a time, like the HDFS lease), keeping its attributes."""
        info = self.nn.get_file_info(path)
        if info is None or info["is_dir"]:
            raise FileNotFoundError(f"failed to append to non-existent file {path}")
        with self._append_lock:
            tmp = f"{path}._append_{secrets.token_hex(4)}"
            with fs.open(path) as src, fs.create(tmp, replication=info["replication"] or None,
                                                 block_size=info["block_size"] or None,
                                                 permission=info.get("permission"),
                                                 owner=info.get("owner")) as dst:
                while True:
                    chunk = src.read(8 << 20)
                    if not chunk:
                        break
                    dst.write(chunk)
                dst.write(data)
            self.nn.delete(path, False)
            self.nn.rename(tmp, path)
            if info.get("group"):
                self.nn.set_owner(path, None, info["group"])

    _append_lock = threading.Lock()


# -- client ----------------------------------------------------------------------------------
def split_uri(path: str):
    p = str(path)
    if not p.startswith(f"{SCHEME}://"):
        raise ValueError(f"not a {SCHEME}:// path: {p}")
    auth, _, tail = p[len(SCHEME) + 3:].partition("/")
    return auth, "/" + tail


class WebHdfsFileStatus(FileStatus):
    def __init__(self, path, j):
        super().__init__(path, j["length"], j["type"] == "DIRECTORY", j["blockSize"],
                         j["modificationTime"] / 1000.0)
        self.owner, self.group = j["owner"], j["group"]
        self.permission = int(j["permission"], 8)
        self.access_time = j["accessTime"] / 1000.0
        self.replication = j["replication"]

    def getPermission(self):  # noqa: N802
        return self.permission

    def getOwner(self):  # noqa: N802
        return self.owner

    def getGroup(self):  # noqa: N802
        return self.group

    def getReplication(self):  # noqa: N802
        return self.replication


class _OffsetReader(io.RawIOBase):
    """OffsetUrlInputStream: reads are ranged OPENs from the current offset,
    so seek() costs nothing until the next read."""

    CHUNK = 8 << 20

    def __init__(self, fs, path, length):
        self.fs, self.path, self.length, self.pos = fs, path, length, 0

    def readable(self):
        return True

    def seekable(self):
        return True

    def seek(self, off, whence=0):
        self.pos = off if whence == 0 else self.pos + off if whence == 1 else self.length + off
        return self.pos

    def tell(self):
        return self.pos

    def readinto(self, buf):
        if self.pos >= self.length or not len(buf):
            return 0
        n = min(len(buf), self.CHUNK, self.length - self.pos)
        data = self.fs._call("GET", "OPEN", self.path, offset=self.pos, length=n)
        buf[:len(data)] = data
        self.pos += len(data)
        return len(data)


class _SpoolWriter(io.RawIOBase):
    """Bytes spool to a temporary file; close() sends them in one CREATE (or
    APPEND) request with a Content-Length."""

    def __init__(self, fs, op, path, params):
        self.fs, self.op, self.path, self.params = fs, op, path, params
        self.spool = tempfile.SpooledTemporaryFile(max_size=64 << 20)
        self._done = False

    def writable(self):
        return True

    def write(self, b):
        return self.spool.write(b)

    def close(self):
        if self._done:
            return
        self._done = True
        try:
            self.spool.seek(0)
            self.fs._call("PUT" if self.op == "CREATE" else "POST", self.op, self.path,
                          body=self.spool.read(), **self.params)
        finally:
            self.spool.close()
            super().close()


class WebHdfsFileSystem:
    scheme = SCHEME

    def __init__(self, authority, conf=None, user=None, token=None):
        self.authority = authority
        self.conf = conf
        host, _, port = authority.rpartition(":")
        self.host, self.port = host or authority, int(port or 50070)
        self.user = user or (conf.get("user.name") if conf is not None else None)
        if not self.user:
            import getpass
            self.user = getpass.getuser()
        self.token = token

    # -- transport
    def _p(self, path):
        p = str(path)
        if p.startswith(f"{SCHEME}://"):
            p = split_uri(p)[1]
        return "/" + p.strip("/") if p.strip("/") else "/"

    def _uri(self, p):
        return f"{SCHEME}://{self.authority}{p}"

    def url(self, op, path, **params):
        q = {"op": op}
        if self.token:
            q["delegation"] = self.token
        else:
            q["user.name"] = self.user
        q.update({k: v for k, v in params.items() if v is not None})
        return f"{PREFIX}{urllib.parse.quote(self._p(path))}?{urllib.parse.urlencode(q)}"

    @staticmethod
    def _raise(status, data):
        try:
            r = json.loads(data)["RemoteException"]
        except Exception:  # noqa: BLE001
            raise IOError(f"HTTP {status}: {data[:200]!r}") from None
        cls = _FROM_JAVA.get(r.get("exception"), IOError)
        raise cls(r.get("message"))

    def _request(self, host, port, method, url, body=None):
        c = http.client.HTTPConnection(host, port, timeout=120)
        try:
            headers = {"Content-Length": str(len(body))} if body is not None else {}
            c.request(method, url, body=body, headers=headers)
            r = c.getresponse()
            return r.status, dict(r.getheaders()), r.read()
        finally:
            c.close()

    def _call(self, method, op, path, body=None, **params):
        url = self.url(op, path, **params)
        if op in ("CREATE", "APPEND"):
            # two-step: the NameNode answers 307 without reading data
            st, hdr, data = self._request(self.host, self.port, method, url, body=b"")
        else:
            st, hdr, data = self._request(self.host, self.port, method, url)
        if st == 307:
            loc = urllib.parse.urlsplit(hdr.get("Location") or hdr.get("location"))
            st, hdr, data = self._request(loc.hostname, loc.port, method,
                                          f"{loc.path}?{loc.query}", body=body)
        if st >= 300:
            self._raise(st, data)
        if op == "OPEN":
            return data
        return json.loads(data) if data else None

    # -- FileSystem API
    def get_file_status(self, path):
        return WebHdfsFileStatus(self._uri(self._p(path)),
                                 self._call("GET", "GETFILESTATUS", path)["FileStatus"])

    getFileStatus = get_file_status  # noqa: N815

    def exists(self, path):
        try:
            self.get_file_status(path)
            return True
        except FileNotFoundError:
            return False

    def is_dir(self, path):
        try:
            return self.get_file_status(path).is_dir
        except FileNotFoundError:
            return False

    def list_status(self, path, filter_hidden=True):
        p = self._p(path)
        out = []
        for j in self._call("GET", "LISTSTATUS", p)["FileStatuses"]["FileStatus"]:
            q = p if not j["pathSuffix"] else p.rstrip("/") + "/" + j["pathSuffix"]
            out.append(WebHdfsFileStatus(self._uri(q), j))
        return [s for s in out if not (filter_hidden and hidden(s.path))]

    listStatus = list_status  # noqa: N815

    def listdir(self, path):
        return [j["pathSuffix"] for j in
                self._call("GET", "LISTSTATUS", path)["FileStatuses"]["FileStatus"]]

    def glob_status(self, pattern):
        parts = self._p(pattern).strip("/").split("/")
        cur = ["/"]
        for part in parts:
            nxt = []
            for c in cur:
                if not any(ch in part for ch in "*?["):
                    q = c.rstrip("/") + "/" + part
                    if self.exists(q):
                        nxt.append(q)
                    continue
                if self.is_dir(c):
                    nxt += [c.rstrip("/") + "/" + n for n in self.listdir(c)
                            if fnmatch.fnmatch(n, part)]
            cur = nxt
        return [self.get_file_status(q) for q in sorted(cur)]

    globStatus = glob_status  # noqa: N815

    def mkdirs(self, path, permission=None):
        perm = format(permission, "o") if permission is not None else None
        return self._call("PUT", "MKDIRS", path, permission=perm)["boolean"]

    def create(self, path, overwrite=True, replication=None, block_size=None, permission=None):
        params = {"overwrite": str(bool(overwrite)).lower(), "replication": replication,
                  "blocksize": block_size,
                  "permission": format(permission, "o") if permission is not None else None}
        return io.BufferedWriter(_SpoolWriter(self, "CREATE", self._p(path), params), 1 << 20)

    def append(self, path):
        return io.BufferedWriter(_SpoolWriter(self, "APPEND", self._p(path), {}), 1 << 20)

    def open(self, path, buffering=1 << 20):
        st = self.get_file_status(path)
        if st.is_dir:
            raise FileNotFoundError(f"{path} is a directory")
        return io.BufferedReader(_OffsetReader(self, self._p(path), st.length),
                                 max(buffering, 8192))

    def rename(self, src, dst):
        return self._call("PUT", "RENAME", src, destination=self._p(dst))["boolean"]

    def delete(self, path, recursive=True):
        return self._call("DELETE", "DELETE", path, recursive=str(bool(recursive)).lower())[
            "boolean"]

    def set_replication(self, path, r):
        return self._call("PUT", "SETREPLICATION", path, replication=r)["boolean"]

    def set_owner(self, path, owner=None, group=None):
        self._call("PUT", "SETOWNER", path, owner=owner, group=group)

    def set_permission(self, path, permission):
        self._call("PUT", "SETPERMISSION", path, permission=format(permission, "o"))

    def set_times(self, path, mtime=-1, atime=-1):
        """Milliseconds since the epoch (FileSystem.setTimes); -1 = unchanged."""
        self._call("PUT", "SETTIMES", path, modificationtime=mtime, accesstime=atime)

    def get_content_summary(self, path):
        return self._call("GET", "GETCONTENTSUMMARY", path)["ContentSummary"]

    def get_file_checksum(self, path):
        j = self._call("GET", "GETFILECHECKSUM", path)["FileChecksum"]
        return j["algorithm"], bytes.fromhex(j["bytes"])

    def get_home_directory(self):
        return self._call("GET", "GETHOMEDIRECTORY", "/")["Path"]

    def get_file_block_locations(self, path, start, length):
        j = self._call("GET", "GET_BLOCK_LOCATIONS", path, offset=start, length=length)
        return [(b["startOffset"], b["block"]["numBytes"], [x["hostName"] for x in b["locations"]])
                for b in j["LocatedBlocks"]["locatedBlocks"]]

    def get_delegation_token(self, renewer=None):
        return self._call("GET", "GETDELEGATIONTOKEN", "/", renewer=renewer)["Token"]["urlString"]

    def renew_delegation_token(self, token):
        return self._call("PUT", "RENEWDELEGATIONTOKEN", "/", token=token)["long"]

    def cancel_delegation_token(self, token):
        self._call("PUT", "CANCELDELEGATIONTOKEN", "/", token=token)

    def get_default_block_size(self):
        return self.conf.get_long("dfs.block.size", 64 << 20) if self.conf is not None \
            else 64 << 20

    getDefaultBlockSize = get_default_block_size  # noqa: N815
