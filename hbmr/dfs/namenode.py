"""NameNode: namespace, block map, placement, replication and safe mode.

Redesign of hadoop-1.0.3/src/hdfs/org/apache/hadoop/hdfs/server/namenode/
(FSNamesystem.java, FSDirectory.java, FSEditLog.java, FSImage.java,
LeaseManager.java, ReplicationTargetChooser / BlockPlacementPolicyDefault,
ReplicationMonitor inside FSNamesystem) for one node whose DataNodes are the
per-GPU NVMe / page-cache stores:

* namespace: absolute paths → directory or file inode (blocks, replication,
  block size, length, mtime, under-construction flag + lease holder);
* persistence: every mutation is appended to ``<dfs.name.dir>/edits`` (JSON
  lines) before it is applied; ``save_namespace`` writes ``fsimage.json`` and
  truncates the log (the SecondaryNameNode checkpoint); start-up loads the
  image and replays the log;
* block map: block id → length and the DataNodes holding it, rebuilt from
  DataNode block reports; the NameNode starts in **safe mode** and leaves it
  once ``dfs.safemode.threshold.pct`` of the blocks have a reported replica;
* placement: first replica on the writer's DataNode (same host), second on
  another rack when there is one, third on the second's rack, rest random;
* replication monitor: DataNodes silent for ``dfs.namenode.dead.interval.ms``
  are dead, their replicas dropped; under-replicated blocks get a replicate
  command (source → target) on the source's next heartbeat; deleted files'
  blocks and corrupt replicas are sent as invalidate commands.

All methods are plain calls (in-process) or RPC (``NameNode.METHODS`` over
:class:`hbmr.mapred.rpc.RpcServer`).
"""
from __future__ import annotations

import json
import logging
import os
import posixpath
import random
import threading
import time

log = logging.getLogger("hbmr.dfs.namenode")

DEFAULT_BLOCK_SIZE = 64 * 1024 * 1024


class SafeModeException(RuntimeError):
    pass


def norm(path: str) -> str:
    p = str(path)
    if "://" in p:
        p = p.split("://", 1)[1]
        p = "/" + p.split("/", 1)[1] if "/" in p else "/"
    p = posixpath.normpath("/" + p.lstrip("/"))
    return p


class QuotaExceededException(IOError):
    pass


class NameNode:
    METHODS = ["mkdirs", "create", "add_block", "complete", "get_block_locations",
               "get_file_info", "list_status", "rename", "delete", "set_replication",
               "register_datanode", "dn_heartbeat", "block_received", "block_report",
               "report_bad_block", "fsck", "datanode_report", "save_namespace", "safemode",
               "datanode_address", "decommission", "roll_edit_log", "get_checkpoint_files",
               "install_checkpoint", "get_blocks", "move_block", "pending_moves",
               "set_quota", "get_content_summary", "set_owner", "set_permission", "set_times"]

    def __init__(self, conf=None, name_dir=None, checkpoint_only=False):
        """checkpoint_only: load image + edits for an offline merge (the
        SecondaryNameNode's working copy): no monitor thread, no edit log."""
        g = (lambda k, d: conf.get_int(k, d)) if conf is not None else (lambda k, d: d)
        gl = (lambda k, d: conf.get_long(k, d)) if conf is not None else (lambda k, d: d)
        gf = (lambda k, d: conf.get_float(k, d)) if conf is not None else (lambda k, d: d)
        self.block_size = gl("dfs.block.size", DEFAULT_BLOCK_SIZE)
        self.replication = g("dfs.replication", 3)
        self.dead_interval = g("dfs.namenode.dead.interval.ms", 630000) / 1000.0
        self.monitor_interval = g("dfs.replication.interval.ms", 1000) / 1000.0
        self.safemode_pct = gf("dfs.safemode.threshold.pct", 0.999)
        self.name_dir = name_dir
        import getpass
        self.superuser = getpass.getuser()      # the NameNode's user owns what no one else does
        self.supergroup = conf.get("dfs.permissions.supergroup", "supergroup") \
            if conf is not None else "supergroup"
        self.lock = threading.RLock()
        self.inodes: dict[str, dict] = {"/": {"type": "dir", "mtime": time.time()}}
        self.blocks: dict[int, dict] = {}         # id -> {"len", "locs": set, "file"}
        self.datanodes: dict[str, dict] = {}
        self.invalidate: dict[str, set] = {}      # dn -> block ids to delete
        self.pending_repl: dict[int, float] = {}  # block -> deadline
        self.leases: dict[str, str] = {}
        self.lease_time: dict[str, float] = {}
        self.lease_hard_limit = g("dfs.lease.hard.limit.ms", 3600 * 1000) / 1000.0
        self.moves: dict[int, tuple] = {}          # block -> (src, dst, deadline) (Balancer)
        self.quotas: dict[str, dict] = {}          # dir -> {"ns": n, "ds": bytes}; -1 = none
        self.segment = 0                           # id of the open edit-log segment
        self.image_through = -1                    # last segment merged into fsimage
        self.next_block = 1
        self.safe_mode = False
        self.manual_safe_mode = False
        self._edits = None
        self._stop = threading.Event()
        if name_dir:
            os.makedirs(name_dir, exist_ok=True)
            self._load()
            if checkpoint_only:
                return
            ed = os.path.join(name_dir, "edits")
            fresh = not os.path.exists(ed) or os.path.getsize(ed) == 0
            self._edits = open(ed, "a", buffering=1)
            if fresh:
                self._log("segment", id=self.segment)
        self.safe_mode = bool(self.blocks)
        self._mon = threading.Thread(target=self._monitor, daemon=True, name="ReplicationMonitor")
        self._mon.start()

    # -- persistence (FSImage / FSEditLog) -------------------------------------------
    def _log(self, op, **kw):
        if self._edits is not None:
            self._edits.write(json.dumps({"op": op, **kw}) + "\n")
            self._edits.flush()
            os.fsync(self._edits.fileno())

    def _load(self):
        img = os.path.join(self.name_dir, "fsimage.json")
        if os.path.exists(img):
            with open(img) as f:
                d = json.load(f)
            self.inodes = d["inodes"]
            self.next_block = d["next_block"]
            self.quotas = d.get("quotas", {})
            self.image_through = d.get("through_segment", -1)
            self.segment = self.image_through + 1
        for ino in self.inodes.values():
            if ino["type"] == "file":
                for b in ino["blocks"]:
                    self.blocks[b["id"]] = {"len": b["len"], "locs": set(), "file": None}
        # edits.old = a rolled segment a checkpoint has not merged yet (a crash between
        # roll and install); skipped when the image already went through it
        for name in ("edits.old", "edits"):
            ed = os.path.join(self.name_dir, name)
            if not os.path.exists(ed):
                continue
            with open(ed) as f:
                lines = [json.loads(x) for x in f if x.strip()]
            if lines and lines[0].get("op") == "segment":
                if lines[0]["id"] <= self.image_through:
                    continue
                self.segment = max(self.segment, lines[0]["id"])
            for e in lines:
                self._replay(e)
        for path, ino in self.inodes.items():
            if ino["type"] == "file":
                for b in ino["blocks"]:
                    self.blocks.setdefault(b["id"], {"len": b["len"], "locs": set()})["file"] = path

    def _replay(self, e):
        op = e["op"]
        if op == "segment":
            return
        attrs = {k: e[k] for k in self.ATTRS if k in e}
        if op == "mkdir":
            self.inodes[e["path"]] = {"type": "dir", "mtime": e["t"], **attrs}
        elif op == "create":
            self.inodes[e["path"]] = {"type": "file", "blocks": [], "repl": e["repl"],
                                      "bs": e["bs"], "len": 0, "mtime": e["t"], "uc": True,
                                      **attrs}
        elif op == "add_block":
            ino = self.inodes[e["path"]]
            if ino["blocks"]:
                ino["blocks"][-1]["len"] = e["prev_len"]
            ino["blocks"].append({"id": e["id"], "len": 0})
            self.blocks[e["id"]] = {"len": 0, "locs": set(), "file": e["path"]}
            self.next_block = max(self.next_block, e["id"] + 1)
        elif op == "complete":
            ino = self.inodes[e["path"]]
            if ino["blocks"]:
                ino["blocks"][-1]["len"] = e["last_len"]
            ino["len"] = sum(b["len"] for b in ino["blocks"])
            ino["uc"] = False
            for b in ino["blocks"]:
                self.blocks.setdefault(b["id"], {"locs": set(), "file": e["path"]})["len"] = b["len"]
        elif op == "rename":
            self._do_rename(e["src"], e["dst"])
        elif op == "delete":
            self._do_delete(e["path"])
        elif op == "set_repl":
            self.inodes[e["path"]]["repl"] = e["repl"]
        elif op == "abandon_block":
            ino = self.inodes[e["path"]]
            ino["blocks"] = [b for b in ino["blocks"] if b["id"] != e["id"]]
            self.blocks.pop(e["id"], None)
        elif op == "set_quota":
            self.quotas[e["path"]] = {"ns": e["ns"], "ds": e["ds"]}
        elif op == "set_attrs":
            self.inodes[e["path"]].update(attrs)
        elif op == "set_times":
            self.inodes[e["path"]].update({k: e[k] for k in ("mtime", "atime") if k in e})

    def _image(self, through):
        return {"inodes": self.inodes, "next_block": self.next_block, "quotas": self.quotas,
                "through_segment": through}

    def save_namespace(self):
        """Checkpoint in place (dfsadmin -saveNamespace): write fsimage.json, start a
        new edit-log segment."""
        if not self.name_dir:
            return False
        with self.lock:
            tmp = os.path.join(self.name_dir, "fsimage.json.tmp")
            with open(tmp, "w") as f:
                json.dump(self._image(self.segment), f)
            os.replace(tmp, os.path.join(self.name_dir, "fsimage.json"))
            self.image_through = self.segment
            self.segment += 1
            old = os.path.join(self.name_dir, "edits.old")
            if os.path.exists(old):
                os.remove(old)
            if self._edits is not None:
                self._edits.close()
            self._edits = open(os.path.join(self.name_dir, "edits"), "w", buffering=1)
            self._log("segment", id=self.segment)
        return True

    # -- SecondaryNameNode protocol (rollEditLog / GetImageServlet / rollFsImage) ----------
    def roll_edit_log(self):
        """Close the current segment as edits.old and open a new one; the
        SecondaryNameNode then merges fsimage + edits.old offline."""
        if not self.name_dir:
            raise IOError("NameNode has no name dir")
        with self.lock:
            old = os.path.join(self.name_dir, "edits.old")
            if os.path.exists(old):
                return {"segment": self._old_segment(old), "rolled": False}
            self._edits.close()
            os.replace(os.path.join(self.name_dir, "edits"), old)
            rolled = self.segment
            self.segment += 1
            self._edits = open(os.path.join(self.name_dir, "edits"), "w", buffering=1)
            self._log("segment", id=self.segment)
        return {"segment": rolled, "rolled": True}

    @staticmethod
    def _old_segment(path):
        with open(path) as f:
            first = f.readline()
        return json.loads(first)["id"] if first.strip() else -1

    def get_checkpoint_files(self):
        """(fsimage text, edits.old text) — what GetImageServlet serves."""
        img = os.path.join(self.name_dir, "fsimage.json")
        old = os.path.join(self.name_dir, "edits.old")
        read = (lambda q: open(q).read() if os.path.exists(q) else "")
        return {"image": read(img), "edits": read(old)}

    def install_checkpoint(self, image_text, through_segment):
        """Replace fsimage with the merged one and drop edits.old (rollFsImage)."""
        with self.lock:
            old = os.path.join(self.name_dir, "edits.old")
            if not os.path.exists(old) or self._old_segment(old) != through_segment:
                raise IOError("checkpoint does not match the rolled edit log")
            d = json.loads(image_text)
            if d.get("through_segment") != through_segment:
                raise IOError("image was not merged through the rolled segment")
            tmp = os.path.join(self.name_dir, "fsimage.json.ckpt")
            with open(tmp, "w") as f:
                f.write(image_text)
            os.replace(tmp, os.path.join(self.name_dir, "fsimage.json"))
            os.remove(old)
            self.image_through = through_segment
        return True

    # -- namespace ----------------------------------------------------------------------
    def _check_safe(self):
        if self.safe_mode or self.manual_safe_mode:
            raise SafeModeException("Name node is in safe mode")

    def _parents(self, p):
        out = []
        while p != "/":
            p = posixpath.dirname(p)
            out.append(p)
        return out

    def mkdirs(self, path, owner=None, permission=None):
        p = norm(path)
        with self.lock:
            self._check_safe()
            t = time.time()
            new = [q for q in [p] + self._parents(p) if q not in self.inodes]
            if new:
                self._check_ns_quota(p, len(new))
            for q in reversed([p] + self._parents(p)):
                ino = self.inodes.get(q)
                if ino is None:
                    attrs = self._new_attrs(owner, permission if q == p else None)
                    self._log("mkdir", path=q, t=t, **attrs)
                    self.inodes[q] = {"type": "dir", "mtime": t, **attrs}
                elif ino["type"] != "dir":
                    raise NotADirectoryError(q)
        return True

    def create(self, path, overwrite=True, replication=None, block_size=None, client="",
               owner=None, permission=None):
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is not None:
                if ino["type"] == "dir":
                    raise IsADirectoryError(p)
                if not overwrite:
                    raise FileExistsError(p)
                if ino.get("uc") and self.leases.get(p) not in (None, client):
                    raise PermissionError(f"{p} is being written by {self.leases[p]}")
                self._delete_locked(p)
            parent = posixpath.dirname(p)
            if parent not in self.inodes:
                self.mkdirs(parent, owner)
            self._check_ns_quota(p, 1)
            repl = int(replication or self.replication)
            bs = int(block_size or self.block_size)
            t = time.time()
            attrs = self._new_attrs(owner, permission)
            self._log("create", path=p, repl=repl, bs=bs, t=t, **attrs)
            self.inodes[p] = {"type": "file", "blocks": [], "repl": repl, "bs": bs, "len": 0,
                              "mtime": t, "uc": True, **attrs}
            self.leases[p] = client
            self.lease_time[p] = time.time()
        return {"block_size": bs, "replication": repl}

    def add_block(self, path, client="", prev_len=0, writer_host=None):
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is None or ino["type"] != "file" or not ino.get("uc"):
                raise FileNotFoundError(f"{p} is not open for writing")
            if ino["blocks"]:
                ino["blocks"][-1]["len"] = prev_len
                self.blocks[ino["blocks"][-1]["id"]]["len"] = prev_len
            self._check_ds_quota(p, ino["bs"] * ino["repl"])
            self.lease_time[p] = time.time()
            bid = self.next_block
            self.next_block += 1
            self._log("add_block", path=p, id=bid, prev_len=prev_len)
            ino["blocks"].append({"id": bid, "len": 0})
            self.blocks[bid] = {"len": 0, "locs": set(), "file": p}
            targets = self.choose_targets(ino["repl"], writer_host)
            if not targets:
                raise IOError("no live DataNodes to place a block on")
        return {"block": bid, "targets": targets}

    def complete(self, path, client="", last_len=0):
        p = norm(path)
        with self.lock:
            ino = self.inodes.get(p)
            if ino is None or ino["type"] != "file":
                raise FileNotFoundError(p)
            self._log("complete", path=p, last_len=last_len)
            if ino["blocks"]:
                ino["blocks"][-1]["len"] = last_len
                self.blocks[ino["blocks"][-1]["id"]]["len"] = last_len
            ino["len"] = sum(b["len"] for b in ino["blocks"])
            ino["uc"] = False
            ino["mtime"] = time.time()
            self.leases.pop(p, None)
            self.lease_time.pop(p, None)
        return True

    # -- quotas (dfsadmin -setQuota/-setSpaceQuota, fs -count -q) ------------------------
    def _usage(self, d):
        pre = d.rstrip("/") + "/"
        names = space = 0
        dirs = files = length = 0
        for q, ino in self.inodes.items():
            if q == d or q.startswith(pre) or d == "/":
                names += 1
                if ino["type"] == "dir":
                    dirs += 1
                else:
                    files += 1
                    length += ino["len"]
                    space += sum(max(b["len"], 0) for b in ino["blocks"]) * ino["repl"]
                    if ino.get("uc") and ino["blocks"]:   # open last block: charged in full
                        space += max(0, ino["bs"] - ino["blocks"][-1]["len"]) * ino["repl"]
        return {"names": names, "space": space, "dirs": dirs, "files": files, "length": length}

    def _quota_dirs(self, p):
        return [q for q in [p] + self._parents(p) if q in self.quotas]

    def _check_ns_quota(self, p, n_new):
        for q in self._quota_dirs(p):
            ns = self.quotas[q]["ns"]
            if ns >= 0 and self._usage(q)["names"] + n_new > ns:
                raise QuotaExceededException(f"The NameSpace quota (directories and files) "
                                             f"of directory {q} is exceeded: quota={ns}")

    def _check_ds_quota(self, p, nbytes):
        for q in self._quota_dirs(p):
            ds = self.quotas[q]["ds"]
            if ds >= 0 and self._usage(q)["space"] + nbytes > ds:
                raise QuotaExceededException(f"The DiskSpace quota of {q} is exceeded: "
                                             f"quota={ds}")

    def set_quota(self, path, ns_quota=-1, ds_quota=-1):
        """ns_quota / ds_quota < 0 clears that quota (HdfsConstants.QUOTA_RESET)."""
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is None or ino["type"] != "dir":
                raise FileNotFoundError(f"{p} is not a directory")
            self._log("set_quota", path=p, ns=int(ns_quota), ds=int(ds_quota))
            if ns_quota < 0 and ds_quota < 0:
                self.quotas.pop(p, None)
            else:
                self.quotas[p] = {"ns": int(ns_quota), "ds": int(ds_quota)}
        return True

    def get_content_summary(self, path):
        p = norm(path)
        with self.lock:
            if p not in self.inodes:
                raise FileNotFoundError(p)
            u = self._usage(p)
            q = self.quotas.get(p, {"ns": -1, "ds": -1})
            return {"directoryCount": u["dirs"], "fileCount": u["files"], "length": u["length"],
                    "spaceConsumed": u["space"], "quota": q["ns"], "spaceQuota": q["ds"]}

    # -- Balancer support (NamenodeProtocol.getBlocks + replace-block) -----------------------
    def get_blocks(self, dn_id, max_bytes=None):
        with self.lock:
            out, tot = [], 0
            for bid, info in self.blocks.items():
                if dn_id in info["locs"] and info.get("file") and bid not in self.moves:
                    out.append({"block": bid, "len": info["len"], "locs": sorted(info["locs"])})
                    tot += info["len"]
                    if max_bytes is not None and tot >= max_bytes:
                        break
            return out

    def move_block(self, block, src, dst):
        """Copy a replica src → dst, then drop it from src (the Balancer's move)."""
        with self.lock:
            info = self.blocks.get(block)
            if info is None or src not in info["locs"] or dst in info["locs"]:
                return False
            d = self.datanodes.get(dst)
            if d is None or not d["alive"] or d["decommission"]:
                return False
            self.moves[block] = (src, dst, time.time() + 60.0)
            self.datanodes[src].setdefault("repl_cmds", []).append(
                {"cmd": "replicate", "block": block, "targets": [dst]})
        return True

    def pending_moves(self):
        with self.lock:
            now = time.time()
            for b in [b for b, m in self.moves.items() if m[2] < now]:
                self.moves.pop(b)
            return len(self.moves)

    def _info(self, p, ino):
        isdir = ino["type"] == "dir"
        perm = ino.get("perm", 0o777 if p == "/" else 0o755 if isdir else 0o644)
        attrs = {"owner": ino.get("owner") or self.superuser, "group": ino.get("group") or
                 self.supergroup, "permission": perm, "atime": ino.get("atime", 0.0 if isdir else
                                                                      ino["mtime"])}
        if isdir:
            return {"path": p, "length": 0, "is_dir": True, "block_size": 0, "replication": 0,
                    "mtime": ino["mtime"], **attrs}
        return {"path": p, "length": ino["len"], "is_dir": False, "block_size": ino["bs"],
                "replication": ino["repl"], "mtime": ino["mtime"],
                "under_construction": bool(ino.get("uc")), **attrs}

    # -- owner / permission / times (FSNamesystem.setOwner/setPermission/setTimes) -------
    ATTRS = ("owner", "group", "perm", "atime")

    def _new_attrs(self, owner, permission):
        a = {}
        if owner:
            a["owner"] = str(owner)
        if permission is not None:
            a["perm"] = int(permission) & 0o7777
        return a

    def _set_attrs(self, path, **attrs):
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is None:
                raise FileNotFoundError(p)
            self._log("set_attrs", path=p, **attrs)
            ino.update(attrs)
        return True

    def set_owner(self, path, owner=None, group=None):
        """Both None is an error (HDFS: "Both owner and group are null")."""
        if not owner and not group:
            raise ValueError("Both owner and group are empty")
        a = {}
        if owner:
            a["owner"] = str(owner)
        if group:
            a["group"] = str(group)
        return self._set_attrs(path, **a)

    def set_permission(self, path, permission):
        return self._set_attrs(path, perm=int(permission) & 0o7777)

    def set_times(self, path, mtime=-1, atime=-1):
        """Seconds since the epoch; -1 leaves a time unchanged."""
        a = {}
        if mtime is not None and mtime >= 0:
            a["mtime"] = float(mtime)
        if atime is not None and atime >= 0:
            a["atime"] = float(atime)
        if not a:
            return True
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is None:
                raise FileNotFoundError(p)
            self._log("set_times", path=p, **a)
            ino.update(a)
        return True

    def get_file_info(self, path):
        p = norm(path)
        with self.lock:
            ino = self.inodes.get(p)
            return None if ino is None else self._info(p, ino)

    def list_status(self, path):
        p = norm(path)
        with self.lock:
            ino = self.inodes.get(p)
            if ino is None:
                raise FileNotFoundError(p)
            if ino["type"] == "file":
                return [self._info(p, ino)]
            pre = p.rstrip("/") + "/"
            return [self._info(q, i) for q, i in sorted(self.inodes.items())
                    if q.startswith(pre) and "/" not in q[len(pre):] and q != p]

    def get_block_locations(self, path, offset=0, length=None):
        p = norm(path)
        with self.lock:
            ino = self.inodes.get(p)
            if ino is None or ino["type"] != "file":
                raise FileNotFoundError(p)
            out = []
            pos = 0
            end = float("inf") if length is None else offset + length
            for b in ino["blocks"]:
                blen = b["len"] if not (ino.get("uc") and b is ino["blocks"][-1]) else \
                    self.blocks[b["id"]]["len"]
                if pos + blen > offset and pos < end or (blen == 0 and pos == offset):
                    locs = [d for d in self.blocks.get(b["id"], {}).get("locs", ())
                            if self.datanodes.get(d, {}).get("alive")]
                    out.append({"block": b["id"], "offset": pos, "length": blen,
                                "dns": locs, "hosts": [self.datanodes[d]["host"] for d in locs]})
                pos += blen
            return out

    def _do_rename(self, s, d):
        moved = {q: i for q, i in self.inodes.items() if q == s or q.startswith(s.rstrip("/") + "/")}
        for q in moved:
            del self.inodes[q]
        for q, i in moved.items():
            nq = d + q[len(s):]
            self.inodes[nq] = i
            if i["type"] == "file":
                for b in i["blocks"]:
                    if b["id"] in self.blocks:
                        self.blocks[b["id"]]["file"] = nq
            if q in self.leases:
                self.leases[nq] = self.leases.pop(q)

    def rename(self, src, dst):
        s, d = norm(src), norm(dst)
        with self.lock:
            self._check_safe()
            if s not in self.inodes or s == "/":
                return False
            if d in self.inodes and self.inodes[d]["type"] == "dir":
                d = posixpath.join(d, posixpath.basename(s))
            if d in self.inodes or d.startswith(s.rstrip("/") + "/"):
                return False
            parent = posixpath.dirname(d)
            if parent not in self.inodes:
                self.mkdirs(parent)
            self._log("rename", src=s, dst=d)
            self._do_rename(s, d)
        return True

    def _do_delete(self, p):
        gone = [q for q in self.inodes if q == p or q.startswith(p.rstrip("/") + "/")]
        for q in gone:
            ino = self.inodes.pop(q)
            self.leases.pop(q, None)
            if ino["type"] == "file":
                for b in ino["blocks"]:
                    info = self.blocks.pop(b["id"], None)
                    if info:
                        for dn in info["locs"]:
                            self.invalidate.setdefault(dn, set()).add(b["id"])
        if p == "/":
            self.inodes["/"] = {"type": "dir", "mtime": time.time()}

    def _delete_locked(self, p):
        self._log("delete", path=p)
        self._do_delete(p)

    def delete(self, path, recursive=True):
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is None or p == "/":   # FSDirectory refuses to delete the root
                return False
            if ino["type"] == "dir" and not recursive and self.list_status(p):
                raise OSError(f"{p} is a non-empty directory")
            self._delete_locked(p)
        return True

    def set_replication(self, path, replication):
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is None or ino["type"] != "file":
                return False
            self._log("set_repl", path=p, repl=int(replication))
            ino["repl"] = int(replication)
        return True

    # -- DataNode protocol ----------------------------------------------------------------
    def register_datanode(self, dn_id, host, rack="/default-rack", capacity=0, address=None):
        with self.lock:
            self.datanodes[dn_id] = {"id": dn_id, "host": host, "rack": rack,
                                     "capacity": capacity, "used": 0, "alive": True,
                                     "last": time.time(), "address": address,
                                     "decommission": None}
        return {"block_size": self.block_size}

    def datanode_address(self, dn_id):
        with self.lock:
            d = self.datanodes.get(dn_id)
            return None if d is None else d.get("address")

    def dn_heartbeat(self, dn_id, used=0, remaining=0):
        with self.lock:
            d = self.datanodes.get(dn_id)
            if d is None:
                return [{"cmd": "register"}]
            d["last"] = time.time()
            d["used"] = used
            if not d["alive"]:
                d["alive"] = True
            cmds = []
            inv = self.invalidate.pop(dn_id, None)
            if inv:
                cmds.append({"cmd": "delete", "blocks": sorted(inv)})
            for item in d.pop("repl_cmds", []):
                cmds.append(item)
            return cmds

    def block_received(self, dn_id, block, length):
        with self.lock:
            info = self.blocks.get(block)
            if info is None:   # file deleted meanwhile: drop the replica
                self.invalidate.setdefault(dn_id, set()).add(block)
                return False
            info["locs"].add(dn_id)
            info["len"] = max(info.get("len", 0), length)
            self.pending_repl.pop(block, None)
            # a fresh good replica must not be hit by an older queued delete
            self.invalidate.get(dn_id, set()).discard(block)
            mv = self.moves.get(block)
            if mv is not None and mv[1] == dn_id:   # balancer move landed: drop the source
                self.moves.pop(block)
                if mv[0] in info["locs"] and len(info["locs"]) > 1:
                    info["locs"].discard(mv[0])
                    self.invalidate.setdefault(mv[0], set()).add(block)
        return True

    def block_report(self, dn_id, blocks):
        with self.lock:
            for bid, length in blocks:
                info = self.blocks.get(bid)
                if info is None:
                    self.invalidate.setdefault(dn_id, set()).add(bid)
                else:
                    info["locs"].add(dn_id)
            self._check_leave_safemode()
        return True

    def report_bad_block(self, block, dn_id):
        with self.lock:
            info = self.blocks.get(block)
            if info is not None and dn_id in info["locs"]:
                info["locs"].discard(dn_id)
                self.invalidate.setdefault(dn_id, set()).add(block)
                log.warning("corrupt replica of block %s on %s", block, dn_id)
        return True

    def decommission(self, dn_id):
        """Start decommissioning: the node takes no new replicas and its blocks
        are re-replicated elsewhere; it is decommissioned once none depends on it."""
        with self.lock:
            d = self.datanodes.get(dn_id)
            if d is None:
                return False
            d["decommission"] = "in progress"
        return True

    def _check_leave_safemode(self):
        if not self.safe_mode:
            return
        total = len(self.blocks)
        have = sum(1 for b in self.blocks.values() if b["locs"])
        if total == 0 or have >= self.safemode_pct * total:
            self.safe_mode = False
            log.info("leaving safe mode: %d/%d blocks reported", have, total)

    def safemode(self, action="get"):
        with self.lock:
            if action == "enter":
                self.manual_safe_mode = True
            elif action == "leave":
                self.manual_safe_mode = False
                self.safe_mode = False
            return self.safe_mode or self.manual_safe_mode

    # -- placement ----------------------------------------------------------------------------
    def _live(self, exclude=()):
        return [d for d in self.datanodes.values()
                if d["alive"] and d["id"] not in exclude and not d["decommission"]]

    def choose_targets(self, n, writer_host=None, exclude=()):
        live = self._live(exclude)
        random.shuffle(live)
        out = []
        if writer_host:
            local = [d for d in live if d["host"] == writer_host]
            if local:
                out.append(local[0])
        for d in live:
            if len(out) >= n:
                break
            if d in out:
                continue
            if len(out) == 1 and len({x["rack"] for x in live}) > 1 and d["rack"] == out[0]["rack"]:
                continue   # second replica off the first's rack
            if len(out) == 2 and d["rack"] != out[1]["rack"] and \
                    any(x["rack"] == out[1]["rack"] and x not in out for x in live):
                continue   # third replica on the second's rack
            out.append(d)
        for d in live:      # relax rack rules if we could not fill
            if len(out) >= n:
                break
            if d not in out:
                out.append(d)
        return [d["id"] for d in out[:n]]

    # -- replication monitor -------------------------------------------------------------------
    def _monitor(self):
        while not self._stop.wait(self.monitor_interval):
            try:
                self.check_replication()
            except Exception:  # noqa: BLE001
                log.exception("replication monitor")

    def recover_leases(self):
        """Files whose writer vanished past the hard limit are closed with the
        lengths the DataNodes hold (LeaseManager.Monitor → internalReleaseLease)."""
        now = time.time()
        with self.lock:
            for p, t in list(self.lease_time.items()):
                ino = self.inodes.get(p)
                if ino is None or not ino.get("uc"):
                    self.lease_time.pop(p, None)
                    continue
                if now - t < self.lease_hard_limit:
                    continue
                last = 0
                if ino["blocks"]:
                    info = self.blocks.get(ino["blocks"][-1]["id"], {})
                    last = info.get("len", 0)
                    if not info.get("locs"):   # last block never reached a DataNode
                        dead = ino["blocks"].pop()
                        self.blocks.pop(dead["id"], None)
                        self._log("abandon_block", path=p, id=dead["id"])
                        last = ino["blocks"][-1]["len"] if ino["blocks"] else 0
                log.warning("lease of %s (holder %s) expired; closing the file", p,
                            self.leases.get(p))
                self.complete(p, self.leases.get(p, ""), last)

    def check_replication(self):
        now = time.time()
        self.recover_leases()
        with self.lock:
            for d in self.datanodes.values():
                if d["alive"] and now - d["last"] > self.dead_interval:
                    d["alive"] = False
                    log.warning("DataNode %s is dead", d["id"])
                    for info in self.blocks.values():
                        info["locs"].discard(d["id"])
            for path, ino in self.inodes.items():
                if ino["type"] != "file" or ino.get("uc"):
                    continue
                for b in ino["blocks"]:
                    info = self.blocks.get(b["id"])
                    if info is None:
                        continue
                    live = [x for x in info["locs"] if self.datanodes.get(x, {}).get("alive")]
                    counted = [x for x in live if not self.datanodes[x]["decommission"]]
                    need = ino["repl"] - len(counted)
                    if need <= 0 or not live:
                        continue
                    if self.pending_repl.get(b["id"], 0) > now:
                        continue
                    doomed = {dn for dn, inv in self.invalidate.items() if b["id"] in inv}
                    targets = self.choose_targets(need, exclude=set(info["locs"]) | doomed)
                    if not targets:
                        continue
                    src = random.choice(live)
                    self.datanodes[src].setdefault("repl_cmds", []).append(
                        {"cmd": "replicate", "block": b["id"], "targets": targets})
                    self.pending_repl[b["id"]] = now + 10 * self.monitor_interval + 5
            for d in self.datanodes.values():
                if d["decommission"] == "in progress" and not any(
                        d["id"] in info["locs"] and len([x for x in info["locs"]
                                                         if not self.datanodes[x]["decommission"]
                                                         and self.datanodes[x]["alive"]]) <
                        self.inodes.get(info.get("file") or "", {}).get("repl", 1)
                        for info in self.blocks.values()):
                    d["decommission"] = "decommissioned"

    # -- reports ---------------------------------------------------------------------------------
    def fsck(self, path="/"):
        """Health of the files under path (DFSck / NamenodeFsck)."""
        p = norm(path)
        with self.lock:
            files = blocks = missing = under = 0
            size = 0
            bad = []
            for q, ino in sorted(self.inodes.items()):
                if ino["type"] != "file" or not (q == p or q.startswith(p.rstrip("/") + "/")):
                    continue
                files += 1
                size += ino["len"]
                for b in ino["blocks"]:
                    blocks += 1
                    info = self.blocks.get(b["id"], {"locs": set()})
                    live = [x for x in info["locs"] if self.datanodes.get(x, {}).get("alive")]
                    if not live:
                        missing += 1
                        bad.append(f"{q}: block {b['id']} MISSING")
                    elif len(live) < ino["repl"]:
                        under += 1
            return {"path": p, "files": files, "blocks": blocks, "bytes": size,
                    "missing_blocks": missing, "under_replicated_blocks": under,
                    "status": "HEALTHY" if missing == 0 else "CORRUPT", "problems": bad[:100]}

    def datanode_report(self):
        with self.lock:
            out = []
            for d in self.datanodes.values():
                nblocks = sum(1 for b in self.blocks.values() if d["id"] in b["locs"])
                out.append({k: d[k] for k in ("id", "host", "rack", "capacity", "used", "alive",
                                              "decommission")} | {"blocks": nblocks})
            return out

    def shutdown(self):
        self._stop.set()
        if self._edits is not None:
            self._edits.close()
            self._edits = None
