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


class NameNode:
    METHODS = ["mkdirs", "create", "add_block", "complete", "get_block_locations",
               "get_file_info", "list_status", "rename", "delete", "set_replication",
               "register_datanode", "dn_heartbeat", "block_received", "block_report",
               "report_bad_block", "fsck", "datanode_report", "save_namespace", "safemode",
               "datanode_address", "decommission"]

    def __init__(self, conf=None, name_dir=None):
        g = (lambda k, d: conf.get_int(k, d)) if conf is not None else (lambda k, d: d)
        gl = (lambda k, d: conf.get_long(k, d)) if conf is not None else (lambda k, d: d)
        gf = (lambda k, d: conf.get_float(k, d)) if conf is not None else (lambda k, d: d)
        self.block_size = gl("dfs.block.size", DEFAULT_BLOCK_SIZE)
        self.replication = g("dfs.replication", 3)
        self.dead_interval = g("dfs.namenode.dead.interval.ms", 630000) / 1000.0
        self.monitor_interval = g("dfs.replication.interval.ms", 1000) / 1000.0
        self.safemode_pct = gf("dfs.safemode.threshold.pct", 0.999)
        self.name_dir = name_dir
        self.lock = threading.RLock()
        self.inodes: dict[str, dict] = {"/": {"type": "dir", "mtime": time.time()}}
        self.blocks: dict[int, dict] = {}         # id -> {"len", "locs": set, "file"}
        self.datanodes: dict[str, dict] = {}
        self.invalidate: dict[str, set] = {}      # dn -> block ids to delete
        self.pending_repl: dict[int, float] = {}  # block -> deadline
        self.leases: dict[str, str] = {}
        self.next_block = 1
        self.safe_mode = False
        self.manual_safe_mode = False
        self._edits = None
        self._stop = threading.Event()
        if name_dir:
            os.makedirs(name_dir, exist_ok=True)
            self._load()
            self._edits = open(os.path.join(name_dir, "edits"), "a", buffering=1)
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
        for ino in self.inodes.values():
            if ino["type"] == "file":
                for b in ino["blocks"]:
                    self.blocks[b["id"]] = {"len": b["len"], "locs": set(), "file": None}
        ed = os.path.join(self.name_dir, "edits")
        if os.path.exists(ed):
            with open(ed) as f:
                for line in f:
                    line = line.strip()
                    if line:
                        self._replay(json.loads(line))
        for path, ino in self.inodes.items():
            if ino["type"] == "file":
                for b in ino["blocks"]:
                    self.blocks.setdefault(b["id"], {"len": b["len"], "locs": set()})["file"] = path

    def _replay(self, e):
        op = e["op"]
        if op == "mkdir":
            self.inodes[e["path"]] = {"type": "dir", "mtime": e["t"]}
        elif op == "create":
            self.inodes[e["path"]] = {"type": "file", "blocks": [], "repl": e["repl"],
                                      "bs": e["bs"], "len": 0, "mtime": e["t"], "uc": True}
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

    def save_namespace(self):
        """Checkpoint: write fsimage.json, truncate the edit log."""
        if not self.name_dir:
            return False
        with self.lock:
            tmp = os.path.join(self.name_dir, "fsimage.json.tmp")
            with open(tmp, "w") as f:
                json.dump({"inodes": self.inodes, "next_block": self.next_block}, f)
            os.replace(tmp, os.path.join(self.name_dir, "fsimage.json"))
            self._edits.close()
            self._edits = open(os.path.join(self.name_dir, "edits"), "w", buffering=1)
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

    def mkdirs(self, path):
        p = norm(path)
        with self.lock:
            self._check_safe()
            t = time.time()
            for q in reversed([p] + self._parents(p)):
                ino = self.inodes.get(q)
                if ino is None:
                    self._log("mkdir", path=q, t=t)
                    self.inodes[q] = {"type": "dir", "mtime": t}
                elif ino["type"] != "dir":
                    raise NotADirectoryError(q)
        return True

    def create(self, path, overwrite=True, replication=None, block_size=None, client=""):
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
                self.mkdirs(parent)
            repl = int(replication or self.replication)
            bs = int(block_size or self.block_size)
            t = time.time()
            self._log("create", path=p, repl=repl, bs=bs, t=t)
            self.inodes[p] = {"type": "file", "blocks": [], "repl": repl, "bs": bs, "len": 0,
                              "mtime": t, "uc": True}
            self.leases[p] = client
        return {"block_size": bs, "replication": repl}

    def add_block(self, path, client="", prev_len=0, writer_host=None):
        p = norm(path)
        with self.lock:
            self._check_safe()
            ino = self.inodes.get(p)
            if ino is None or ino["type"] != "file" or not ino.get("uc"):
                raise FileNotFoundError(f"{p} is not open for writing")
            bid = self.next_block
            self.next_block += 1
            self._log("add_block", path=p, id=bid, prev_len=prev_len)
            if ino["blocks"]:
                ino["blocks"][-1]["len"] = prev_len
                self.blocks[ino["blocks"][-1]["id"]]["len"] = prev_len
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
        return True

    def _info(self, p, ino):
        if ino["type"] == "dir":
            return {"path": p, "length": 0, "is_dir": True, "block_size": 0, "replication": 0,
                    "mtime": ino["mtime"]}
        return {"path": p, "length": ino["len"], "is_dir": False, "block_size": ino["bs"],
                "replication": ino["repl"], "mtime": ino["mtime"],
                "under_construction": bool(ino.get("uc"))}

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
            if ino is None:
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

    def check_replication(self):
        now = time.time()
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
                    targets = self.choose_targets(need, exclude=set(info["locs"]))
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
