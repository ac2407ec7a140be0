"""DFSClient / DistributedFileSystem: the ``hdfs://`` FileSystem.

Redesign of hadoop-1.0.3/src/hdfs/org/apache/hadoop/hdfs/DFSClient.java
(DFSOutputStream: buffer a block, ``addBlock`` for targets, write the
pipeline, ``complete`` on close; DFSInputStream: block locations, read from
the closest replica, on a checksum error report the bad block and fail over
to the next replica) and DistributedFileSystem.java (the FileSystem API the
MapReduce layer uses: status, listing, globbing, rename, delete, mkdirs,
block locations for split placement).

``hdfs://<authority>/path``: the authority names a NameNode registered in
this process (:func:`register_namenode`, as MiniDFSCluster does) or a
``host:port`` NameNode RPC endpoint.
"""
from __future__ import annotations

import fnmatch
import io
import logging
import os
import socket
import threading
import uuid

from ..fs import STATS
from .datanode import ChecksumError, resolve_datanode
from .namenode import norm

log = logging.getLogger("hbmr.dfs.client")

_namenodes: dict = {}
_lock = threading.Lock()


def register_namenode(authority: str, nn):
    with _lock:
        _namenodes[authority] = nn


def unregister_namenode(authority: str):
    with _lock:
        _namenodes.pop(authority, None)


class RpcProxy:
    """Method calls → RPC calls (NameNode / DataNode over hbmr.mapred.rpc)."""

    def __init__(self, address):
        from ..mapred.rpc import RpcClient
        self._rpc = RpcClient(address)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return lambda *a, **k: self._rpc.call(name, *a, **k)


def namenode_for(authority: str):
    with _lock:
        nn = _namenodes.get(authority)
    if nn is not None:
        return nn
    if ":" in authority:
        return RpcProxy(authority)
    raise IOError(f"unknown NameNode {authority!r}")


def split_uri(path: str):
    p = str(path)
    if not p.startswith("hdfs://"):
        raise ValueError(f"not an hdfs:// path: {p}")
    rest = p[len("hdfs://"):]
    auth, _, tail = rest.partition("/")
    return auth, "/" + tail


class DFSOutputStream(io.RawIOBase):
    def __init__(self, fs, path, block_size):
        self.fs = fs
        self.path = path
        self.block_size = block_size
        self.buf = bytearray()
        self.prev_len = 0
        self.total = 0
        self._closed = False

    def writable(self):
        return True

    def write(self, b):
        STATS.add("hdfs", written=len(b))
        self.buf += b
        while len(self.buf) >= self.block_size:
            self._flush_block(bytes(self.buf[:self.block_size]))
            del self.buf[:self.block_size]
        return len(b)

    def _flush_block(self, data: bytes):
        nn = self.fs.nn
        r = nn.add_block(self.path, self.fs.client, self.prev_len, self.fs.host)
        targets = r["targets"]
        last = None
        for i, t in enumerate(targets):   # pipeline, skipping dead heads
            try:
                resolve_datanode(nn, t).write_block(r["block"], data, targets[i + 1:])
                last = None
                break
            except Exception as e:  # noqa: BLE001
                last = e
        if last is not None:
            raise IOError(f"could not write block {r['block']} to any of {targets}: {last}")
        self.prev_len = len(data)
        self.total += len(data)

    def tell(self):
        return self.total + len(self.buf)

    def close(self):
        if self._closed:
            return
        self._closed = True
        if self.buf:
            self._flush_block(bytes(self.buf))
            self.buf.clear()
        self.fs.nn.complete(self.path, self.fs.client, self.prev_len)
        super().close()


class DFSInputStream(io.RawIOBase):
    def __init__(self, fs, path):
        self.fs = fs
        self.path = path
        self.blocks = fs.nn.get_block_locations(path, 0, None)
        self.length = sum(b["length"] for b in self.blocks)
        self.pos = 0
        self.dead = set()

    def readable(self):
        return True

    def seekable(self):
        return True

    def seek(self, off, whence=0):
        if whence == 0:
            self.pos = off
        elif whence == 1:
            self.pos += off
        else:
            self.pos = self.length + off
        return self.pos

    def tell(self):
        return self.pos

    def _replicas(self, b):
        dns = list(b["dns"])
        local = [d for d, h in zip(b["dns"], b["hosts"]) if h == self.fs.host]
        return local + [d for d in dns if d not in local]

    def _read_at(self, b, off, n):
        last = None
        for dn in self._replicas(b):
            if dn in self.dead:
                continue
            try:
                return resolve_datanode(self.fs.nn, dn).read_block(b["block"], off, n)
            except ChecksumError as e:
                self.fs.nn.report_bad_block(b["block"], dn)
                last = e
            except Exception as e:  # noqa: BLE001
                self.dead.add(dn)
                last = e
        raise IOError(f"could not read block {b['block']} of {self.path}: {last}")

    def readinto(self, buf):
        n = len(buf)
        if self.pos >= self.length or n == 0:
            return 0
        for b in self.blocks:
            if b["offset"] <= self.pos < b["offset"] + b["length"]:
                off = self.pos - b["offset"]
                want = min(n, b["length"] - off, 8 << 20)
                data = self._read_at(b, off, want)
                buf[:len(data)] = data
                self.pos += len(data)
                STATS.add("hdfs", read=len(data))
                return len(data)
        return 0


class DistributedFileSystem:
    scheme = "hdfs"

    def __init__(self, authority, conf=None, host=None):
        self.authority = authority
        self.conf = conf
        self.nn = namenode_for(authority)
        self.host = host or (conf.get("slave.host.name") if conf is not None else None) or \
            socket.gethostname()
        self.client = f"DFSClient_{uuid.uuid4().hex[:8]}"

    def _p(self, path):
        if str(path).startswith("hdfs://"):
            return split_uri(path)[1]
        return norm(path)

    def _uri(self, p):
        return f"hdfs://{self.authority}{p}"

    def _status(self, d):
        from ..fs import FileStatus
        return FileStatus(self._uri(d["path"]), d["length"], d["is_dir"],
                          d["block_size"] or 0, d["mtime"])

    def get_file_status(self, path):
        d = self.nn.get_file_info(self._p(path))
        if d is None:
            raise FileNotFoundError(path)
        return self._status(d)

    getFileStatus = get_file_status  # noqa: N815

    def exists(self, path):
        return self.nn.get_file_info(self._p(path)) is not None

    def is_dir(self, path):
        d = self.nn.get_file_info(self._p(path))
        return bool(d and d["is_dir"])

    def list_status(self, path, filter_hidden=True):
        from ..fs import hidden
        out = [self._status(d) for d in self.nn.list_status(self._p(path))]
        return [s for s in out if not (filter_hidden and hidden(s.path))]

    listStatus = list_status  # noqa: N815

    def listdir(self, path):
        return [os.path.basename(d["path"]) for d in self.nn.list_status(self._p(path))]

    def glob_status(self, pattern):
        p = self._p(pattern)
        parts = p.strip("/").split("/")
        cur = ["/"]
        for part in parts:
            nxt = []
            for c in cur:
                if not any(ch in part for ch in "*?["):
                    q = (c.rstrip("/") + "/" + part)
                    if self.nn.get_file_info(q) is not None:
                        nxt.append(q)
                    continue
                for d in self.nn.list_status(c) if self.is_dir(c) else []:
                    if fnmatch.fnmatch(os.path.basename(d["path"]), part):
                        nxt.append(d["path"])
            cur = nxt
        return [self.get_file_status(q) for q in sorted(cur)]

    globStatus = glob_status  # noqa: N815

    def mkdirs(self, path, permission=None, owner=None):
        if permission is None and owner is None:
            return self.nn.mkdirs(self._p(path))
        return self.nn.mkdirs(self._p(path), owner=owner, permission=permission)

    def create(self, path, overwrite=True, replication=None, block_size=None, permission=None,
               owner=None):
        p = self._p(path)
        if permission is None and owner is None:
            r = self.nn.create(p, overwrite, replication, block_size, self.client)
        else:
            r = self.nn.create(p, overwrite, replication, block_size, self.client, owner=owner,
                               permission=permission)
        return io.BufferedWriter(DFSOutputStream(self, p, r["block_size"]), 1 << 20)

    def open(self, path, buffering=1 << 20):
        return io.BufferedReader(DFSInputStream(self, self._p(path)), max(buffering, 8192))

    def rename(self, src, dst):
        return self.nn.rename(self._p(src), self._p(dst))

    def delete(self, path, recursive=True):
        return self.nn.delete(self._p(path), recursive)

    def set_replication(self, path, r):
        return self.nn.set_replication(self._p(path), r)

    def set_quota(self, path, ns_quota=-1, ds_quota=-1):
        return self.nn.set_quota(self._p(path), ns_quota, ds_quota)

    def get_content_summary(self, path):
        return self.nn.get_content_summary(self._p(path))

    def set_owner(self, path, owner=None, group=None):
        return self.nn.set_owner(self._p(path), owner, group)

    def set_permission(self, path, permission):
        return self.nn.set_permission(self._p(path), permission)

    def set_times(self, path, mtime=-1, atime=-1):
        return self.nn.set_times(self._p(path), mtime, atime)

    def get_file_checksum(self, path):
        """MD5MD5CRC32FileChecksum (DFSClient.getFileChecksum): the MD5 of the
        per-block MD5s of each block's CRC32s (``io.bytes.per.checksum`` chunks);
        crcPerBlock is 0 for a one-block file.  Returns (algorithm, 28 bytes)."""
        import hashlib
        import struct
        p = self._p(path)
        if self.is_dir(path):
            raise FileNotFoundError(f"{path} is a directory")
        blocks = self.nn.get_block_locations(p, 0, None)
        md5s, bpc, cpb = [], 512, 0
        for i, b in enumerate(blocks):
            last = None
            for dn in b["dns"]:
                try:
                    r = resolve_datanode(self.nn, dn).block_checksum(b["block"])
                    break
                except Exception as e:  # noqa: BLE001 — try the next replica
                    last = e
            else:
                raise IOError(f"no replica of block {b['block']} answered: {last}")
            md5s.append(bytes.fromhex(r["md5"]))
            bpc = r["bpc"]
            if i == 0 and len(blocks) > 1:
                cpb = r["crc_per_block"]
        md5 = hashlib.md5(b"".join(md5s)).digest()
        return f"MD5-of-{cpb}MD5-of-{bpc}CRC32", struct.pack(">iq", bpc, cpb) + md5

    def get_file_block_locations(self, path, start, length):
        """[(offset, length, [hosts])] of the blocks overlapping [start, start+length)."""
        return [(b["offset"], b["length"], b["hosts"])
                for b in self.nn.get_block_locations(self._p(path), start, length)]

    def get_default_block_size(self):
        return self.conf.get_long("dfs.block.size", 64 << 20) if self.conf is not None \
            else 64 << 20

    getDefaultBlockSize = get_default_block_size  # noqa: N815
