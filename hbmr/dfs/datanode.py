"""DataNode: block storage with per-chunk CRC32, pipelined writes, heartbeats.

Redesign of hadoop-1.0.3/src/hdfs/org/apache/hadoop/hdfs/server/datanode/
(DataNode.java, FSDataset.java, BlockReceiver.java, BlockSender.java,
DataBlockScanner.java; DataTransferProtocol OP_WRITE_BLOCK / OP_READ_BLOCK,
protocol/DataTransferProtocol.java:43-47).  One DataNode per storage device
(on an 8×MI355X node: the NVMe drive next to each GPU's NUMA domain), named
by the host its TaskTracker uses so input splits read by a GPU come from its
local drive:

* a block is ``blk_<id>`` plus ``blk_<id>.meta``: one CRC32 per
  ``io.bytes.per.checksum`` (512) bytes, verified on every read and by the
  block scanner; a mismatch is reported to the NameNode, which invalidates
  that replica and re-replicates from a good one;
* writes are pipelined: the client sends the block to the first target,
  which stores it and forwards it to the rest of the pipeline;
* a heartbeat thread reports usage and executes the NameNode's commands
  (delete blocks, replicate a block to other DataNodes).
"""
from __future__ import annotations

import logging
import os
import struct
import threading
import time
import zlib

log = logging.getLogger("hbmr.dfs.datanode")

_registry: dict[str, "DataNode"] = {}


class ChecksumError(IOError):
    pass


def resolve_datanode(nn, dn_id):
    """In-process DataNode object, else an RPC proxy from the NameNode's record."""
    dn = _registry.get(dn_id)
    if dn is not None:
        return dn
    addr = nn.datanode_address(dn_id)
    if not addr:
        raise IOError(f"DataNode {dn_id} unreachable")
    from .client import RpcProxy
    return RpcProxy(addr)


class DataNode:
    METHODS = ["write_block", "read_block", "block_length", "block_checksum", "ping"]

    def __init__(self, conf, namenode, dn_id, host, data_dir, rack="/default-rack",
                 serve_rpc=False):
        g = (lambda k, d: conf.get_int(k, d)) if conf is not None else (lambda k, d: d)
        self.conf = conf
        self.bpc = g("io.bytes.per.checksum", 512)
        self.hb_interval = g("dfs.heartbeat.interval.ms", 3000) / 1000.0
        self.nn = namenode
        self.id = dn_id
        self.host = host
        self.rack = rack
        self.dir = data_dir
        os.makedirs(data_dir, exist_ok=True)
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self.server = None
        address = None
        if serve_rpc:
            from ..mapred.rpc import RpcServer
            self.server = RpcServer(self, self.METHODS, host="127.0.0.1").start()
            address = f"127.0.0.1:{self.server.port}"
        _registry[dn_id] = self
        self.nn.register_datanode(dn_id, host, rack, capacity=self._capacity(), address=address)
        self.nn.block_report(dn_id, self.stored_blocks())
        self._hb = threading.Thread(target=self._heartbeats, daemon=True, name=f"dn-{dn_id}")
        self._hb.start()

    # -- storage ----------------------------------------------------------------------------
    def _path(self, bid):
        return os.path.join(self.dir, f"blk_{bid}")

    def _capacity(self):
        """Configured capacity (``dfs.datanode.capacity`` bytes, hbmr key) or the
        volume size, minus ``dfs.datanode.du.reserved``."""
        c = self.conf
        fixed = c.get_long("dfs.datanode.capacity", 0) if c is not None else 0
        reserved = c.get_long("dfs.datanode.du.reserved", 0) if c is not None else 0
        if fixed > 0:
            return max(0, fixed - reserved)
        try:
            st = os.statvfs(self.dir)
            return max(0, st.f_blocks * st.f_frsize - reserved)
        except OSError:
            return 0

    def stored_blocks(self):
        out = []
        for fn in os.listdir(self.dir):
            if fn.startswith("blk_") and not fn.endswith((".meta", ".tmp")):
                try:
                    size = os.path.getsize(os.path.join(self.dir, fn))
                except FileNotFoundError:
                    continue        # deleted (an invalidation) since the listing
                out.append([int(fn[4:]), size])
        return out

    def _crcs(self, data: bytes) -> bytes:
        b = self.bpc
        return b"".join(struct.pack(">I", zlib.crc32(data[i:i + b]) & 0xFFFFFFFF)
                        for i in range(0, len(data), b))

    def write_block(self, bid, data: bytes, pipeline=()):
        """Store a block, forward it down the pipeline (OP_WRITE_BLOCK)."""
        data = bytes(data)
        tmp = self._path(bid) + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        with open(self._path(bid) + ".meta", "wb") as f:
            f.write(struct.pack(">I", self.bpc) + self._crcs(data))
        os.replace(tmp, self._path(bid))
        self.nn.block_received(self.id, bid, len(data))
        if pipeline:
            nxt = resolve_datanode(self.nn, pipeline[0])
            try:
                nxt.write_block(bid, data, list(pipeline[1:]))
            except Exception as e:  # noqa: BLE001 — the NameNode re-replicates later
                log.warning("pipeline forward of block %s to %s failed: %s", bid, pipeline[0], e)
        return len(data)

    def block_length(self, bid):
        p = self._path(bid)
        return os.path.getsize(p) if os.path.exists(p) else -1

    def read_block(self, bid, offset=0, length=None):
        """Bytes [offset, offset+length) of a block, checksum-verified (OP_READ_BLOCK)."""
        p = self._path(bid)
        if not os.path.exists(p):
            raise FileNotFoundError(f"block {bid} not on {self.id}")
        size = os.path.getsize(p)
        end = size if length is None else min(size, offset + length)
        b = self.bpc
        c0, c1 = offset // b, (end + b - 1) // b
        with open(p, "rb") as f:
            f.seek(c0 * b)
            chunk = f.read((c1 - c0) * b)
        with open(p + ".meta", "rb") as f:
            f.seek(4 + 4 * c0)
            sums = f.read(4 * (c1 - c0))
        for i in range(c1 - c0):
            piece = chunk[i * b:(i + 1) * b]
            if struct.pack(">I", zlib.crc32(piece) & 0xFFFFFFFF) != sums[4 * i:4 * i + 4]:
                raise ChecksumError(f"checksum error in block {bid} chunk {c0 + i} on {self.id}")
        return chunk[offset - c0 * b:end - c0 * b]

    def block_checksum(self, bid):
        """OP_BLOCK_CHECKSUM: bytes per CRC, CRCs in the block, MD5 of its CRCs."""
        import hashlib
        p = self._path(bid) + ".meta"
        if not os.path.exists(p):
            raise FileNotFoundError(f"block {bid} not on {self.id}")
        with open(p, "rb") as f:
            meta = f.read()
        crcs = meta[4:]
        return {"bpc": struct.unpack(">I", meta[:4])[0], "crc_per_block": len(crcs) // 4,
                "md5": hashlib.md5(crcs).hexdigest()}

    def verify_all(self):
        """DataBlockScanner pass: returns (and reports) corrupt block ids."""
        bad = []
        for bid, _ in self.stored_blocks():
            try:
                self.read_block(bid)
            except ChecksumError:
                bad.append(bid)
                self.nn.report_bad_block(bid, self.id)
            except FileNotFoundError:
                pass   # invalidated and deleted while we scanned
        return bad

    def ping(self):
        return self.id

    # -- heartbeat + commands ---------------------------------------------------------------
    def _heartbeats(self):
        while not self._stop.wait(self.hb_interval):
            try:
                self.heartbeat()
            except Exception as e:  # noqa: BLE001
                log.debug("heartbeat of %s failed: %s", self.id, e)

    def heartbeat(self):
        used = sum(s for _, s in self.stored_blocks())
        for cmd in self.nn.dn_heartbeat(self.id, used, 0):
            kind = cmd["cmd"]
            if kind == "delete":
                for bid in cmd["blocks"]:
                    for q in (self._path(bid), self._path(bid) + ".meta"):
                        if os.path.exists(q):
                            os.remove(q)
            elif kind == "replicate":
                try:
                    data = self.read_block(cmd["block"])
                except (ChecksumError, FileNotFoundError):
                    self.nn.report_bad_block(cmd["block"], self.id)
                    continue
                tgt = cmd["targets"]
                resolve_datanode(self.nn, tgt[0]).write_block(cmd["block"], data, tgt[1:])
            elif kind == "register":
                self.nn.register_datanode(self.id, self.host, self.rack, self._capacity())
                self.nn.block_report(self.id, self.stored_blocks())

    def shutdown(self):
        self._stop.set()
        _registry.pop(self.id, None)
        if self.server is not None:
            self.server.stop()
