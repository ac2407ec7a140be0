"""Pipes binary protocol, parent side.

Message codes and framing are the Hadoop Pipes ones (hadoop-1.0.3/src/mapred/
org/apache/hadoop/mapred/pipes/BinaryProtocol.java:66-85): Hadoop VInts and
VInt-length-prefixed byte strings over a loopback TCP socket, 128 KB buffers.
Down (parent → child): START, SET_JOB_CONF, SET_INPUT_TYPES, RUN_MAP, MAP_ITEM,
RUN_REDUCE, REDUCE_KEY, REDUCE_VALUE, CLOSE, ABORT, AUTHENTICATION_REQ.
Up (child → parent): OUTPUT, PARTITIONED_OUTPUT, STATUS, PROGRESS, DONE,
REGISTER_COUNTER, INCREMENT_COUNTER, AUTHENTICATION_RESP — parsed by
:class:`UplinkReader` on its own thread and dispatched to an OutputHandler.
Authentication: HMAC-SHA1(job token, challenge), base64 (Application.java:197-211).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import io
import logging
import os
import struct
import threading

from ..io.vint import encode_vint, read_vint
from ..io.writable import BytesWritable, Text, Writable

log = logging.getLogger("hbmr.pipes")

CURRENT_PROTOCOL_VERSION = 0

START, SET_JOB_CONF, SET_INPUT_TYPES, RUN_MAP, MAP_ITEM, RUN_REDUCE, REDUCE_KEY, REDUCE_VALUE, \
    CLOSE, ABORT, AUTHENTICATION_REQ = range(11)
OUTPUT, PARTITIONED_OUTPUT, STATUS, PROGRESS, DONE, REGISTER_COUNTER, INCREMENT_COUNTER, \
    AUTHENTICATION_RESP = range(50, 58)

BUFFER_SIZE = 128 * 1024


def create_digest(password: bytes, msg: str) -> str:
    return base64.b64encode(hmac.new(password, msg.encode(), hashlib.sha1).digest()).decode()


def to_wire(obj) -> bytes:
    """Text/BytesWritable go as their raw bytes, other Writables serialised
    (BinaryProtocol.writeObject, BinaryProtocol.java:349-369)."""
    if isinstance(obj, Text):
        return obj.bytes
    if isinstance(obj, BytesWritable):
        return obj.bytes
    if isinstance(obj, Writable):
        return obj.serialize()
    if isinstance(obj, str):
        return obj.encode()
    return bytes(obj)


def from_wire(raw: bytes, cls):
    if cls is Text:
        return Text(raw)
    if cls is BytesWritable:
        return BytesWritable(raw)
    return cls.deserialize(raw)


_SMALL_VINTS = [bytes((n,)) for n in range(128)]

# HBMR_PIPES_RAW=0: records go through Writable objects both ways (the byte
# paths below off; for A/B measurement)
RAW_FRAMES = os.environ.get("HBMR_PIPES_RAW", "1") != "0"


def frame_of_serialized(cls):
    """``cls``'s serialised bytes -> the VInt-length-prefixed frame its object
    goes down the pipe as (``_bytes(to_wire(obj))``), without building the
    object; None for subclasses of Text/BytesWritable (their to_wire differs)."""
    if not RAW_FRAMES:
        return None
    if cls is Text:
        return lambda s: s          # VInt length + UTF-8 already (bytes or memoryview)
    if cls is BytesWritable:
        return lambda s: encode_vint(len(s) - 4) + s[4:]
    if issubclass(cls, (Text, BytesWritable)) or not issubclass(cls, Writable):
        return None
    return lambda s: encode_vint(len(s)) + s


def frame_parts_of_serialized(cls):
    """frame_of_serialized as (VInt prefix, body view) — the frame written in
    two pieces, so a large value (a K-Means partials block, ~1 MB) goes to the
    socket from where it lies instead of through a joined copy."""
    if not RAW_FRAMES:
        return None
    if cls is Text:
        return lambda s: (b"", s)
    if cls is BytesWritable:
        return lambda s: (encode_vint(len(s) - 4), memoryview(s)[4:])
    if issubclass(cls, (Text, BytesWritable)) or not issubclass(cls, Writable):
        return None
    return lambda s: (encode_vint(len(s)), s)


class DownwardProtocol:
    def __init__(self, sock):
        self.sock = sock
        self.out = sock.makefile("wb", buffering=BUFFER_SIZE)
        self._lock = threading.Lock()

    def _int(self, v):
        self.out.write(encode_vint(int(v)))

    def _bytes(self, b):
        b = b if isinstance(b, (bytes, bytearray)) else str(b).encode()
        self.out.write(encode_vint(len(b)))
        self.out.write(b)

    def authenticate(self, digest, challenge):
        with self._lock:
            self._int(AUTHENTICATION_REQ)
            self._bytes(digest.encode())
            self._bytes(challenge.encode())
            self.out.flush()

    def start(self):
        with self._lock:
            self._int(START)
            self._int(CURRENT_PROTOCOL_VERSION)

    def set_job_conf(self, conf):
        items = list(conf) if not isinstance(conf, dict) else list(conf.items())
        # one buffer for the whole message (a few hundred strings per task)
        parts = [encode_vint(SET_JOB_CONF), encode_vint(2 * len(items))]
        small = _SMALL_VINTS            # lengths 0..127 are one byte (Hadoop VInt)
        for k, v in items:
            kb = str(k).encode()
            vb = ("" if v is None else str(v)).encode()
            nk, nv = len(kb), len(vb)
            parts += (small[nk] if nk < 128 else encode_vint(nk), kb,
                      small[nv] if nv < 128 else encode_vint(nv), vb)
        msg = b"".join(parts)
        with self._lock:
            self.out.write(msg)

    def set_input_types(self, key_type, value_type):
        with self._lock:
            self._int(SET_INPUT_TYPES)
            self._bytes(key_type.encode())
            self._bytes(value_type.encode())

    def run_map(self, split_bytes: bytes, num_reduces: int, piped_input: bool):
        with self._lock:
            self._int(RUN_MAP)
            self._bytes(split_bytes)
            self._int(num_reduces)
            self._int(1 if piped_input else 0)
            self.out.flush()

    def map_item(self, key, value):
        with self._lock:
            self._int(MAP_ITEM)
            self._bytes(to_wire(key))
            self._bytes(to_wire(value))

    def run_reduce(self, partition: int, piped_output: bool):
        with self._lock:
            self._int(RUN_REDUCE)
            self._int(partition)
            self._int(1 if piped_output else 0)

    def reduce_key(self, key):
        with self._lock:
            self._int(REDUCE_KEY)
            self._bytes(to_wire(key))

    def reduce_value(self, value):
        with self._lock:
            self._int(REDUCE_VALUE)
            self._bytes(to_wire(value))

    def reduce_group(self, key_frame: bytes, value_frames: list):
        """REDUCE_KEY and the REDUCE_VALUEs of one key group in one write
        (frames as made by :func:`frame_of_serialized`)."""
        sep = _SMALL_VINTS[REDUCE_VALUE]
        with self._lock:
            if sum(map(len, value_frames)) < (1 << 16):
                # small values: one joined write
                msg = _SMALL_VINTS[REDUCE_KEY] + key_frame
                if value_frames:
                    msg += sep + sep.join(value_frames)
                self.out.write(msg)
                return
            # big values (a K-Means partials block is ~1 MB): written as they
            # are (memoryviews, no joined copy); the buffered writer passes
            # writes above its buffer size straight to the socket
            w = self.out.write
            w(_SMALL_VINTS[REDUCE_KEY])
            w(key_frame)
            for f in value_frames:
                w(sep)
                w(f)

    def reduce_group_parts(self, key_frame: bytes, parts: list):
        """reduce_group with each value frame as (prefix, body) pieces
        (frame_parts_of_serialized): no per-value joined copy."""
        sep = _SMALL_VINTS[REDUCE_VALUE]
        with self._lock:
            w = self.out.write
            w(_SMALL_VINTS[REDUCE_KEY])
            w(key_frame)
            for pre, body in parts:
                w(sep + pre if pre else sep)
                w(body)

    def end_of_input(self):
        with self._lock:
            self._int(CLOSE)
            self.out.flush()

    def abort(self):
        with self._lock:
            try:
                self._int(ABORT)
                self.out.flush()
            except OSError:
                pass

    def flush(self):
        with self._lock:
            self.out.flush()

    def close(self):
        try:
            self.out.close()
        except OSError:
            pass


class UplinkReader(threading.Thread):
    """Reads child → parent messages and dispatches them to ``handler``."""

    def __init__(self, sock, handler, reuse=False):
        super().__init__(daemon=True, name="pipes-uplink")
        self.inp = sock.makefile("rb", buffering=BUFFER_SIZE)
        self.handler = handler
        # a reused child runs task after task on this connection: DONE ends a
        # task, not the stream, and each task installs its own handler
        self.reuse = reuse

    def _bytes(self):
        n = read_vint(self.inp)
        return self.inp.read(n) if n else b""

    #: room left in front of a large value read by _value: the longest
    #: serialisation prefix of a Text / BytesWritable payload (a 5-byte VInt)
    ROOM = 8

    def _value(self):
        """An OUTPUT value: small ones as bytes; a large one (a K-Means block)
        read in place into a buffer with ROOM spare bytes in front and handed
        on as a memoryview of its payload, so the map output buffer can put
        the serialisation prefix there instead of copying the value
        (hbmr.io.writable.serialize_in_place)."""
        n = read_vint(self.inp)
        if n < (1 << 16):
            return self.inp.read(n) if n else b""
        buf = bytearray(self.ROOM + n)
        mv = memoryview(buf)
        got = self.ROOM
        while got < len(buf):
            r = self.inp.readinto(mv[got:])
            if not r:
                raise EOFError("pipe child exited in a value")
            got += r
        return mv[self.ROOM:]

    def run(self):
        h = self.handler
        try:
            while True:
                cmd = read_vint(self.inp)
                h = self.handler
                if cmd == OUTPUT:
                    k = self._bytes()
                    v = self._value()
                    h.output(k, v)
                elif cmd == PARTITIONED_OUTPUT:
                    part = read_vint(self.inp)
                    k = self._bytes()
                    v = self._value()
                    h.partitioned_output(part, k, v)
                elif cmd == STATUS:
                    h.status(self._bytes().decode(errors="replace"))
                elif cmd == PROGRESS:
                    h.progress(struct.unpack(">f", self.inp.read(4))[0])
                elif cmd == DONE:
                    h.done()
                    if not self.reuse:
                        return
                elif cmd == REGISTER_COUNTER:
                    cid = read_vint(self.inp)
                    grp = self._bytes().decode()
                    name = self._bytes().decode()
                    h.register_counter(cid, grp, name)
                elif cmd == INCREMENT_COUNTER:
                    cid = read_vint(self.inp)
                    amount = read_vint(self.inp)
                    h.increment_counter(cid, amount)
                elif cmd == AUTHENTICATION_RESP:
                    h.authenticate(self._bytes().decode())
                else:
                    raise IOError(f"Bad command code: {cmd}")
        # (the handler installed NOW: one swapped in while this thread was
        # blocked reading — a reused child's next task, the GPU mux's FIFO
        # dispatcher — is the one waiting for the outcome; the stale one left
        # a mux child's maps waiting forever on a child that had died)
        except EOFError:
            self.handler.failed(IOError("pipe child exited before DONE"))
        except BaseException as e:  # noqa: BLE001
            self.handler.failed(e)


def read_all(data: bytes):
    """Decode a recorded downlink stream (debugging aid, cf. downlink.data tee)."""
    b = io.BytesIO(data)
    out = []
    while b.tell() < len(data):
        out.append(read_vint(b))
    return out
