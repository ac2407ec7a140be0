"""The shared GPU Pipes child (hbmr/pipes/mux.py): what goes down its
command stream per attempt, and its in-flight depth.  Driven on a
bare MuxChild with a recording downlink; the GPU path itself runs in
tests/test_kmeans_pipes.py."""
import collections
import threading
import time

from hbmr.mapred.jobconf import JobConf
from hbmr.pipes import mux


class _Down:
    def __init__(self):
        self.log = []

    def set_job_conf(self, job):
        self.log.append(("conf", job.get("mapred.task.id")))

    def run_map(self, split, num_reduces, piped):
        self.log.append(("run_map", split))


class _App:
    def __init__(self):
        self.downlink = _Down()


def _bare(depth, first_conf):
    m = mux.MuxChild.__new__(mux.MuxChild)
    m.depth = depth
    m.fifo = collections.deque()
    m.cond = threading.Condition()
    m.dead = None
    m.send_lock = threading.Lock()
    m.maps = 0
    m.app = _App()
    shared = first_conf.get_boolean(mux.SHARED_CONF, False)
    m.conf_job = mux._job_key(first_conf) if shared else \
        (mux._job_key(first_conf),) + tuple(first_conf.get(k) for k in mux.TASK_KEYS)
    return m


def _attempt(i, job="202610180000_0001", shared=False):
    c = JobConf()
    c.set("mapred.task.id", f"attempt_{job}_m_{i:06d}_0")
    c.set("mapred.task.partition", str(i))
    c.set_boolean(mux.SHARED_CONF, shared)
    return c


def test_each_attempt_gets_its_own_conf_by_default():
    m = _bare(8, _attempt(0))
    for i in range(3):
        m.submit(_attempt(i), None, None, None, None, None, f"split{i}", 1)
    # attempt 0's conf went with the child's start; 1 and 2 get theirs
    assert m.app.downlink.log == [
        ("run_map", "split0"),
        ("conf", "attempt_202610180000_0001_m_000001_0"), ("run_map", "split1"),
        ("conf", "attempt_202610180000_0001_m_000002_0"), ("run_map", "split2")]


def test_shared_conf_apps_get_it_once_per_job():
    m = _bare(8, _attempt(0, shared=True))
    for i in range(3):
        m.submit(_attempt(i, shared=True), None, None, None, None, None, f"s{i}", 1)
    m.submit(_attempt(0, job="202610180000_0002", shared=True), None, None, None, None, None,
             "t0", 1)
    confs = [e for e in m.app.downlink.log if e[0] == "conf"]
    assert confs == [("conf", "attempt_202610180000_0002_m_000000_0")]


def test_maps_in_flight_never_exceed_the_depth():
    m = _bare(2, _attempt(0))
    peak = [0]
    real_append = m.fifo.append

    class Q(collections.deque):
        def append(self, x):
            super().append(x)
            peak[0] = max(peak[0], len(self))

    m.fifo = Q()
    del real_append
    threads = [threading.Thread(target=m.submit,
                                args=(_attempt(i), None, None, None, None, None, i, 1))
               for i in range(6)]
    for t in threads:
        t.start()
    # a consumer completes maps (the uplink's DONE) one at a time
    done = 0
    end = time.time() + 10
    while done < 6 and time.time() < end:
        with m.cond:
            if m.fifo:
                m.fifo.popleft()
                done += 1
                m.cond.notify_all()
        time.sleep(0.002)
    for t in threads:
        t.join(5)
    assert done == 6 and peak[0] <= 2


def test_a_child_dying_after_the_handler_swap_fails_the_new_handler():
    """The uplink reader reports EOF to the handler installed when the child
    dies, not the one it held while blocked in its read: the mux swaps in its
    FIFO dispatcher after the child started, and a child that then died
    (e.g. a bad input file) left every queued map waiting forever."""
    import socket

    from hbmr.pipes.protocol import UplinkReader

    class _H:
        def __init__(self):
            self.err = None
            self.ev = threading.Event()

        def failed(self, e):
            self.err = e
            self.ev.set()

    a, b = socket.socketpair()
    first, second = _H(), _H()
    r = UplinkReader(a, first)
    r.start()
    time.sleep(0.05)                 # the reader is blocked in its first read
    r.handler = second
    b.close()                        # the child exits
    assert second.ev.wait(5)
    assert isinstance(second.err, IOError) and first.err is None
    r.join(5)
    a.close()


def test_a_large_output_value_is_serialised_in_its_own_buffer():
    """The uplink reads a large OUTPUT value (a K-Means partials block) in
    place, with room in front; the map output buffer writes the Writable's
    prefix there (serialize_in_place) instead of copying the value, and the
    bytes equal the copying serialisation for BytesWritable and Text."""
    import socket

    from hbmr.io.vint import encode_vint
    from hbmr.io.writable import BytesWritable, Text, payload_serializer, serialize_in_place
    from hbmr.pipes.protocol import OUTPUT, UplinkReader

    got = []

    class _H:
        def output(self, k, v):
            got.append((k, v))

        def failed(self, e):
            got.append(("failed", e))

    a, b = socket.socketpair()
    big = bytes(range(256)) * 600                  # 153,600 bytes
    msg = encode_vint(OUTPUT) + encode_vint(1) + b"*" + encode_vint(len(big)) + big
    msg += encode_vint(OUTPUT) + encode_vint(1) + b"s" + encode_vint(3) + b"abc"
    r = UplinkReader(a, _H())
    r.start()
    b.sendall(msg)
    b.close()
    r.join(5)
    (k1, v1), (k2, v2) = got[0], got[1]
    assert k1 == b"*" and v1.__class__ is memoryview and bytes(v1) == big
    assert v2 == b"abc"
    for cls in (BytesWritable, Text):
        ser = payload_serializer(cls)
        want = ser(big)
        bb = bytearray(8 + len(big))
        bb[8:] = big
        assert bytes(serialize_in_place(ser, memoryview(bb)[8:])) == want
        assert serialize_in_place(ser, b"xyz") == ser(b"xyz")
    a.close()
