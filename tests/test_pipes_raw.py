"""The Pipes byte paths that skip Writable objects: a map's OUTPUT frames go
into the map output buffer as serialised records (MapOutputBuffer.raw_sink),
and a reduce's key groups go down the pipe as ready-made frames
(PipesReducer.raw_reduce / DownwardProtocol.reduce_group).  Each must produce
exactly the bytes of the object path it replaces (OutputHandler.output ->
collect; reduce_key + reduce_value, BinaryProtocol.java:349-369)."""
import io
import os
import types

import pytest

from hbmr.io.vint import encode_vint
from hbmr.io.writable import BytesWritable, IntWritable, Text, payload_serializer
from hbmr.mapred import JobConf
from hbmr.mapred.task import MapOutputBuffer
from hbmr.pipes.application import OutputHandler
from hbmr.pipes.protocol import DownwardProtocol, frame_of_serialized, to_wire
from hbmr.pipes.runner import PipesPartitioner


class _Sock:
    def __init__(self):
        self.buf = _Buf()

    def makefile(self, mode, buffering=None):
        return self.buf


class _Buf(io.BytesIO):
    def close(self):
        pass


@pytest.mark.parametrize("obj", [Text("k1"), Text("x" * 300), Text(""), BytesWritable(b"\x00\x01"),
                                 BytesWritable(b"y" * 200), IntWritable(-7)])
def test_frame_of_serialized_equals_object_frame(obj):
    f = frame_of_serialized(type(obj))
    w = to_wire(obj)
    assert f(obj.serialize()) == encode_vint(len(w)) + w


def test_payload_serializer_round_trips():
    for cls, raw in [(Text, b"abc"), (Text, b"z" * 500), (BytesWritable, b"\x00" * 9)]:
        assert cls.deserialize(payload_serializer(cls)(raw)).bytes == raw
    assert payload_serializer(IntWritable) is None


def test_reduce_group_matches_key_and_value_messages():
    vals = [Text(f"v{i}" * (i * 40)) for i in range(5)]
    a, b = _Sock(), _Sock()
    da, db = DownwardProtocol(a), DownwardProtocol(b)
    da.reduce_key(Text("key"))
    for v in vals:
        da.reduce_value(v)
    da.flush()
    f = frame_of_serialized(Text)
    db.reduce_group(f(Text("key").serialize()), [f(v.serialize()) for v in vals])
    db.reduce_group(f(Text("empty").serialize()), [])
    db.flush()
    da.reduce_key(Text("empty"))
    da.flush()
    assert a.buf.getvalue() == b.buf.getvalue()


def _buffer(tmp_path, name, R):
    job = JobConf()
    job.set_num_reduce_tasks(R)
    job.set_map_output_key_class(Text)
    job.set_map_output_value_class(Text)
    job.set_partitioner_class(PipesPartitioner)
    task = types.SimpleNamespace(check_killed=lambda: None, attempt_id="attempt_x_m_000000_0")
    from hbmr.mapred.task import TaskReporter
    return MapOutputBuffer(task, job, TaskReporter(), str(tmp_path / name))


@pytest.mark.parametrize("R", [1, 3])
def test_raw_sink_writes_the_object_paths_map_output(tmp_path, R):
    recs = [(f"key{i % 17}".encode(), (f"val{i}" * (i % 50)).encode()) for i in range(400)]
    outs = []
    for name, raw in (("obj", False), ("raw", True)):
        buf = _buffer(tmp_path, name, R)
        h = OutputHandler(buf, None, Text, Text, PipesPartitioner())
        assert h.sink is not None
        if not raw:
            h.sink = None           # the object path: from_wire + collect
        for i, (k, v) in enumerate(recs):
            if i % 3 == 0 and R > 1:
                h.partitioned_output(i % R, k, v)
            else:
                h.output(k, v)
        assert h.records == len(recs)
        path = buf.flush()
        outs.append((open(path, "rb").read(), open(path + ".index", "rb").read(), buf.n_out,
                     buf.bytes_out))
    assert outs[0] == outs[1]
    assert outs[1][2] == len(recs)
    assert os.path.exists(path)
