"""Batch.for_reduce (hbmr/mapred/sortbuf.py): a reduce partition of few large
records keeps its values as views into the map output segments; its sort
order, groups and values equal the joined-buffer Batch's."""
import numpy as np

from hbmr.mapred import sortbuf
from hbmr.io.writable import BytesWritable, Text


def _body(recs):
    b = sortbuf.Batch.from_lists([k for k, _ in recs], [v for _, v in recs])
    perm = np.arange(b.n, dtype=np.int64)
    return b.ifile_body(perm, 0, b.n)


def test_view_batch_equals_joined_batch_for_large_values():
    rng = np.random.default_rng(1)
    kb = b"\x01*"
    bodies = []
    for m in range(12):
        recs = [(kb, rng.integers(0, 255, (1 << 20) + m, dtype=np.uint8).tobytes())]
        if m % 3 == 0:
            recs.append((b"\x01a", rng.integers(0, 255, 70000, dtype=np.uint8).tobytes()))
        bodies.append(_body(recs))
    kind = sortbuf.TEXT
    a = sortbuf.Batch.from_ifile_bodies(bodies)
    v = sortbuf.Batch.for_reduce(bodies)
    assert type(v) is not sortbuf.Batch and v.n == a.n
    pa = a.sort(kind, np.zeros(a.n, np.int32))
    pv = v.sort(kind, np.zeros(v.n, np.int32))
    assert pa.tolist() == pv.tolist()
    assert a.group_ends(kind, pa, 0, a.n).tolist() == v.group_ends(kind, pv, 0, v.n).tolist()
    for r in range(a.n):
        assert a.key(r) == v.key(r)
        assert bytes(a.value_view(r)) == bytes(v.value_view(r)) == v.value(r)


def test_small_records_keep_the_joined_batch():
    bodies = [_body([(b"\x01k%d" % i, b"v" * 100) for i in range(50)]) for _ in range(4)]
    assert type(sortbuf.Batch.for_reduce(bodies)) is sortbuf.Batch
    _ = BytesWritable
