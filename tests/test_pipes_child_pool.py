"""ChildPool (hbmr/pipes/application.py): an idle reusable Pipes child that
already mapped a split is handed that split again (a GPU binary keeps it in
HBM); otherwise the most recently idle child."""
from hbmr.pipes.application import ChildPool


class _App:
    def __init__(self, name):
        self.name = name

    def alive(self):
        return True

    def cleanup(self):
        pass

    def close_child(self):
        pass


def test_pool_prefers_the_child_holding_the_split():
    pool = ChildPool(idle_s=60)
    a, b = _App("a"), _App("b")
    pool.release("k", a, split=b"s0")
    pool.release("k", b, split=b"s1")
    assert pool.acquire("k", b"s0") is a          # not the most recent (b)
    pool.release("k", a, split=b"s2")
    assert pool.acquire("k", b"s1") is b
    assert pool.acquire("k", b"s9") is a          # nobody holds it: most recent idle
    assert pool.acquire("k", b"s0") is None
    assert a.splits_seen == {b"s0", b"s2"}
