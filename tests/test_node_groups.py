"""Process-group construction of the multi-rank node (node.py group_plan /
Node._init_dist, gpu/worker.py _make_comm): which backend each group gets and
that the RCCL group is bound to the rank's device.  The real RCCL run is the
driver's 8-GPU bench; here torch.distributed is replaced by a recorder."""
import pytest
import torch

from hbmr.gpu import worker as W
from hbmr.mapred import node as N
from hbmr.parallel import collectives as CO


@pytest.mark.parametrize("use_gpu,worker,shared,want", [
    (True, False, False, ("nccl", "nccl")),     # in-process device work: RCCL everywhere
    (True, True, False, ("gloo", "nccl")),      # rank processes host-only; workers on RCCL
    (True, True, True, ("gloo", "gloo")),       # 1-GPU rehearsal: gloo, staged device tensors
    (True, False, True, ("gloo", "gloo")),
    (False, False, False, ("gloo", "gloo")),
    (False, True, False, ("gloo", "gloo")),
])
def test_group_plan(use_gpu, worker, shared, want):
    assert N.group_plan(use_gpu, worker, shared) == want


class _FakeDist:
    def __init__(self, backend):
        self.calls = []
        self._backend = backend

    def init_process_group(self, backend, **kw):
        self.calls.append(("init", backend, kw))

    def new_group(self, **kw):
        self.calls.append(("new_group", kw))
        return "cpu-group"

    def get_rank(self, *a):
        return 1

    def get_world_size(self, *a):
        return 4

    def get_backend(self, group=None):
        return self._backend


def _patch(monkeypatch, fake):
    import sys
    monkeypatch.setattr(torch, "distributed", fake, raising=False)
    monkeypatch.setitem(sys.modules, "torch.distributed", fake)
    return fake


def test_node_nccl_branch_builds_device_and_host_groups(monkeypatch):
    fake = _patch(monkeypatch, _FakeDist("nccl"))
    node = N.Node.__new__(N.Node)
    node.dist, node.local_rank = fake, 3
    comm = node._init_dist("nccl")
    init = fake.calls[0]
    assert init[0] == "init" and init[1] == "nccl"
    assert init[2]["device_id"] == torch.device("cuda", 3)      # bound to this rank's GPU
    assert fake.calls[1] == ("new_group", {"backend": "gloo"})   # host tensors
    assert isinstance(comm, CO.TorchComm) and comm.cpu_group == "cpu-group"
    assert comm.group is None and not comm.stage
    assert comm._grp(torch.zeros(1)) == "cpu-group"


def test_node_gloo_branch_has_one_group(monkeypatch):
    fake = _patch(monkeypatch, _FakeDist("gloo"))
    node = N.Node.__new__(N.Node)
    node.dist, node.local_rank = fake, 0
    comm = node._init_dist("gloo")
    assert [c[0] for c in fake.calls] == ["init"] and "device_id" not in fake.calls[0][2]
    assert comm.cpu_group is None and comm.stage       # device tensors staged via host


def test_worker_comm_nccl_generation_prefix(monkeypatch):
    fake = _FakeDist("nccl")
    stores = []

    class Store:
        def __init__(self, host, port, **kw):
            stores.append(("tcp", host, port, kw["is_master"]))

    def prefix(p, st):
        stores.append(("prefix", p))
        return "prefixed"
    fake.TCPStore, fake.PrefixStore = Store, prefix
    _patch(monkeypatch, fake)
    comm = W._make_comm({"comm": {"host": "127.0.0.1", "port": 1234, "rank": 1, "world": 4,
                                  "backend": "nccl"}, "generation": 2, "devices": [5]})
    assert stores == [("tcp", "127.0.0.1", 1234, False), ("prefix", "hbmr/gpuworker/g2/")]
    init = fake.calls[0]
    assert init[1] == "nccl" and init[2]["store"] == "prefixed"
    assert init[2]["rank"] == 1 and init[2]["world_size"] == 4
    assert init[2]["device_id"] == torch.device("cuda", 5)
    assert fake.calls[1] == ("new_group", {"backend": "gloo"})
    assert isinstance(comm, CO.TorchComm)
    assert isinstance(W._make_comm({"comm": None}), CO.SoloComm)
