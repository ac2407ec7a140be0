"""TorchComm's variable all-to-alls exchange their row counts
as host tensors over the host (gloo) group — never a device tensor read back
on the host (which would wait for the device stream).  A recording fake of
torch.distributed stands in for RCCL + gloo; device tensors are ``meta``
tensors (no GPU here): the path taken depends only on the device type."""
import collections

import torch

from hbmr.parallel.collectives import TorchComm


class FakeDist:
    def __init__(self, rank, world, peers_counts):
        self.rank, self.world = rank, world
        self.peers = peers_counts          # peers[j] = the counts rank j sends
        self.calls = []

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None,
                          group=None):
        self.calls.append(("a2a_single", out.device.type, inp.device.type, group,
                           output_split_sizes))
        if inp.dtype == torch.int64 and inp.dim() == 1 and out.device.type == "cpu":
            out.copy_(torch.tensor([self.peers[j][self.rank] for j in range(self.world)]))

    def all_to_all(self, ins, outs, group=None):
        self.calls.append(("a2a", ins[0].device.type, group, [t.shape[0] for t in ins]))


def _comm(dist, cpu_group="host-grp", stage=False):
    c = TorchComm.__new__(TorchComm)
    c.dist, c.group, c.cpu_group = dist, "rccl-grp", cpu_group
    c.rank, c.world_size, c.stage = dist.rank, dist.world, stage
    c.backend = "gloo" if stage else "nccl"
    c.stats = collections.Counter()
    return c


def test_all_to_all_v_sizes_go_over_the_host_group():
    peers = [[3, 5, 0], [1, 1, 1], [7, 0, 2]]
    d = FakeDist(rank=1, world=3, peers_counts=peers)
    c = _comm(d)
    send = torch.empty(sum(peers[1]), 4, device="meta")
    recv, rc = c.all_to_all_v(send, peers[1])
    assert rc == [5, 1, 0] and recv.shape == (6, 4) and recv.device.type == "meta"
    sizes, data = d.calls
    # the counts: host tensors on the host group; the data: device, RCCL group,
    # split sizes from the host exchange
    assert sizes[1:4] == ("cpu", "cpu", "host-grp")
    assert data[1:5] == ("meta", "meta", "rccl-grp", [5, 1, 0])
    assert c.stats.get("ALL_TO_ALL_V_HOST_READS", 0) == 0


def test_all_to_all_list_sizes_go_over_the_host_group():
    peers = [[2, 4], [6, 1]]
    d = FakeDist(rank=0, world=2, peers_counts=peers)
    c = _comm(d)
    outs = [torch.empty(2, 3, device="meta"), torch.empty(4, 3, device="meta")]
    ins = c.all_to_all(outs)
    assert [t.shape[0] for t in ins] == [2, 6]
    assert d.calls[0][1:4] == ("cpu", "cpu", "host-grp")
    assert d.calls[1] == ("a2a", "meta", "rccl-grp", [2, 6])
    assert c.stats.get("ALL_TO_ALL_HOST_READS", 0) == 0


def test_without_a_host_group_the_device_exchange_is_counted():
    d = FakeDist(rank=0, world=2, peers_counts=[[1, 1], [1, 1]])
    c = _comm(d, cpu_group=None)
    send = torch.empty(2, 4, device="meta")
    try:
        c.all_to_all_v(send, [1, 1])
    except (NotImplementedError, RuntimeError):
        pass                   # meta tensors cannot be read back: the path is what matters
    assert d.calls[0][1:4] == ("meta", "meta", "rccl-grp")
    assert c.stats["ALL_TO_ALL_V_HOST_READS"] == 1
