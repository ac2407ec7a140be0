"""Collective communication for the MapReduce data plane.

The reference moves map output over an HTTP shuffle (TaskTracker
MapOutputServlet, TaskTracker.java:4050-4180; ReduceTask copier threads,
ReduceTask.java:1231-1922) and ships side data through the DistributedCache.
On one 8×MI355X node those become collectives over xGMI:

* shuffle of partitioned map output      -> all-to-all(v)
* combine-then-reduce of small partials  -> all-reduce (or reduce-scatter)
* DistributedCache side data (centroids) -> broadcast / all-gather

:class:`TorchComm` drives ``torch.distributed`` (backend ``nccl`` = RCCL for
device tensors, ``gloo`` for CPU tensors, one process per GPU).
:class:`InProcessComm` lets several TaskTrackers living in one process (the
mini-cluster used by tests, like the reference's MiniMRCluster) run the same
collective code paths.  :class:`SoloComm` is the 1-tracker no-op.
"""
from __future__ import annotations

import collections
import threading

import torch

COLLECTIVE_GROUP = "hbmr.CollectiveCounters"


class Comm:
    rank = 0
    world_size = 1
    stats: collections.Counter = None

    def _note(self, op: str, t: torch.Tensor):
        """Count a collective by op and tensor device (reported per reduce task
        as ``hbmr.CollectiveCounters``: which path the data plane really took)."""
        if self.stats is None:
            self.stats = collections.Counter()
        self.stats[f"{op.upper()}_{t.device.type.upper()}"] += 1

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def all_gather(self, t: torch.Tensor) -> list:
        raise NotImplementedError

    def all_to_all(self, outs: list) -> list:
        """outs[j] goes to rank j; returns ins[j] received from rank j."""
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def barrier(self):
        raise NotImplementedError

    def all_to_all_v(self, send: torch.Tensor, counts: list):
        """Variable all-to-all of one buffer: rows [sum(counts[:j]), +counts[j]) of
        ``send`` go to rank j.  Returns (recv, recv_counts), recv ordered by source."""
        self._note("all_to_all_v", send)
        outs = list(torch.split(send, [int(c) for c in counts]))
        ins = self.all_to_all(outs)
        return (torch.cat(ins) if ins else send[:0]), [int(t.shape[0]) for t in ins]

    def all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        """Element-wise maximum over ranks of a small tensor (host tensors go
        over the host group: a shape agreement that never waits for a device)."""
        if self.world_size <= 1:
            return t
        return torch.stack([x.to(t.device) for x in self.all_gather(t)]).amax(0)

    def all_to_all_v_static(self, send: torch.Tensor, counts: list, cap: int):
        """Variable all-to-all with static shapes: rows [sum(counts[:j]),
        +counts[j]) of ``send`` go to rank j through a slot of ``cap`` rows
        (the same ``cap`` on every rank).  Returns (recv, rcounts): the W
        received slots ``[W * cap, ...]`` ordered by source and their valid
        row counts as a DEVICE tensor — no size exchange is read on the host,
        so nothing here waits for the device (TorchComm.all_to_all_v reads
        the incoming sizes before it can allocate).  A count above ``cap`` is
        truncated in the slot and shows as rcounts > cap: the caller checks
        when it next reads host data (:func:`compact_static`) and re-runs the
        exchange with all_to_all_v."""
        self._note("all_to_all_v_static", send)
        W = self.world_size
        cap = max(1, int(cap))
        rest = tuple(send.shape[1:])
        slots = send.new_zeros((W * cap,) + rest)
        off = 0
        for j, c in enumerate(counts):
            c = int(c)
            n = min(c, cap)
            if n:
                slots[j * cap:j * cap + n] = send[off:off + n]
            off += c
        ct = torch.tensor([int(c) for c in counts], dtype=torch.int64)
        if send.device.type != "cpu":
            ct = ct.pin_memory().to(send.device, non_blocking=True)
        recv = self.all_to_all_fixed(slots)
        rc = self.all_to_all_fixed(ct)
        return recv, rc

    def all_to_all_fixed(self, send: torch.Tensor) -> torch.Tensor:
        """Static-shape all-to-all: ``send`` is W equal slots along dim 0, slot j
        goes to rank j; returns the W slots received, ordered by source.  No
        sizes are exchanged first, so nothing waits on the host: the caller
        sends the valid counts as another fixed-shape tensor and reads them on
        the device (TeraSort's shuffle waves)."""
        self._note("all_to_all_fixed", send)
        ins = self.all_to_all(list(torch.chunk(send, self.world_size)))
        return torch.cat(ins)

    def reduce_scatter(self, t: torch.Tensor) -> torch.Tensor:
        """Sum over ranks, rank r keeps rows [r*n/W, (r+1)*n/W) (dim 0 padded by caller)."""
        full = self.all_reduce(t)
        n = full.shape[0]
        per = (n + self.world_size - 1) // self.world_size
        return full[self.rank * per:min(n, (self.rank + 1) * per)]


class SoloComm(Comm):
    def all_reduce(self, t):
        return t

    def all_gather(self, t):
        return [t]

    def all_to_all(self, outs):
        return list(outs)

    def broadcast(self, t, src=0):
        return t

    def barrier(self):
        pass


class _Rendezvous:
    def __init__(self, n):
        self.n = n
        self.barrier_obj = threading.Barrier(n)
        self.slots = [None] * n
        self.lock = threading.Lock()


class InProcessComm(Comm):
    """Collectives among ``world_size`` threads of one process."""

    def __init__(self, rv: _Rendezvous, rank: int):
        self.rv = rv
        self.rank = rank
        self.world_size = rv.n

    @classmethod
    def group(cls, n):
        rv = _Rendezvous(n)
        return [cls(rv, r) for r in range(n)]

    @staticmethod
    def _sync(obj):
        """Device tensors: the posting (or copying) stream has finished with
        them — every rank's stream is its own, and the peers read on theirs."""
        t = obj[0] if isinstance(obj, (list, tuple)) else obj
        if torch.is_tensor(t) and t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()

    def _exchange(self, obj, take=None):
        """Post ``obj``, read every rank's; ``take`` (optional) copies what this
        rank needs out of the posted objects while the peers still hold them
        (their streams may reuse the memory once the exchange returns)."""
        rv = self.rv
        self._sync(obj)
        rv.slots[self.rank] = obj
        rv.barrier_obj.wait()
        got = list(rv.slots)
        if take is not None:
            got = take(got)
            self._sync(got)
        rv.barrier_obj.wait()
        return got

    def all_reduce(self, t):
        self._note("all_reduce", t)
        # exchange snapshots: peers may still be reading while we write into t
        def take(got):
            out = got[0].to(t.device).clone()
            for g in got[1:]:
                out += g.to(t.device)
            return [out]
        t.copy_(self._exchange(t.detach().clone(), take)[0])
        return t

    def all_gather(self, t):
        self._note("all_gather", t)
        return self._exchange(t, lambda got: [g.to(t.device, copy=True) for g in got])

    def all_to_all(self, outs):
        self._note("all_to_all", outs[0])
        me = self.rank
        return self._exchange(list(outs),
                              lambda got: [got[j][me].clone() for j in range(self.world_size)])

    def broadcast(self, t, src=0):
        self._note("broadcast", t)
        got = self._exchange(t.detach().clone(), lambda got: [got[src].to(t.device, copy=True)])
        t.copy_(got[0])
        return t

    def barrier(self):
        self.rv.barrier_obj.wait()


class TorchComm(Comm):
    """torch.distributed collectives (nccl/RCCL for device tensors, gloo for host).

    Device tensors on a ``gloo`` group (the 1-GPU rehearsal of the multi-rank
    path, ``HBMR_SHARED_DEVICE``: RCCL refuses two ranks on one GPU) are staged
    through host memory — one D2H, the gloo collective, one H2D — so the same
    device-tensor code runs unchanged; counted as ``<OP>_STAGED``.  Under RCCL
    they go device to device."""

    def __init__(self, group=None, cpu_group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.cpu_group = cpu_group
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        self.backend = str(dist.get_backend(group))
        self.stage = self.backend == "gloo"

    def _grp(self, t):
        if t.device.type == "cpu" and self.cpu_group is not None:
            return self.cpu_group
        return self.group

    def _staged(self, op, t):
        """True when device tensor ``t`` must go through host memory."""
        self._note(op, t)
        if self.stage and t.device.type != "cpu":
            self.stats[f"{op.upper()}_STAGED"] += 1
            return True
        return False

    def all_reduce(self, t):
        if self._staged("all_reduce", t):
            h = t.cpu()
            self.dist.all_reduce(h, group=self.cpu_group or self.group)
            t.copy_(h)
            return t
        self.dist.all_reduce(t, group=self._grp(t))
        return t

    def all_gather(self, t):
        if self._staged("all_gather", t):
            h = t.contiguous().cpu()
            out = [torch.empty_like(h) for _ in range(self.world_size)]
            self.dist.all_gather(out, h, group=self.cpu_group or self.group)
            return [o.to(t.device) for o in out]
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        self.dist.all_gather(out, t.contiguous(), group=self._grp(t))
        return out

    def all_to_all(self, outs):
        dev = outs[0].device
        if self._staged("all_to_all", outs[0]):
            return [x.to(dev) for x in self._all_to_all_host([o.cpu() for o in outs])]
        # sizes first (tensors may differ in length along dim 0); they are
        # known on the host, so they travel over the host group
        in_sizes = self._exchange_sizes([int(o.shape[0]) for o in outs], dev, "ALL_TO_ALL")
        ins = [torch.empty((n,) + tuple(outs[0].shape[1:]), dtype=outs[0].dtype, device=dev)
               for n in in_sizes]
        self.dist.all_to_all(ins, [o.contiguous() for o in outs], group=self._grp(outs[0]))
        return ins

    def _exchange_sizes(self, sizes, dev, op, group=None):
        """Per-destination row counts → per-source row counts.  The counts are
        host integers, so they go over the host (gloo) group as a host tensor:
        nothing waits for the device, and the data all-to-all is enqueued on
        the device stream behind the kernels that produced it.  Only a comm
        with no host group (an RCCL group alone) exchanges them on the device
        and reads the result back — counted as ``<OP>_HOST_READS``."""
        if self.cpu_group is not None or self.stage or dev.type == "cpu":
            hg = self.cpu_group if self.cpu_group is not None else \
                (self.group if self.stage else group)
            sc = torch.tensor(sizes, dtype=torch.int64)
            rc = torch.empty_like(sc)
            self.dist.all_to_all_single(rc, sc, group=hg)
            return [int(x) for x in rc.tolist()]
        sc = torch.tensor(sizes, dtype=torch.int64, device=dev)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc, group=group if group is not None else self.group)
        if self.stats is not None:
            self.stats[f"{op}_HOST_READS"] += 1
        return [int(x) for x in rc.tolist()]

    def _all_to_all_host(self, outs):
        send, counts = torch.cat(outs), [int(o.shape[0]) for o in outs]
        recv, rcounts = self._a2av(send, counts, self.cpu_group or self.group)
        return list(torch.split(recv, rcounts))

    def broadcast(self, t, src=0):
        if self._staged("broadcast", t):
            h = t.cpu()
            self.dist.broadcast(h, src, group=self.cpu_group or self.group)
            t.copy_(h)
            return t
        self.dist.broadcast(t, src, group=self._grp(t))
        return t

    def _a2av(self, send, counts, group):
        # one all_to_all_single with split sizes: a single RCCL alltoallv (grouped
        # point-to-point over the xGMI mesh) instead of per-peer tensors
        dev = send.device
        rcounts = self._exchange_sizes([int(c) for c in counts], dev, "ALL_TO_ALL_V", group)
        recv = torch.empty((sum(rcounts),) + tuple(send.shape[1:]), dtype=send.dtype, device=dev)
        self.dist.all_to_all_single(recv, send.contiguous(), output_split_sizes=rcounts,
                                    input_split_sizes=[int(c) for c in counts], group=group)
        return recv, rcounts

    def all_to_all_fixed(self, send):
        if send.shape[0] % self.world_size:
            raise ValueError("all_to_all_fixed: dim 0 must be W equal slots")
        if self._staged("all_to_all_fixed", send):
            h = send.contiguous().cpu()
            out = torch.empty_like(h)
            self.dist.all_to_all_single(out, h, group=self.cpu_group or self.group)
            return out.to(send.device)
        out = torch.empty_like(send)
        # one RCCL alltoall of equal slots: enqueued on the current stream
        # behind the kernels that filled ``send``, no host round trip
        self.dist.all_to_all_single(out, send.contiguous(), group=self._grp(send))
        return out

    def all_to_all_v(self, send, counts):
        if self._staged("all_to_all_v", send):
            recv, rcounts = self._a2av(send.cpu(), counts, self.cpu_group or self.group)
            return recv.to(send.device), rcounts
        return self._a2av(send, counts, self._grp(send))

    def barrier(self):
        self.dist.barrier(group=self.cpu_group or self.group)

    def reduce_scatter(self, t):
        if self.stage:
            # gloo has no reduce_scatter_tensor: all-reduce and keep this rank's rows
            return Comm.reduce_scatter(self, t)
        self._note("reduce_scatter", t)
        n = t.shape[0]
        per = (n + self.world_size - 1) // self.world_size
        if per * self.world_size != n:
            pad = torch.zeros((per * self.world_size - n,) + tuple(t.shape[1:]), dtype=t.dtype,
                              device=t.device)
            t = torch.cat([t, pad])
        out = torch.empty((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        self.dist.reduce_scatter_tensor(out, t.contiguous(), group=self._grp(t))
        lo = self.rank * per
        return out[:max(0, min(per, n - lo))]


def compact_static(recv: torch.Tensor, rcounts: torch.Tensor, cap: int):
    """The valid rows of all_to_all_v_static's slots, back to back by source,
    and their counts (a host list) — the one host read of the exchange.
    Returns None when a slot overflowed (a count above ``cap``): re-run the
    exchange with all_to_all_v."""
    rc = [int(x) for x in rcounts.tolist()]
    if any(c > cap for c in rc):
        return None
    parts = [recv[j * cap:j * cap + c] for j, c in enumerate(rc)]
    return (torch.cat(parts) if parts else recv[:0]), rc
