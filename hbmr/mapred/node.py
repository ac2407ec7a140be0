"""Multi-process node bring-up: one process per GPU, JobTracker on rank 0.

Launch with ``torchrun --nproc-per-node N`` (or ``python -m torch.distributed.run``).
Every rank runs a TaskTracker for its GPU (LOCAL_RANK) plus its CPU slots;
rank 0 additionally hosts the JobTracker and its RPC endpoint, whose address is
published in the torch.distributed store.  Collectives of the data plane use
the process group: ``nccl`` (RCCL over xGMI) for device tensors and a ``gloo``
group for host tensors.
"""
from __future__ import annotations

import datetime
import logging
import os
import socket
import time

import torch

from ..parallel.collectives import SoloComm, TorchComm
from .jobconf import JobConf
from .jobtracker import JobTracker
from ..security import rpc_secret
from .rpc import JT_METHODS, JobTrackerProxy, RpcServer
from .tasktracker import TaskTracker

log = logging.getLogger("hbmr.node")


def group_plan(use_gpu: bool, worker_mode: bool, shared: bool, backend: str | None = None):
    """(backend of the rank processes' group, backend of the device collectives).

    Device collectives run on ``nccl`` (RCCL over xGMI) unless there is no GPU
    or every rank shares one device (``HBMR_SHARED_DEVICE``, where RCCL refuses
    two ranks on one GPU and gloo stages device tensors through host memory).
    In worker mode the device work — and so the device group — lives in the
    per-rank GPU workers; the rank processes then only need host collectives
    (gloo) and never create a HIP context."""
    dev = "gloo" if (shared or not use_gpu) else (backend or "nccl")
    rank = "gloo" if (worker_mode or not use_gpu) else dev
    return rank, dev


class Node:
    def __init__(self, conf: JobConf | None = None, use_gpu: bool | None = None,
                 backend: str | None = None):
        self.conf = conf or JobConf()
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # rehearsal of the multi-process path on a 1-GPU box: every rank drives
        # device 0 and collectives go over gloo (RCCL refuses two ranks on one GPU)
        shared = os.environ.get("HBMR_SHARED_DEVICE")
        if shared is not None:
            self.local_rank = int(shared)
        simulate = self.conf.get_boolean("hbmr.gpu.simulate", False)
        # device_count() does not initialise HIP; is_available() would
        self.use_gpu = (torch.cuda.device_count() > 0) if use_gpu is None else use_gpu
        # default: device work in a per-rank GPU worker process, so this process
        # (TaskTracker, and the JobTracker on rank 0) never holds a HIP context
        self.worker_mode = self.conf.get_boolean("hbmr.gpu.worker.process",
                                                 self.use_gpu or simulate)
        if self.worker_mode:
            self.conf.set("hbmr.gpu.worker.process", "true")
        rank_be, dev_backend = group_plan(self.use_gpu, self.worker_mode, shared is not None,
                                          backend)
        self.jt = None
        self.server = None
        self.dist = None
        self.comm = SoloComm()
        worker_comm = None
        if self.use_gpu and not self.worker_mode:
            torch.cuda.set_device(self.local_rank)
        if self.world > 1:
            import torch.distributed as dist
            self.dist = dist
            self.comm = self._init_dist(rank_be)
            self.store = dist.distributed_c10d._get_default_store()
            if self.worker_mode:
                worker_comm = {"host": os.environ.get("MASTER_ADDR", "127.0.0.1"),
                               "port": int(os.environ["MASTER_PORT"]), "rank": self.rank,
                               "world": self.world, "backend": dev_backend}
        # 8+ ranks: the JobTracker runs in a process of its own (not under
        # rank 0's interpreter lock with its tracker and the driver): the
        # 16-CPU-host rehearsal measured 8.1 vs 9.0 ms per job at 8 ranks (rank
        # 0's CPU 9.8 -> 1.6 ms per job) and no gain at 2-4 ranks
        # (profiles/r04_final_b_terasort_rehearsal.json); the key overrides
        self.jt_process = self.rank == 0 and self.conf.get_boolean(
            "hbmr.jobtracker.process", self.world >= 8)
        if self.jt_process:
            from .jtprocess import RemoteJobTracker
            self.jt = RemoteJobTracker(self.conf)
            if self.world > 1:
                host = os.environ.get("MASTER_ADDR", "127.0.0.1")
                self.store.set("hbmr/jobtracker", f"{host}:{self.jt.port}")
            jt_handle = JobTrackerProxy(self.jt.address, self.conf)
        elif self.rank == 0:
            self.jt = JobTracker(self.conf)
            if self.world > 1:
                self.server = RpcServer(self.jt, JT_METHODS, secret=rpc_secret(self.conf)).start()
                host = os.environ.get("MASTER_ADDR", "127.0.0.1")
                self.store.set("hbmr/jobtracker", f"{host}:{self.server.port}")
            jt_handle = self.jt
        else:
            addr = self.store.get("hbmr/jobtracker").decode()
            jt_handle = JobTrackerProxy(addr, self.conf)
        gpus = [self.local_rank] if (self.use_gpu or simulate) else []
        self.tt = TaskTracker(self.conf, jt_handle,
                              name=f"tracker_{socket.gethostname()}_r{self.rank}", rank=self.rank,
                              world_size=self.world, gpu_devices=gpus, comm=self.comm,
                              worker_comm=worker_comm)
        # one rank with its JobTracker in this process: every reduce reads here
        self.tt.all_trackers_local = self.world == 1 and not self.jt_process
        self.tt.start()
        if self.jt is not None:
            if not self.jt.wait_for_trackers(self.world, timeout=300):
                raise RuntimeError("not all TaskTrackers registered with the JobTracker")
            self.jt.start_expiry_thread()
        # start-up state into the permanent GC generation, rarer collections
        # (hbmr/utils/gctune.py: full collections were ~60 ms GIL pauses)
        from ..utils.gctune import tune
        tune()

    def _init_dist(self, be: str):
        """The default process group on backend ``be`` (plus a gloo group for
        host tensors when ``be`` is nccl); returns the data-plane comm."""
        dist = self.dist
        kw = {}
        if be == "nccl":
            kw["device_id"] = torch.device("cuda", self.local_rank)
        dist.init_process_group(be, timeout=datetime.timedelta(seconds=600), **kw)
        cpu_group = dist.new_group(backend="gloo") if be != "gloo" else None
        return TorchComm(group=None, cpu_group=cpu_group)

    @property
    def is_master(self):
        return self.rank == 0

    def submit_job(self, job):
        return self.jt.submit_job(job)

    def job_result(self, rj, partition=0):
        r = rj._impl.result
        if r is None:
            return None
        return r.get(partition, r.get(str(partition)))

    def serve_until_shutdown(self):
        """Non-master ranks: run the tracker until the JobTracker says shutdown."""
        while not self.tt._stop.is_set():
            time.sleep(0.05)

    def shutdown(self):
        if self.jt is not None:
            self.jt.broadcast_shutdown()
            # wait for the other trackers to receive the shutdown action
            deadline = time.time() + 30
            while time.time() < deadline:
                if self.jt_process:
                    others = self.jt.live_trackers(self.tt.name, 0.5)
                else:
                    with self.jt.lock:
                        others = [t for t in self.jt.trackers.values()
                                  if t.name != self.tt.name and time.time() - t.last_seen < 0.5]
                if not others or time.time() > deadline:
                    break
                time.sleep(0.1)
        self.tt.stop()
        if self.jt is not None:
            time.sleep(0.2)
            self.jt.shutdown()
        if self.dist is not None:
            try:
                self.dist.barrier(group=self.comm.cpu_group)
            except Exception:  # noqa: BLE001
                pass
            self.dist.destroy_process_group()
        if self.server is not None:
            self.server.stop()
