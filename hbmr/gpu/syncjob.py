"""A map-less collective job that synchronises every tracker (and its device).

Used to bracket timed regions across processes (benchmarks) and as a cheap
liveness check of the whole gang: its single pinned reduce per tracker does a
communicator barrier followed by a device synchronize.
"""
from __future__ import annotations

import time

from .splitjob import SplitJob


class SyncSplitJob(SplitJob):
    collective_reduce = True
    needs_reduce = True

    def get_splits(self, conf, trackers):
        return []

    def combine(self, ctx, outputs):
        return None

    def reduce(self, ctx, combined):
        import torch
        if torch.cuda.is_available() and ctx.device is not None:
            torch.cuda.synchronize(ctx.device)
        ctx.comm.barrier()
        if torch.cuda.is_available() and ctx.device is not None:
            torch.cuda.synchronize(ctx.device)
        return {"t": time.time(), "rank": ctx.rank}


def sync_conf(base=None):
    from ..mapred.jobconf import JobConf
    job = JobConf(base)
    job.set_job_name("sync")
    job.set("hbmr.splitjob.class", "hbmr.gpu.syncjob:SyncSplitJob")
    job.set_boolean("hbmr.job.cpu.capable", False)
    return job
