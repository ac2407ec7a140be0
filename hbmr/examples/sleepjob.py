"""SleepJob: a job whose tasks only sleep — measures framework overhead.

Two forms:

* :func:`sleep_job_conf` — the classic record-level job of the reference
  (src/examples/org/apache/hadoop/examples/SleepJob.java): ``m`` maps over empty
  splits, each reading ``sleep.job.map.sleep.count`` synthetic records, sleeping
  ``sleep.job.map.sleep.time`` ms per record and emitting IntWritable keys so
  every one of the ``r`` reduces receives ``sleep.job.reduce.sleep.count`` keys,
  on each of which it sleeps ``sleep.job.reduce.sleep.time`` ms.
* :class:`SplitSleepJob` — the split-level form: each map task sleeps
  ``hbmr.sleep.map.ms`` on its slot (on a GPU slot it occupies the HIP stream
  with a device-side spin so stream ordering and overlap are exercised) and
  the collective reduce sums the task counts.  With 0 ms it measures the pure
  control-plane cost per task / per job (tools/profile_control_plane.py).
"""
from __future__ import annotations

import argparse
import time

from ..gpu.splitjob import SplitJob, SplitSpec
from ..io.writable import IntWritable, NullWritable
from ..mapred.api import InputFormat, InputSplit, Mapper, Partitioner, RecordReader, Reducer
from ..mapred.formats import NullOutputFormat
from ..mapred.jobconf import JobConf


# --------------------------------------------------------------------------- classic
class EmptySplit(InputSplit):
    def serialize(self) -> bytes:
        return b""

    @classmethod
    def deserialize(cls, raw: bytes):
        return cls()


class SleepInputFormat(InputFormat):
    def getSplits(self, job, num_splits):  # noqa: N802
        return [EmptySplit() for _ in range(max(1, num_splits))]

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        count = job.get_int("sleep.job.map.sleep.count", 1)
        redcount = job.get_int("sleep.job.reduce.sleep.count", 1)
        if count < 0 or redcount < 0:
            raise ValueError("invalid sleep counts")
        return _SleepReader(count, redcount * job.get_num_reduce_tasks())


class _SleepReader(RecordReader):
    """count records; record i = (first key, how many keys to emit) so that the
    map's total emission is spread evenly over its records."""

    def __init__(self, count, emit_total):
        self.count, self.emit_total = count, emit_total
        self.records = 0
        self.next_key = 0

    def next(self):
        if self.records >= self.count:
            return None
        emit = self.emit_total // self.count + (1 if self.emit_total % self.count > self.records
                                               else 0)
        kv = (IntWritable(self.next_key), IntWritable(emit))
        self.next_key += emit
        self.records += 1
        return kv

    def getProgress(self):  # noqa: N802
        return self.records / max(1, self.count)


class SleepMapper(Mapper):
    def configure(self, job):
        self.ms = job.get_int("sleep.job.map.sleep.time", 100)

    def map(self, key, value, output, reporter):
        reporter.setStatus(f"Sleeping... {self.ms} ms")
        time.sleep(self.ms / 1000.0)
        k = key.get()
        for i in range(value.get()):
            output.collect(IntWritable(k + i), NullWritable.get())


class SleepReducer(Reducer):
    def configure(self, job):
        self.ms = job.get_int("sleep.job.reduce.sleep.time", 100)

    def reduce(self, key, values, output, reporter):
        for _ in values:
            pass
        reporter.setStatus(f"Sleeping... {self.ms} ms")
        time.sleep(self.ms / 1000.0)


class SleepPartitioner(Partitioner):
    def getPartition(self, key, value, num_partitions):  # noqa: N802
        return key.get() % num_partitions


def sleep_job_conf(maps=1, reduces=1, map_ms=100, reduce_ms=100, map_count=1, reduce_count=1,
                   base=None) -> JobConf:
    job = JobConf(base)
    job.set_job_name("Sleep job")
    job.set_num_map_tasks(maps)
    job.set_num_reduce_tasks(reduces)
    job.set_int("sleep.job.map.sleep.time", map_ms)
    job.set_int("sleep.job.reduce.sleep.time", reduce_ms)
    job.set_int("sleep.job.map.sleep.count", map_count)
    job.set_int("sleep.job.reduce.sleep.count", reduce_count)
    job.set_input_format(SleepInputFormat)
    job.set_output_format(NullOutputFormat)
    job.set_mapper_class(SleepMapper)
    job.set_reducer_class(SleepReducer)
    job.set_partitioner_class(SleepPartitioner)
    job.set("mapred.mapoutput.key.class", "hbmr.io.writable:IntWritable")
    job.set("mapred.mapoutput.value.class", "hbmr.io.writable:NullWritable")
    job.set_speculative_execution(False)
    return job


# --------------------------------------------------------------------------- split-level
class SplitSleepJob(SplitJob):
    collective_reduce = True
    needs_reduce = True

    def configure(self, conf):
        super().configure(conf)
        self.maps = conf.get_int("hbmr.sleep.maps", 1)
        self.map_ms = conf.get_float("hbmr.sleep.map.ms", 0.0)
        self.reduce_ms = conf.get_float("hbmr.sleep.reduce.ms", 0.0)

    def get_splits(self, conf, trackers):
        out = []
        for i in range(self.maps):
            loc = [trackers[i * len(trackers) // self.maps]] if trackers else []
            out.append(SplitSpec(i, f"sleep:{i}", "range", {"i": i}, loc, 0))
        return out

    def load_split(self, spec, device):
        return spec.params["i"]

    def split_nbytes(self, data):
        return 0

    def load_split_sample(self, spec, device, fraction):
        return ("sample", fraction)

    def map_cpu(self, ctx, data):
        frac = data[1] if isinstance(data, tuple) else 1.0   # a sampled probe sleeps pro rata
        if self.map_ms > 0:
            # sleep in slices so a killed attempt (preemption) frees its slot
            kill = getattr(ctx, "kill_event", None)
            end = time.time() + self.map_ms * frac / 1000.0
            while True:
                left = end - time.time()
                if left <= 0:
                    break
                if kill is not None and kill.is_set():
                    raise RuntimeError("killed")
                time.sleep(min(left, 0.01))
        return 1

    def map_gpu(self, ctx, data):
        if self.map_ms > 0:
            import torch
            # ~2.1 GHz shader clock: occupy the slot's stream, not the host
            torch.cuda._sleep(int(self.map_ms * 2.1e6))
        return 1

    def map_sim(self, ctx, data):
        # simulated GPU slot: the runtime charges hbmr.gpu.simulate.task.ms
        return 1

    def map_gpu_batch(self, ctxs, datas):
        return [self.map_gpu(c, d) for c, d in zip(ctxs, datas)]

    def combine(self, ctx, outputs):
        return sum(outputs)

    def reduce(self, ctx, combined):
        import torch
        if self.reduce_ms > 0:
            time.sleep(self.reduce_ms / 1000.0)
        t = torch.tensor([combined], dtype=torch.int64)
        if ctx.device is not None and ctx.device.type == "cuda":
            t = t.to(ctx.device)
        ctx.comm.all_reduce(t)
        return {"maps": int(t.item())}


def split_sleep_conf(maps=128, map_ms=0.0, reduce_ms=0.0, base=None, cpu_capable=True) -> JobConf:
    job = JobConf(base)
    job.set_job_name(f"split sleep x{maps}")
    job.set("hbmr.splitjob.class", "hbmr.examples.sleepjob:SplitSleepJob")
    job.set_int("hbmr.sleep.maps", maps)
    job.set_float("hbmr.sleep.map.ms", map_ms)
    job.set_float("hbmr.sleep.reduce.ms", reduce_ms)
    job.set_boolean("hbmr.job.cpu.capable", cpu_capable)
    return job


def main(argv=None, cluster=None):
    from ..mapred.jobclient import JobClient
    ap = argparse.ArgumentParser(prog="hbmr sleep")
    ap.add_argument("-m", type=int, default=1)
    ap.add_argument("-r", type=int, default=1)
    ap.add_argument("-mt", type=int, default=100)
    ap.add_argument("-rt", type=int, default=100)
    ap.add_argument("-recordt", type=int, default=None)
    a = ap.parse_args(argv)
    job = sleep_job_conf(a.m, a.r, a.mt, a.rt)
    if a.recordt is not None:
        job.set_int("sleep.job.map.sleep.time", a.recordt)
        job.set_int("sleep.job.reduce.sleep.time", a.recordt)
    rj = JobClient.runJob(job, cluster=cluster)
    return 0 if rj.isSuccessful() else 1

