"""Gridmix: trace-driven synthetic workload generator / cluster load test.

Behaviour from hadoop-1.0.3/src/contrib/gridmix (Gridmix.java, GenerateData,
JobCreator LOADJOB/SLEEPJOB, LoadJob, SleepJob, JobSubmitter, JobMonitor,
Statistics, submission policies REPLAY/STRESS/SERIAL in
GridmixJobSubmissionPolicy, ReplayJobFactory, StressJobFactory,
SerialJobFactory) and src/benchmarks/gridmix2 (the fixed job mix):

* ``generate_data`` — GenerateData: a pool of random input files.
* a Rumen trace (hbmr.tools.rumen) is replayed job by job as
  - **LOADJOB**: each map reads its share of the job's recorded input bytes
    from the pool, emits its share of the recorded map-output bytes spread
    over the reduces, and each reduce writes its share of the output bytes
    (gridmix.* byte ratios from the job's counters), or
  - **SLEEPJOB**: each task sleeps its recorded runtime (× ``time_scale``) —
    GPU-placed maps of the trace are marked so the hybrid scheduler sees the
    same CPU/GPU mix;
* **REPLAY** honours the recorded inter-arrival gaps (scaled), **SERIAL**
  submits the next job when the previous finished, **STRESS** keeps
  ``max_in_flight`` jobs running.

Statistics returned per job: submit/finish wall times, runtime, success.
"""
from __future__ import annotations

import argparse
import json
import os
import threading
import time

import numpy as np

from ..io.writable import BytesWritable, IntWritable, NullWritable
from ..mapred import FileOutputFormat, JobClient, JobConf
from ..mapred.api import InputFormat, InputSplit, Mapper, Partitioner, RecordReader, Reducer
from ..mapred.formats import NullOutputFormat, SequenceFileOutputFormat
from .rumen import ZombieJobProducer

REC = 64 << 10  # synthetic record payload size


def generate_data(path, total_bytes, files=4, seed=0):
    """GenerateData: ``files`` random binary files totalling ``total_bytes``."""
    os.makedirs(path, exist_ok=True)
    rng = np.random.default_rng(seed)
    per = -(-total_bytes // files)
    out = []
    for i in range(files):
        p = os.path.join(path, f"part-{i:05d}")
        left = min(per, total_bytes - i * per)
        with open(p, "wb") as f:
            while left > 0:
                n = min(left, 8 << 20)
                f.write(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
                left -= n
        out.append(p)
    return out


class GridmixSplit(InputSplit):
    def __init__(self, index=0):
        self.index = index

    def serialize(self) -> bytes:
        return str(self.index).encode()

    @classmethod
    def deserialize(cls, raw: bytes):
        return cls(int(raw.decode() or 0))

    def getLength(self):  # noqa: N802
        return 0

    def getLocations(self):  # noqa: N802
        return []


class _OneRecord(RecordReader):
    def __init__(self, index):
        self.index, self.done = index, False

    def next(self):
        if self.done:
            return None
        self.done = True
        return IntWritable(self.index), NullWritable.get()


class GridmixInputFormat(InputFormat):
    """One split per map of the traced job; the map's spec is in the conf."""

    def getSplits(self, job, num_splits):  # noqa: N802
        return [GridmixSplit(i) for i in range(job.get_int("gridmix.maps", 1))]

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return _OneRecord(split.index)


def _specs(job, key):
    return json.loads(job.get(key, "[]"))


class LoadMapper(Mapper):
    """Reads recorded input bytes from the pool, emits recorded output bytes."""

    def configure(self, job):
        self.maps = _specs(job, "gridmix.map.specs")
        self.pool = sorted(job.get_strings("gridmix.pool") or [])
        self.reduces = job.get_num_reduce_tasks()
        self.gpu_maps = set(json.loads(job.get("gridmix.gpu.maps", "[]")))

    def map(self, key, value, output, reporter):
        spec = self.maps[key.get()]
        left = spec["in"]
        if self.pool and left > 0:
            f_i = key.get() % len(self.pool)
            while left > 0:
                with open(self.pool[f_i], "rb") as f:
                    f.seek((key.get() * 7919 * REC) % max(1, os.path.getsize(self.pool[f_i])))
                    while left > 0:
                        b = f.read(min(left, 1 << 20))
                        if not b:
                            break
                        left -= len(b)
                        reporter.progress()
                f_i = (f_i + 1) % len(self.pool)
        if spec["ms"]:
            time.sleep(spec["ms"] / 1000.0)
        out = spec["out"]
        payload = os.urandom(min(REC, max(out, 1)))
        r = 0
        while out > 0 and self.reduces:
            n = min(out, REC)
            output.collect(IntWritable(r), BytesWritable(payload[:n]))
            r = (r + 1) % self.reduces
            out -= n
        reporter.incrCounter("gridmix", "MAPS_ON_GPU_IN_TRACE", int(key.get() in self.gpu_maps))


class LoadReducer(Reducer):
    def configure(self, job):
        self.specs = _specs(job, "gridmix.reduce.specs")
        self.part = job.get_int("mapred.task.partition", 0)
        self.written = 0

    def reduce(self, key, values, output, reporter):
        spec = self.specs[self.part] if self.part < len(self.specs) else {"out": 0, "ms": 0}
        for _ in values:
            reporter.progress()
        if spec["ms"]:
            time.sleep(spec["ms"] / 1000.0)
        left = spec["out"] - self.written
        while left > 0:
            n = min(left, REC)
            output.collect(NullWritable.get(), BytesWritable(b"\0" * n))
            self.written += n
            left -= n


class GridmixPartitioner(Partitioner):
    def getPartition(self, key, value, num_partitions):  # noqa: N802
        return key.get() % num_partitions


def _even(total, n):
    return [total // n + (1 if i < total % n else 0) for i in range(n)] if n else []


def job_from_story(story, kind, pool, time_scale, out_dir, base_conf=None) -> JobConf:
    """JobCreator: a LOADJOB or SLEEPJOB JobConf reproducing one traced job."""
    lj = story.job
    maps, reds = max(1, story.getNumberMaps()), story.getNumberReduces()
    cs = lj.get("counters", {})

    def counter(name):
        for grp in cs.values():
            if isinstance(grp, dict) and name in grp:
                return int(grp[name])
        return 0

    in_b = counter("HDFS_BYTES_READ") or counter("FILE_BYTES_READ")
    mo_b = counter("MAP_OUTPUT_BYTES")
    out_b = counter("HDFS_BYTES_WRITTEN") or counter("FILE_BYTES_WRITTEN")
    m_info = [story.getTaskAttemptInfo("MAP", i) for i in range(maps)]
    r_info = [story.getTaskAttemptInfo("REDUCE", i) for i in range(reds)]
    sleep = kind == "SLEEPJOB"
    map_specs = [{"in": 0 if sleep else a, "out": 0 if sleep else b,
                  "ms": int(inf["runtime_ms"] * time_scale) if sleep else 0}
                 for a, b, inf in zip(_even(in_b, maps), _even(mo_b, maps), m_info)]
    red_specs = [{"out": 0 if sleep else a, "ms": int(inf["runtime_ms"] * time_scale)
                  if sleep else 0} for a, inf in zip(_even(out_b, reds), r_info)]
    job = JobConf(base_conf)
    job.set_job_name(f"GRIDMIX{kind}.{lj['jobID']}")
    job.set("gridmix.job.original-job-id", lj["jobID"])
    job.set_int("gridmix.maps", maps)
    job.set("gridmix.map.specs", json.dumps(map_specs))
    job.set("gridmix.reduce.specs", json.dumps(red_specs))
    job.set("gridmix.gpu.maps", json.dumps([i for i, inf in enumerate(m_info) if inf["gpu"]]))
    job.set_strings("gridmix.pool", list(pool or []))
    job.set_num_map_tasks(maps)
    job.set_num_reduce_tasks(reds)
    job.set_input_format(GridmixInputFormat)
    job.set_mapper_class(LoadMapper)
    job.set_reducer_class(LoadReducer)
    job.set_partitioner_class(GridmixPartitioner)
    job.set_map_output_key_class(IntWritable)
    job.set_map_output_value_class(BytesWritable)
    job.set_output_key_class(NullWritable)
    job.set_output_value_class(BytesWritable)
    job.set_speculative_execution(False)
    if sleep or not out_dir or reds == 0:
        job.set_output_format(NullOutputFormat)
    else:
        job.set_output_format(SequenceFileOutputFormat)
        FileOutputFormat.setOutputPath(job, os.path.join(out_dir, lj["jobID"]))
    return job


def run(trace, kind="LOADJOB", policy="STRESS", pool=None, time_scale=1.0, out_dir=None,
        cluster=None, conf=None, max_in_flight=4, max_jobs=None, seed=0) -> dict:
    """Replay a trace; returns Statistics ({jobs: [...], makespan_s})."""
    kind, policy = kind.upper(), policy.upper()
    if kind not in ("LOADJOB", "SLEEPJOB") or policy not in ("REPLAY", "STRESS", "SERIAL"):
        raise ValueError(f"bad job type / policy {kind}/{policy}")
    producer = ZombieJobProducer(trace, seed)
    stories = []
    while max_jobs is None or len(stories) < max_jobs:
        s = producer.getNextJob()
        if s is None:
            break
        stories.append(s)
    client = JobClient(conf, cluster=cluster)
    stats, lock = [], threading.Lock()
    running = []
    t0 = time.time()
    first_submit = stories[0].getSubmissionTime() if stories else 0
    sem = threading.Semaphore(1 if policy == "SERIAL" else
                              (max_in_flight if policy == "STRESS" else 1 << 30))

    def monitor(rj, rec):
        rj.waitForCompletion()
        rec["finish_s"] = time.time() - t0
        rec["runtime_s"] = rec["finish_s"] - rec["submit_s"]
        rec["successful"] = rj.isSuccessful()
        sem.release()

    for s in stories:
        if policy == "REPLAY":
            due = (s.getSubmissionTime() - first_submit) / 1000.0 * time_scale
            wait = due - (time.time() - t0)
            if wait > 0:
                time.sleep(wait)
        sem.acquire()
        job = job_from_story(s, kind, pool, time_scale, out_dir, conf)
        rec = {"job": s.job["jobID"], "maps": s.getNumberMaps(),
               "reduces": s.getNumberReduces(), "submit_s": time.time() - t0}
        rj = client.submitJob(job)
        th = threading.Thread(target=monitor, args=(rj, rec), daemon=True)
        th.start()
        with lock:
            stats.append(rec)
            running.append(th)
    for th in running:
        th.join()
    return {"kind": kind, "policy": policy, "jobs": stats, "makespan_s": time.time() - t0,
            "succeeded": sum(1 for r in stats if r.get("successful"))}


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr gridmix",
                                 description="gridmix [-generate <bytes>] <iopath> <trace>")
    ap.add_argument("-generate", type=int, default=0)
    ap.add_argument("-jobtype", default="LOADJOB", choices=["LOADJOB", "SLEEPJOB"])
    ap.add_argument("-policy", default="STRESS", choices=["REPLAY", "STRESS", "SERIAL"])
    ap.add_argument("-timescale", type=float, default=1.0)
    ap.add_argument("iopath")
    ap.add_argument("trace")
    a = ap.parse_args(argv)
    pool_dir = os.path.join(a.iopath, "input")
    pool = generate_data(pool_dir, a.generate) if a.generate else \
        ([os.path.join(pool_dir, f) for f in sorted(os.listdir(pool_dir))]
         if os.path.isdir(pool_dir) else [])
    st = run(a.trace, a.jobtype, a.policy, pool, a.timescale,
             os.path.join(a.iopath, "output"), cluster=cluster)
    print(json.dumps(st, indent=1))
    return 0 if st["succeeded"] == len(st["jobs"]) else 1
