"""NNBench: NameNode metadata-operation load test.

Behaviour from hadoop-1.0.3/src/test/org/apache/hadoop/hdfs/NNBench.java:
operations ``create_write``, ``open_read``, ``rename``, ``delete``; ``-maps``,
``-numberOfFiles`` per map, ``-bytesToWrite``, ``-baseDir``,
``-startTime`` (maps wait so they hit the NameNode together); every map
records successful operations, exceptions and per-operation latency; the
reducer sums them and the driver prints TPS (successful file operations over
the longest map's wall time), average latency and exceptions.

Runs against ``hdfs://`` (hbmr.dfs NameNode RPC) or a local directory.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import tempfile
import time

from ..fs import get_fs
from ..io.writable import Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.api import Mapper, Reducer
from ..tools.distcp import _ChunkInputFormat

OPS = ("create_write", "open_read", "rename", "delete")


class NNBenchMapper(Mapper):
    def configure(self, job):
        self.job = job
        self.op = job.get("test.nnbench.operation")
        self.n = job.get_int("test.nnbench.numberoffiles", 1)
        self.nbytes = job.get_int("test.nnbench.bytestowrite", 0)
        self.base = job.get("test.nnbench.basedir")
        self.start_at = job.get_float("test.nnbench.starttime", 0.0)

    def map(self, key, value, output, reporter):
        name = str(value).strip()
        fs = get_fs(self.base, self.job)
        d = f"{self.base}/data"
        wait = self.start_at - time.time()
        if wait > 0:  # barrier: all maps start together (NNBench -startTime)
            time.sleep(wait)
        ok = exc = 0
        lat = 0.0
        t_start = time.time()
        payload = b"a" * self.nbytes
        for i in range(self.n):
            f = f"{d}/file_{name}_{i}"
            t0 = time.perf_counter()
            try:
                if self.op == "create_write":
                    with fs.create(f, overwrite=True) as out:
                        if payload:
                            out.write(payload)
                elif self.op == "open_read":
                    with fs.open(f) as inp:
                        inp.read()
                elif self.op == "rename":
                    if not fs.rename(f, f"{d}/file_{name}_{i}_r"):
                        raise OSError("rename failed")
                elif self.op == "delete":
                    p = f"{d}/file_{name}_{i}_r" if fs.exists(f"{d}/file_{name}_{i}_r") else f
                    if not fs.delete(p, recursive=False):
                        raise OSError("delete failed")
                ok += 1
                lat += (time.perf_counter() - t0) * 1000.0
            except Exception:  # noqa: BLE001 - counted, as NNBench's numOfExceptions
                exc += 1
            reporter.progress()
        t_end = time.time()
        output.collect(Text("stats"), Text(json.dumps(
            {"successful_ops": ok, "exceptions": exc, "latency_ms": lat,
             "start": t_start, "end": t_end})))


class NNBenchReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        acc = {"successful_ops": 0, "exceptions": 0, "latency_ms": 0.0, "start": None,
               "end": None, "maps": 0}
        for v in values:
            s = json.loads(str(v))
            acc["maps"] += 1
            for k in ("successful_ops", "exceptions", "latency_ms"):
                acc[k] += s[k]
            acc["start"] = s["start"] if acc["start"] is None else min(acc["start"], s["start"])
            acc["end"] = s["end"] if acc["end"] is None else max(acc["end"], s["end"])
        output.collect(key, Text(json.dumps(acc)))


def run(operation, maps=2, files_per_map=10, bytes_to_write=0, base_dir=None, conf=None,
        cluster=None, start_delay_s=0.5) -> dict:
    if operation not in OPS:
        raise ValueError(f"operation must be one of {OPS}")
    base = base_dir or os.path.join(tempfile.gettempdir(), "benchmarks", "NNBench")
    job = JobConf(conf)
    get_fs(base, job).mkdirs(f"{base}/data")
    work = tempfile.mkdtemp(prefix="nnbench-ctl-")
    try:
        for i in range(maps):
            with open(os.path.join(work, f"NNBench_Controlfile_{i:05d}"), "w") as f:
                f.write(f"{i}\n")
        job.set_job_name(f"NNBench-{operation}")
        job.set("test.nnbench.operation", operation)
        job.set_int("test.nnbench.numberoffiles", files_per_map)
        job.set_int("test.nnbench.bytestowrite", bytes_to_write)
        job.set("test.nnbench.basedir", base)
        job.set_float("test.nnbench.starttime", time.time() + start_delay_s)
        job.set_boolean("mapred.map.tasks.speculative.execution", False)
        FileInputFormat.setInputPaths(job, work)
        job.set_input_format(_ChunkInputFormat)
        job.set_mapper_class(NNBenchMapper)
        job.set_reducer_class(NNBenchReducer)
        job.set_num_map_tasks(maps)
        job.set_num_reduce_tasks(1)
        for setter in (job.set_map_output_key_class, job.set_map_output_value_class,
                       job.set_output_key_class, job.set_output_value_class):
            setter(Text)
        FileOutputFormat.setOutputPath(job, os.path.join(work, "output"))
        JobClient.runJob(job, cluster=cluster, verbose=False)
        with open(os.path.join(work, "output", "part-00000")) as f:
            acc = json.loads(f.read().split("\t", 1)[1])
    finally:
        shutil.rmtree(work, ignore_errors=True)
    wall = max(acc["end"] - acc["start"], 1e-9)
    ok = acc["successful_ops"]
    return {"operation": operation, "maps": maps, "files_per_map": files_per_map,
            "successful_file_ops": ok, "exceptions": acc["exceptions"],
            "tps": ok / wall, "avg_latency_ms": acc["latency_ms"] / max(ok, 1),
            "wall_s": wall}


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="NNBench")
    ap.add_argument("-operation", required=True, choices=OPS)
    ap.add_argument("-maps", type=int, default=1)
    ap.add_argument("-numberOfFiles", type=int, default=1)
    ap.add_argument("-bytesToWrite", type=int, default=0)
    ap.add_argument("-baseDir", default=None)
    a = ap.parse_args(argv)
    print(json.dumps(run(a.operation, a.maps, a.numberOfFiles, a.bytesToWrite, a.baseDir,
                         cluster=cluster)))
    return 0
