"""TestDFSIO: distributed file-system I/O throughput benchmark.

Behaviour from hadoop-1.0.3/src/test/org/apache/hadoop/fs/TestDFSIO.java:
``-write``/``-read``/``-append``/``-clean``, ``-nrFiles N``, ``-fileSize MB``,
``-bufferSize``, ``-resFile``; one map per file writes (or reads) the file under
``<baseDir>/io_data/test_io_<i>`` and reports ``tasks``, ``size``, ``time`` and
the per-task rate; one reducer sums them; the result lines are
``Throughput mb/sec = size / time``, ``Average IO rate mb/sec = Σrate / tasks``
and ``IO rate std deviation = sqrt(|Σrate² / tasks − avg²|)``.

Works against any hbmr FileSystem: ``hdfs://`` (hbmr.dfs DataNodes on NVMe)
or a local directory (page cache / NVMe).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import tempfile
import time

from ..fs import get_fs
from ..io.writable import Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.api import Mapper, Reducer
from ..tools.distcp import _ChunkInputFormat

MB = 1 << 20


class IOMapper(Mapper):
    def configure(self, job):
        self.job = job
        self.mode = job.get("test.io.mode", "write")
        self.buf = job.get_int("test.io.file.buffer.size", MB)
        self.base = job.get("test.build.data")

    def map(self, key, value, output, reporter):
        name, size_mb = str(value).split("\t")
        size = int(size_mb) * MB
        path = f"{self.base}/io_data/{name}"
        fs = get_fs(path, self.job)
        t0 = time.perf_counter()
        if self.mode in ("write", "append"):
            block = (bytes(range(256)) * (self.buf // 256 + 1))[:self.buf]
            if self.mode == "append" and fs.exists(path):
                with fs.open(path) as f:
                    old = f.read()
            else:
                old = b""
            with fs.create(path, overwrite=True) as f:
                if old:
                    f.write(old)
                left = size
                while left > 0:
                    n = min(left, self.buf)
                    f.write(block[:n])
                    left -= n
                    reporter.progress()
        else:
            left = size
            with fs.open(path) as f:
                while left > 0:
                    b = f.read(min(left, self.buf))
                    if not b:
                        break
                    left -= len(b)
                    reporter.progress()
            size -= left
        ms = max((time.perf_counter() - t0) * 1000.0, 1e-3)
        rate = size / MB / (ms / 1000.0)
        stats = {"tasks": 1, "size": size, "time": ms, "rate": rate, "sqrate": rate * rate}
        output.collect(Text("stats"), Text(json.dumps(stats)))


class AccumulatingReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        acc = {}
        for v in values:
            for k, x in json.loads(str(v)).items():
                acc[k] = acc.get(k, 0) + x
        output.collect(key, Text(json.dumps(acc)))


def run(mode="write", nr_files=4, file_size_mb=16, base_dir=None, buffer_size=MB,
        conf=None, cluster=None, res_file=None) -> dict:
    if mode not in ("write", "read", "append"):
        raise ValueError(mode)
    base = base_dir or os.path.join(tempfile.gettempdir(), "benchmarks", "TestDFSIO")
    job = JobConf(conf)
    work = tempfile.mkdtemp(prefix="dfsio-ctl-")
    try:
        for i in range(nr_files):  # io_control: one control file per map
            with open(os.path.join(work, f"in_file_test_io_{i:05d}"), "w") as f:
                f.write(f"test_io_{i}\t{file_size_mb}\n")
        get_fs(base, job).mkdirs(f"{base}/io_data")
        job.set_job_name(f"TestDFSIO-{mode}")
        job.set("test.io.mode", mode)
        job.set("test.build.data", base)
        job.set_int("test.io.file.buffer.size", buffer_size)
        job.set_boolean("mapred.map.tasks.speculative.execution", False)
        FileInputFormat.setInputPaths(job, work)
        job.set_input_format(_ChunkInputFormat)
        job.set_mapper_class(IOMapper)
        job.set_reducer_class(AccumulatingReducer)
        job.set_num_map_tasks(nr_files)
        job.set_num_reduce_tasks(1)
        job.set_map_output_key_class(Text)
        job.set_map_output_value_class(Text)
        job.set_output_key_class(Text)
        job.set_output_value_class(Text)
        FileOutputFormat.setOutputPath(job, os.path.join(work, "io_write"))
        t0 = time.time()
        JobClient.runJob(job, cluster=cluster, verbose=False)
        exec_s = time.time() - t0
        with open(os.path.join(work, "io_write", "part-00000")) as f:
            acc = json.loads(f.read().split("\t", 1)[1])
    finally:
        shutil.rmtree(work, ignore_errors=True)
    tasks = acc.get("tasks", 0) or 1
    avg = acc.get("rate", 0.0) / tasks
    res = {"mode": mode, "nrFiles": nr_files, "fileSizeMB": file_size_mb,
           "totalMBytes": acc.get("size", 0) / MB,
           "throughput_mb_s": (acc.get("size", 0) / MB) / (acc.get("time", 1) / 1000.0),
           "avg_io_rate_mb_s": avg,
           "io_rate_std_dev": math.sqrt(abs(acc.get("sqrate", 0.0) / tasks - avg * avg)),
           "exec_time_s": exec_s}
    if res_file:
        with open(res_file, "a") as f:
            f.write(f"----- TestDFSIO ----- : {mode}\n"
                    f"           Number of files: {nr_files}\n"
                    f"    Total MBytes processed: {res['totalMBytes']:.0f}\n"
                    f"         Throughput mb/sec: {res['throughput_mb_s']:.3f}\n"
                    f"    Average IO rate mb/sec: {avg:.3f}\n"
                    f"     IO rate std deviation: {res['io_rate_std_dev']:.3f}\n"
                    f"        Test exec time sec: {exec_s:.3f}\n\n")
    return res


def clean(base_dir, conf=None):
    fs = get_fs(base_dir, conf)
    if fs.exists(base_dir):
        fs.delete(base_dir, recursive=True)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="TestDFSIO")
    g = ap.add_mutually_exclusive_group(required=True)
    for m in ("write", "read", "append", "clean"):
        g.add_argument(f"-{m}", dest="mode", action="store_const", const=m)
    ap.add_argument("-nrFiles", type=int, default=1)
    ap.add_argument("-fileSize", type=int, default=1, help="MB")
    ap.add_argument("-bufferSize", type=int, default=MB)
    ap.add_argument("-baseDir", default=None)
    ap.add_argument("-resFile", default="TestDFSIO_results.log")
    a = ap.parse_args(argv)
    if a.mode == "clean":
        clean(a.baseDir or os.path.join(tempfile.gettempdir(), "benchmarks", "TestDFSIO"))
        return 0
    print(json.dumps(run(a.mode, a.nrFiles, a.fileSize, a.baseDir, a.bufferSize,
                         cluster=cluster, res_file=a.resFile)))
    return 0
