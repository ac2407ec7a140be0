"""MRBench: many small jobs, to measure per-job framework latency.

Behaviour from hadoop-1.0.3/src/test/org/apache/hadoop/mapred/MRBench.java:
``-numRuns``, ``-maps``, ``-reduces``, ``-inputLines``, ``-inputType
ascending|descending|random``, ``-baseDir``; generates the input once, runs
the same text-sort job (Map/Reduce identity over ``TextInputFormat`` with the
line as key) ``numRuns`` times and prints
``DataLines Maps Reduces AvgTime (milliseconds)``.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import shutil
import tempfile
import time

from ..io.writable import Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.api import Mapper, Reducer


class MRBenchMapper(Mapper):
    def map(self, key, value, output, reporter):
        output.collect(Text(str(value)), Text(str(value)))


class MRBenchReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        for v in values:
            output.collect(key, v)


def generate_input(path, lines, input_type="ascending", seed=0):
    os.makedirs(path, exist_ok=True)
    order = list(range(lines))
    if input_type == "descending":
        order.reverse()
    elif input_type == "random":
        random.Random(seed).shuffle(order)
    with open(os.path.join(path, "input_0.txt"), "w") as f:
        for i in order:
            f.write(f"{i}\n")


def run(num_runs=1, maps=2, reduces=1, input_lines=1, input_type="ascending", base_dir=None,
        conf=None, cluster=None) -> dict:
    base = base_dir or tempfile.mkdtemp(prefix="mrbench-")
    inp = os.path.join(base, "mr_input")
    generate_input(inp, input_lines, input_type)
    times = []
    try:
        for i in range(num_runs):
            job = JobConf(conf)
            job.set_job_name("MRBench")
            FileInputFormat.setInputPaths(job, inp)
            FileOutputFormat.setOutputPath(job, os.path.join(base, f"mr_output_{i}"))
            job.set_mapper_class(MRBenchMapper)
            job.set_reducer_class(MRBenchReducer)
            for setter in (job.set_map_output_key_class, job.set_map_output_value_class,
                           job.set_output_key_class, job.set_output_value_class):
                setter(Text)
            job.set_num_map_tasks(maps)
            job.set_num_reduce_tasks(reduces)
            t0 = time.perf_counter()
            JobClient.runJob(job, cluster=cluster, verbose=False)
            times.append((time.perf_counter() - t0) * 1000.0)
    finally:
        if base_dir is None:
            shutil.rmtree(base, ignore_errors=True)
    return {"DataLines": input_lines, "Maps": maps, "Reduces": reduces,
            "AvgTime_ms": sum(times) / len(times), "times_ms": times}


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="MRBench")
    ap.add_argument("-numRuns", type=int, default=1)
    ap.add_argument("-maps", type=int, default=2)
    ap.add_argument("-reduces", type=int, default=1)
    ap.add_argument("-inputLines", type=int, default=1)
    ap.add_argument("-inputType", default="ascending", choices=["ascending", "descending", "random"])
    ap.add_argument("-baseDir", default=None)
    a = ap.parse_args(argv)
    r = run(a.numRuns, a.maps, a.reduces, a.inputLines, a.inputType, a.baseDir, cluster=cluster)
    print("DataLines\tMaps\tReduces\tAvgTime (milliseconds)")
    print(f"{r['DataLines']}\t\t{r['Maps']}\t{r['Reduces']}\t{r['AvgTime_ms']:.0f}")
    print(json.dumps(r))
    return 0
