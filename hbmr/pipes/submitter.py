"""Submit Pipes jobs: ``hbmr pipes -input I -output O -cpubin C -gpubin G ...``.

Mirrors hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/pipes/Submitter.java
(setupPipesJob :291-380, CLI :435-557) with the fork's -cpubin/-gpubin
(:419-420, 458-459, 523-529).  Fixed relative to the fork: a GPU-only job
(no CPU binary) is valid — its maps only take GPU slots and its reduces run
the GPU binary in CPU mode (the fork wrote fileCache[1] with count=1 and
crashed).
"""
from __future__ import annotations

import argparse
import logging
import os

from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.formats import NullOutputFormat
from .runner import (JAVA_MAPPER, JAVA_PARTITIONER, JAVA_REDUCER, JAVA_RR, JAVA_RW,
                     PipesGPUMapRunner, PipesMapRunner, PipesNonJavaInputFormat,
                     PipesPartitioner, PipesReducer)

log = logging.getLogger("hbmr.pipes")


DEFAULT_DEBUG_SCRIPT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "debug",
                                    "pipes-default-script")


def _exe(path):
    """``<path>#<name>`` (DistributedCache symlink form) -> (abs path, name)."""
    p, _, link = str(path).partition("#")
    return os.path.abspath(p), link or None


def set_executable(conf, path):
    p, link = _exe(path)
    conf.set_cpu_executable(p)
    if link:
        conf.set("hbmr.pipes.executable.link", link)


def set_gpu_executable(conf, path):
    p, link = _exe(path)
    conf.set_gpu_executable(p)
    if link:
        conf.set("hbmr.pipes.gpu.executable.link", link)


def setup_pipes_job(conf: JobConf):
    """setupPipesJob: wire the Pipes runner/partitioner/reducer/formats."""
    if not conf.get_boolean(JAVA_MAPPER, False):
        conf.set_map_runner_class(PipesMapRunner)
        conf.set_gpu_map_runner_class(PipesGPUMapRunner)
        if conf.get(JAVA_PARTITIONER) is None:
            conf.set(JAVA_PARTITIONER, conf.get("mapred.partitioner.class",
                                                "hbmr.mapred.lib.basic:HashPartitioner"))
        conf.set_partitioner_class(PipesPartitioner)
    if not conf.get_boolean(JAVA_REDUCER, False):
        conf.set_reducer_class(PipesReducer)
        if not conf.get_boolean(JAVA_RW, False):
            conf.set_output_format(NullOutputFormat)
    for k in ("mapred.output.key.class", "mapred.output.value.class"):
        if conf.get(k) is None:
            conf.set(k, "hbmr.io.writable:Text")
    if conf.get("mapred.mapoutput.key.class") is None:
        conf.set("mapred.mapoutput.key.class", conf.get("mapred.output.key.class"))
    if conf.get("mapred.mapoutput.value.class") is None:
        conf.set("mapred.mapoutput.value.class", conf.get("mapred.output.value.class"))
    if not conf.get_boolean(JAVA_RR, False) and \
            not conf.get("mapred.input.format.class", "").endswith("PipesNonJavaInputFormat"):
        if conf.get("mapred.input.format.class") is not None:
            conf.set("mapred.pipes.user.inputformat", conf.get("mapred.input.format.class"))
        conf.set_input_format(PipesNonJavaInputFormat)
    cpu, gpu = conf.get_cpu_executable(), conf.get_gpu_executable()
    if not cpu and not gpu:
        raise ValueError("No application program defined (-program/-cpubin/-gpubin).")
    # executables given as <path>#<name>: default gdb-style debug scripts for
    # failed map and reduce attempts (Submitter.java:341-347)
    if conf.get("hbmr.pipes.executable.link") or conf.get("hbmr.pipes.gpu.executable.link"):
        for key in ("mapred.map.task.debug.script", "mapred.reduce.task.debug.script"):
            if conf.get(key) is None:
                conf.set(key, DEFAULT_DEBUG_SCRIPT)
    for exe in (cpu, gpu):
        if exe and not os.access(exe, os.X_OK):
            raise FileNotFoundError(f"pipes executable {exe} is not executable")
    # a job without a CPU binary must not be placed on CPU slots
    conf.set_boolean("hbmr.job.cpu.capable", bool(cpu))
    return conf


def run_job(conf, cluster=None, verbose=True):
    setup_pipes_job(conf)
    return JobClient.runJob(conf, cluster=cluster, verbose=verbose)


def submit_job(conf, cluster=None):
    setup_pipes_job(conf)
    return JobClient(conf, cluster=cluster).submitJob(conf)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr pipes",
                                 description="Run a Pipes job (CPU and/or GPU binaries)")
    ap.add_argument("-input", required=False)
    ap.add_argument("-output", required=False)
    ap.add_argument("-jar")
    ap.add_argument("-inputformat")
    ap.add_argument("-map")
    ap.add_argument("-partitioner")
    ap.add_argument("-reduce")
    ap.add_argument("-writer")
    ap.add_argument("-program", help="CPU executable (alias of -cpubin)")
    ap.add_argument("-cpubin")
    ap.add_argument("-gpubin")
    ap.add_argument("-reduces", type=int)
    ap.add_argument("-jobconf", action="append", default=[], help="k=v[,k=v...] (deprecated)")
    ap.add_argument("-conf", action="append", default=[])
    ap.add_argument("-D", action="append", default=[], dest="defines")
    ap.add_argument("-lazyOutput", action="store_true")
    a = ap.parse_args(argv)
    conf = JobConf()
    for c in a.conf:
        conf.add_resource(c)
    for d in a.defines:
        k, _, v = d.partition("=")
        conf.set(k, v)
    for jc in a.jobconf:
        for kv in jc.split(","):
            k, _, v = kv.partition("=")
            conf.set(k, v)
    if a.input:
        FileInputFormat.setInputPaths(conf, *a.input.split(","))
    if a.output:
        FileOutputFormat.setOutputPath(conf, a.output)
    if a.inputformat:
        conf.set_boolean(JAVA_RR, True)
        conf.set("mapred.input.format.class", a.inputformat)
    if a.map:
        conf.set_boolean(JAVA_MAPPER, True)
        conf.set("mapred.mapper.class", a.map)
    if a.partitioner:
        conf.set(JAVA_PARTITIONER, a.partitioner)
    if a.reduce:
        conf.set_boolean(JAVA_REDUCER, True)
        conf.set("mapred.reducer.class", a.reduce)
    if a.writer:
        conf.set_boolean(JAVA_RW, True)
        conf.set("mapred.output.format.class", a.writer)
    if a.reduces is not None:
        conf.set_num_reduce_tasks(a.reduces)
    if a.program or a.cpubin:
        set_executable(conf, a.program or a.cpubin)
    if a.gpubin:
        set_gpu_executable(conf, a.gpubin)
    rj = run_job(conf, cluster=cluster)
    return 0 if rj.isSuccessful() else 1


Submitter = type("Submitter", (), {
    "setExecutable": staticmethod(set_executable),
    "setGPUExecutable": staticmethod(set_gpu_executable),
    "runJob": staticmethod(run_job),
    "submitJob": staticmethod(submit_job),
    "main": staticmethod(main),
})
