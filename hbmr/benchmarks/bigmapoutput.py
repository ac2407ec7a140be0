"""BigMapOutput and ThreadedMapBenchmark (hadoop-1.0.3/src/test/org/apache/
hadoop/mapred/BigMapOutput.java, ThreadedMapBenchmark.java).

* ``big_map_output`` — one map whose output is several times ``io.sort.mb``
  (large random BytesWritable keys/values, ``-create`` size), so the map side
  must spill and merge many sorted runs; an identity reduce writes it back
  and the driver checks record/byte counts survive the spill/merge path.
* ``threaded_map_benchmark`` — RandomWriter-style maps generating data then
  a sort over it with ``MultithreadedMapRunner`` and
  ``mapred.map.multithreadedrunner.threads`` threads per map, timed.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import tempfile
import time

from ..examples import randomwriter, sort
from ..io.writable import BytesWritable
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.formats import SequenceFileInputFormat, SequenceFileOutputFormat
from ..mapred.lib.basic import IdentityMapper, IdentityReducer


def big_map_output(workdir, create_mb=24, sort_mb=2, conf=None, cluster=None) -> dict:
    inp, out = os.path.join(workdir, "bigmap-in"), os.path.join(workdir, "bigmap-out")
    gen = randomwriter.make_job(inp, maps=1, bytes_per_map=create_mb << 20, conf=conf)
    gen.set_int("test.randomwrite.min_key", 10)
    gen.set_int("test.randomwrite.max_key", 10000)
    gen.set_int("test.randomwrite.min_value", 0)
    gen.set_int("test.randomwrite.max_value", 20000)
    g = JobClient.runJob(gen, cluster=cluster, verbose=False).getCounters()
    job = JobConf(conf)
    job.set_job_name("BigMapOutput")
    FileInputFormat.setInputPaths(job, inp)
    job.set_input_format(SequenceFileInputFormat)
    # the whole input in one map, so its output is create_mb >> io.sort.mb
    job.set_long("mapred.min.split.size", 1 << 62)
    job.set_mapper_class(IdentityMapper)
    job.set_reducer_class(IdentityReducer)
    job.set_output_key_class(BytesWritable)
    job.set_output_value_class(BytesWritable)
    job.set_output_format(SequenceFileOutputFormat)
    job.set_int("io.sort.mb", sort_mb)
    job.set_num_reduce_tasks(1)
    FileOutputFormat.setOutputPath(job, out)
    t0 = time.time()
    rj = JobClient.runJob(job, cluster=cluster, verbose=False)
    cs = rj.getCounters()
    tg = "org.apache.hadoop.mapred.Task$Counter"
    return {"seconds": time.time() - t0,
            "records_generated": g.get("RandomWriter", "RECORDS_WRITTEN"),
            "map_output_records": cs.get(tg, "MAP_OUTPUT_RECORDS"),
            "reduce_output_records": cs.get(tg, "REDUCE_OUTPUT_RECORDS"),
            "spilled_records": cs.get(tg, "SPILLED_RECORDS"),
            "map_output_bytes": cs.get(tg, "MAP_OUTPUT_BYTES")}


def threaded_map_benchmark(workdir, maps=2, mb_per_map=4, threads=4, reduces=1, conf=None,
                           cluster=None) -> dict:
    inp, out = os.path.join(workdir, "tmb-in"), os.path.join(workdir, "tmb-out")
    t0 = time.time()
    JobClient.runJob(randomwriter.make_job(inp, maps=maps, bytes_per_map=mb_per_map << 20,
                                           conf=conf), cluster=cluster, verbose=False)
    t1 = time.time()
    job = sort.make_job(inp, out, reduces=reduces, conf=conf)
    job.set_map_runner_class("hbmr.mapred.maprunner:MultithreadedMapRunner")
    job.set_int("mapred.map.multithreadedrunner.threads", threads)
    JobClient.runJob(job, cluster=cluster, verbose=False)
    t2 = time.time()
    return {"generate_s": t1 - t0, "sort_s": t2 - t1, "threads": threads, "maps": maps,
            "mb_per_map": mb_per_map}


def main_bigmapoutput(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="BigMapOutput")
    ap.add_argument("-create", type=int, default=24, help="MB of map output")
    ap.add_argument("-sortmb", type=int, default=2)
    a = ap.parse_args(argv)
    d = tempfile.mkdtemp(prefix="bigmapoutput-")
    try:
        print(json.dumps(big_map_output(d, a.create, a.sortmb, cluster=cluster)))
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return 0


def main_threadedmap(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="ThreadedMapBenchmark")
    ap.add_argument("-dataSizePerMap", type=int, default=4, help="MB")
    ap.add_argument("-numSpillsPerMap", type=int, default=2)
    ap.add_argument("-numMapsPerHost", type=int, default=2)
    ap.add_argument("-threads", type=int, default=4)
    a = ap.parse_args(argv)
    d = tempfile.mkdtemp(prefix="threadedmap-")
    conf = JobConf()
    conf.set_int("io.sort.mb", max(1, a.dataSizePerMap // max(1, a.numSpillsPerMap)))
    try:
        print(json.dumps(threaded_map_benchmark(d, a.numMapsPerHost, a.dataSizePerMap,
                                                a.threads, conf=conf, cluster=cluster)))
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return 0
