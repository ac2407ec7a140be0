"""Hadoop Streaming: map/reduce with any executable over text stdin/stdout
(hadoop-1.0.3 contrib/streaming: StreamJob, PipeMapRed, PipeMapper,
PipeReducer).

  hbmr streaming -input IN -output OUT -mapper CMD [-reducer CMD|NONE]
                 [-combiner CMD] [-file F]... [-numReduceTasks N]
                 [-inputformat CLS] [-outputformat CLS] [-partitioner CLS]
                 [-cmdenv K=V]... [-D K=V]...

Protocol (as the reference): the mapper's stdin gets one line per input
record — the value only for TextInputFormat, else ``key\\tvalue`` — and each
stdout line is split at the first tab into (key, value) Text; the reducer's
stdin gets ``key\\tvalue`` lines grouped by key in sorted order.  Lines on stderr
of the form ``reporter:counter:<group>,<counter>,<amount>`` and
``reporter:status:<message>`` update counters / status.  A ``-mapper`` or
``-reducer`` of the form ``module:Class`` is used as an in-process class.
A command exiting non-zero fails the task (stream.non.zero.exit.is.failure).
"""
from __future__ import annotations

import argparse
import logging
import os
import shlex
import subprocess
import sys
import threading

from .io.writable import Text
from .mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from .mapred.api import MapRunnable, Reducer
from .mapred.formats import TextInputFormat

log = logging.getLogger("hbmr.streaming")


def _split_line(line: bytes, sep=b"\t"):
    line = line.rstrip(b"\n").rstrip(b"\r") if line.endswith(b"\n") else line
    k, s, v = line.partition(sep)
    return Text(k), Text(v if s else b"")


class _Proc:
    """A running stream command with stdout/stderr pump threads."""

    def __init__(self, job, cmd_key, output, reporter):
        cmd = job.get(cmd_key)
        env = dict(os.environ)
        for kv in (job.get("stream.addenvironment") or "").split():
            k, _, v = kv.partition("=")
            env[k] = v
        cwd = job.get("stream.work.dir") or None
        self.p = subprocess.Popen(cmd if isinstance(cmd, list) else shlex.split(cmd),
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, env=env, cwd=cwd)
        self.out, self.rep = output, reporter
        self.err: list[str] = []
        self.n_out = 0
        self.t_out = threading.Thread(target=self._pump_out, daemon=True)
        self.t_err = threading.Thread(target=self._pump_err, daemon=True)
        self.t_out.start()
        self.t_err.start()

    def _pump_out(self):
        for line in self.p.stdout:
            k, v = _split_line(line)
            self.out.collect(k, v)
            self.n_out += 1

    def _pump_err(self):
        for raw in self.p.stderr:
            line = raw.decode(errors="replace").rstrip("\n")
            if line.startswith("reporter:counter:"):
                try:
                    g, c, a = line[len("reporter:counter:"):].split(",")
                    self.rep.incrCounter(g, c, int(a))
                except ValueError:
                    self.err.append(line)
            elif line.startswith("reporter:status:"):
                self.rep.setStatus(line[len("reporter:status:"):])
            else:
                self.err.append(line)
                if len(self.err) > 200:
                    self.err.pop(0)

    def write(self, b: bytes):
        self.p.stdin.write(b)

    def finish(self, fail_on_nonzero=True):
        try:
            self.p.stdin.close()
        except BrokenPipeError:
            pass
        rc = self.p.wait()
        self.t_out.join()
        self.t_err.join()
        if rc != 0 and fail_on_nonzero:
            raise RuntimeError(f"PipeMapRed.waitOutputThreads(): subprocess failed with code {rc}"
                               f"\n" + "\n".join(self.err[-20:]))
        return rc


def _bytes(x) -> bytes:
    if x is None:
        return b""
    if isinstance(x, Text):
        return x.bytes
    return str(x).encode()


class PipeMapRunner(MapRunnable):
    """Feeds every input record to the ``stream.map.streamprocessor`` command."""

    def configure(self, job):
        self.job = job
        fmt = job.get("mapred.input.format.class", "")
        self.ignore_key = job.get_boolean("stream.map.input.ignoreKey",
                                          fmt.endswith("TextInputFormat") or not fmt)

    def run(self, reader, output, reporter):
        proc = _Proc(self.job, "stream.map.streamprocessor", output, reporter)
        n = 0
        try:
            while True:
                kv = reader.next()
                if kv is None:
                    break
                k, v = kv
                line = _bytes(v) if self.ignore_key else _bytes(k) + b"\t" + _bytes(v)
                proc.write(line + b"\n")
                n += 1
        except BrokenPipeError:
            pass
        finally:
            proc.finish(self.job.get_boolean("stream.non.zero.exit.is.failure", True))
            reporter.incrCounter("org.apache.hadoop.mapred.Task$Counter", "MAP_INPUT_RECORDS", n)


class PipeReducer(Reducer):
    key = "stream.reduce.streamprocessor"

    def configure(self, job):
        self.job = job
        self.proc = None

    def reduce(self, key, values, output, reporter):
        if self.proc is None:
            self.proc = _Proc(self.job, self.key, output, reporter)
        kb = _bytes(key)
        for v in values:
            self.proc.write(kb + b"\t" + _bytes(v) + b"\n")

    def close(self):
        if self.proc is not None:
            self.proc.finish(self.job.get_boolean("stream.non.zero.exit.is.failure", True))


class PipeCombiner(PipeReducer):
    key = "stream.combine.streamprocessor"


def _is_class(s):
    return ":" in s and " " not in s and not os.path.exists(s.split(":")[0])


def stream_job_conf(args, conf=None) -> JobConf:
    ap = argparse.ArgumentParser(prog="hbmr streaming")
    ap.add_argument("-input", action="append", required=True)
    ap.add_argument("-output", required=True)
    ap.add_argument("-mapper", default="cat")
    ap.add_argument("-reducer", default="NONE")
    ap.add_argument("-combiner")
    ap.add_argument("-file", action="append", default=[])
    ap.add_argument("-numReduceTasks", type=int)
    ap.add_argument("-inputformat")
    ap.add_argument("-outputformat")
    ap.add_argument("-partitioner")
    ap.add_argument("-cmdenv", action="append", default=[])
    ap.add_argument("-D", action="append", default=[], dest="defines")
    ap.add_argument("-verbose", action="store_true")
    a = ap.parse_args(args)
    job = JobConf(conf)
    job.set_job_name("streamjob")
    for d in a.defines:
        k, _, v = d.partition("=")
        job.set(k, v)
    FileInputFormat.setInputPaths(job, *a.input)
    FileOutputFormat.setOutputPath(job, a.output)
    job.set_input_format(a.inputformat or TextInputFormat)
    if a.outputformat:
        job.set("mapred.output.format.class", a.outputformat)
    if a.partitioner:
        job.set("mapred.partitioner.class", a.partitioner)
    job.set_output_key_class(Text)
    job.set_output_value_class(Text)
    job.set_map_output_key_class(Text)
    job.set_map_output_value_class(Text)
    if a.file:
        # -file: shipped next to the command (the task's working directory)
        work = os.path.dirname(os.path.abspath(a.file[0]))
        job.set("stream.work.dir", work)
        job.set("mapred.cache.files", ",".join(os.path.abspath(f) for f in a.file))
    if a.cmdenv:
        job.set("stream.addenvironment", " ".join(a.cmdenv))
    if _is_class(a.mapper):
        job.set("mapred.mapper.class", a.mapper)
    else:
        job.set("stream.map.streamprocessor", a.mapper)
        job.set_map_runner_class(PipeMapRunner)
    if a.reducer == "NONE":
        job.set_num_reduce_tasks(0)
    elif _is_class(a.reducer):
        job.set("mapred.reducer.class", a.reducer)
    else:
        job.set("stream.reduce.streamprocessor", a.reducer)
        job.set_reducer_class(PipeReducer)
    if a.combiner:
        if _is_class(a.combiner):
            job.set("mapred.combiner.class", a.combiner)
        else:
            job.set("stream.combine.streamprocessor", a.combiner)
            job.set_combiner_class(PipeCombiner)
    if a.numReduceTasks is not None and a.reducer != "NONE":
        job.set_num_reduce_tasks(a.numReduceTasks)
    return job


def main(argv=None, cluster=None):
    job = stream_job_conf(list(sys.argv[1:] if argv is None else argv))
    rj = JobClient.runJob(job, cluster=cluster, verbose=True)
    return 0 if rj.isSuccessful() else 1
