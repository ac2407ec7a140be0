"""The streaming task side: map / combine / reduce through an external
command (hadoop-1.0.3 contrib/streaming PipeMapRed, PipeMapRunner,
PipeMapper, PipeReducer, PipeCombiner).

Records go to the command's stdin through the job's InputWriter
(``stream.{map,reduce}.input.writer.class``, text by default: the value only
for TextInputFormat input — ``stream.map.input.ignoreKey`` — else
``key<sep>value``), and come back from its stdout through the OutputReader
(``stream.{map,reduce}.output.reader.class``; text splits each line at the
``stream.num.{map,reduce}.output.key.fields``-th
``stream.{map,reduce}.output.field.separator``).  stderr lines
``<prefix>counter:<group>,<counter>,<amount>`` and ``<prefix>status:<msg>``
(prefix ``stream.stderr.reporter.prefix``, default ``reporter:``) update
counters and the task status.  A command exiting non-zero fails the task
(``stream.non.zero.exit.is.failure``).
"""
from __future__ import annotations

import logging
import os
import shlex
import subprocess
import threading

from ..mapred.api import MapRunnable, Reducer
from ..utils.reflection import load_class
from . import io as sio

log = logging.getLogger("hbmr.streaming")

_DEFAULT_WRITER = {"map": sio.TextInputWriter, "reduce": sio.TextInputWriter}
_DEFAULT_READER = {"map": sio.TextOutputReader, "reduce": sio.TextOutputReader}


def _writer(job, role, out):
    cls = job.get_class(f"stream.{role}.input.writer.class") or _DEFAULT_WRITER[role]
    w = cls()
    w.initialize(job, role, out)
    return w


def _reader(job, role, inp):
    cls = job.get_class(f"stream.{role}.output.reader.class") or _DEFAULT_READER[role]
    r = cls()
    r.initialize(job, role, inp)
    return r


class _Proc:
    """A running stream command: stdin fed by the caller through an
    InputWriter, stdout pumped through an OutputReader into ``output``,
    stderr scanned for reporter lines."""

    def __init__(self, job, cmd_key, role, output, reporter):
        cmd = job.get(cmd_key)
        env = dict(os.environ)
        for kv in (job.get("stream.addenvironment") or "").split():
            k, _, v = kv.partition("=")
            env[k] = v
        cwd = job.get("stream.work.dir") or None
        self.p = subprocess.Popen(cmd if isinstance(cmd, list) else shlex.split(cmd),
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, env=env, cwd=cwd)
        self.writer = _writer(job, role, self.p.stdin)
        self.reader = _reader(job, role, self.p.stdout)
        self.prefix = job.get("stream.stderr.reporter.prefix") or "reporter:"
        self.out, self.rep = output, reporter
        self.err: list[str] = []
        self.n_out = 0
        self.out_error = None
        self.t_out = threading.Thread(target=self._pump_out, daemon=True)
        self.t_err = threading.Thread(target=self._pump_err, daemon=True)
        self.t_out.start()
        self.t_err.start()

    def _pump_out(self):
        try:
            while True:
                kv = self.reader.read_key_value()
                if kv is None:
                    break
                self.out.collect(*kv)
                self.n_out += 1
        except Exception as e:  # noqa: BLE001
            self.out_error = e
            # drain, so the process is not blocked on a full pipe
            for _ in iter(lambda: self.p.stdout.read(1 << 16), b""):
                pass

    def _pump_err(self):
        cpre, spre = self.prefix + "counter:", self.prefix + "status:"
        for raw in self.p.stderr:
            line = raw.decode(errors="replace").rstrip("\n")
            if line.startswith(cpre):
                try:
                    g, c, a = line[len(cpre):].split(",")
                    self.rep.incrCounter(g, c, int(a))
                except ValueError:
                    self.err.append(line)
            elif line.startswith(spre):
                self.rep.setStatus(line[len(spre):])
            else:
                self.err.append(line)
                if len(self.err) > 200:
                    self.err.pop(0)

    def finish(self, fail_on_nonzero=True):
        try:
            self.p.stdin.close()
        except BrokenPipeError:
            pass
        rc = self.p.wait()
        self.t_out.join()
        self.t_err.join()
        if self.out_error is not None:
            raise RuntimeError(f"PipeMapRed: reading the command's output failed: "
                               f"{self.out_error}")
        if rc != 0 and fail_on_nonzero:
            raise RuntimeError(f"PipeMapRed.waitOutputThreads(): subprocess failed with code {rc}"
                               f"\n" + "\n".join(self.err[-20:]))
        return rc


class PipeMapRunner(MapRunnable):
    """Feeds every input record to the ``stream.map.streamprocessor`` command."""

    def configure(self, job):
        self.job = job
        fmt = job.get("mapred.input.format.class", "")
        self.ignore_key = job.get_boolean(
            "stream.map.input.ignoreKey",
            not fmt or fmt.endswith("TextInputFormat") and "KeyValue" not in fmt)

    def run(self, reader, output, reporter):
        proc = _Proc(self.job, "stream.map.streamprocessor", "map", output, reporter)
        w = proc.writer
        n = 0
        try:
            while True:
                kv = reader.next()
                if kv is None:
                    break
                k, v = kv
                if not self.ignore_key:
                    w.write_key(k)
                w.write_value(v)
                n += 1
        except BrokenPipeError:
            pass
        finally:
            proc.finish(self.job.get_boolean("stream.non.zero.exit.is.failure", True))
            reporter.incrCounter("org.apache.hadoop.mapred.Task$Counter", "MAP_INPUT_RECORDS", n)


class PipeReducer(Reducer):
    key = "stream.reduce.streamprocessor"
    role = "reduce"

    def configure(self, job):
        self.job = job
        self.proc = None

    def reduce(self, key, values, output, reporter):
        if self.proc is None:
            self.proc = _Proc(self.job, self.key, self.role, output, reporter)
        w = self.proc.writer
        try:
            for v in values:
                w.write_key(key)
                w.write_value(v)
        except BrokenPipeError:
            pass

    def close(self):
        if self.proc is not None:
            self.proc.finish(self.job.get_boolean("stream.non.zero.exit.is.failure", True))


class PipeCombiner(PipeReducer):
    """The combiner writes the map output's encoding both ways (it reads and
    produces map output records)."""
    key = "stream.combine.streamprocessor"
    role = "map"

    def configure(self, job):
        super().configure(job)
        # the combiner consumes what the map's OutputReader produced: with
        # -io rawbytes/typedbytes that is the map output encoding
        ident = job.get("stream.map.output") or sio.TEXT_ID
        res = sio.IdentifierResolver().resolve(ident)
        self._classes = (res.input_writer_class, res.output_reader_class)

    def reduce(self, key, values, output, reporter):
        if self.proc is None:
            job = self.job
            wcls, rcls = self._classes
            self.proc = _Proc(job, self.key, "map", output, reporter)
            if wcls is not type(self.proc.writer):
                self.proc.writer = wcls()
                self.proc.writer.initialize(job, "map", self.proc.p.stdin)
        super().reduce(key, values, output, reporter)


def load_writer_class(name):
    return load_class(name)
