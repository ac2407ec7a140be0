"""StreamJob: the ``hbmr streaming`` command line (hadoop-1.0.3
contrib/streaming StreamJob.java:287-471 options, :640-800 setJobConf).

  hbmr streaming -input IN [-input IN2 ...] -output OUT
      -mapper CMD|CLASS [-combiner CMD|CLASS] [-reducer CMD|CLASS|NONE|aggregate]
      [-file F]... [-cacheFile URI#link]... [-cacheArchive URI#link]...
      [-inputformat CLS] [-outputformat CLS] [-partitioner CLS]
      [-inputreader "CLASS,k=v,..."] [-io text|rawbytes|typedbytes]
      [-numReduceTasks N] [-cmdenv K=V]... [-D K=V]... [-jobconf K=V]...
      [-mapdebug CMD] [-reducedebug CMD] [-lazyOutput] [-verbose] [-info]

Field separators and key-field counts are plain job properties:
``stream.map.input.field.separator``, ``stream.map.output.field.separator``,
``stream.num.map.output.key.fields`` and the ``reduce`` forms.
"""
from __future__ import annotations

import argparse
import os
import sys

from ..io.writable import Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.formats import (KeyValueTextInputFormat, SequenceFileAsTextInputFormat,
                              SequenceFileInputFormat, TextInputFormat)
from . import io as sio
from .formats import StreamInputFormat, reader_class
from .pipe import PipeCombiner, PipeMapRunner, PipeReducer

_INPUT_FORMATS = {
    "TextInputFormat": TextInputFormat,
    "KeyValueTextInputFormat": KeyValueTextInputFormat,
    "SequenceFileInputFormat": SequenceFileInputFormat,
    "SequenceFileAsTextInputFormat": SequenceFileAsTextInputFormat,
    "AutoInputFormat": "hbmr.streaming.formats:AutoInputFormat",
    "StreamInputFormat": StreamInputFormat,
}


def _short(name: str) -> str:
    return name.rsplit(".", 1)[-1].rsplit(":", 1)[-1]


def _class_spec(name: str) -> str:
    """StreamUtil.goodClassOrNull: a bare class name resolves in the framework's
    packages (the reference tries org.apache.hadoop.mapred.<name>)."""
    if "." in name or ":" in name:
        return name
    from ..utils.reflection import JAVA_ALIASES
    for java, ours in JAVA_ALIASES.items():
        if java.rsplit(".", 1)[-1] == name:
            return ours
    return name


def _is_class(s):
    return ":" in s and " " not in s and not os.path.exists(s.split(":")[0])


def _parser():
    ap = argparse.ArgumentParser(prog="hbmr streaming", add_help=False)
    ap.add_argument("-input", action="append", default=[])
    ap.add_argument("-output")
    ap.add_argument("-mapper")
    ap.add_argument("-combiner")
    ap.add_argument("-reducer")
    ap.add_argument("-file", action="append", default=[])
    ap.add_argument("-cacheFile", action="append", default=[])
    ap.add_argument("-cacheArchive", action="append", default=[])
    ap.add_argument("-dfs")
    ap.add_argument("-jt")
    ap.add_argument("-additionalconfspec")
    ap.add_argument("-inputformat")
    ap.add_argument("-outputformat")
    ap.add_argument("-partitioner")
    ap.add_argument("-numReduceTasks", type=int)
    ap.add_argument("-inputreader")
    ap.add_argument("-mapdebug")
    ap.add_argument("-reducedebug")
    ap.add_argument("-jobconf", action="append", default=[])
    ap.add_argument("-cmdenv", action="append", default=[])
    ap.add_argument("-io")
    ap.add_argument("-D", action="append", default=[], dest="defines")
    ap.add_argument("-lazyOutput", action="store_true")
    ap.add_argument("-verbose", action="store_true")
    ap.add_argument("-info", action="store_true")
    ap.add_argument("-debug", action="store_true")
    ap.add_argument("-help", action="store_true")
    return ap


def usage() -> str:
    return __doc__.split("\n\n", 1)[1]


def stream_job_conf(args, conf=None) -> JobConf:
    a = _parser().parse_args(args)
    if a.help:
        raise SystemExit(usage())
    if not a.input:
        raise ValueError("Required argument: -input <name>")
    if not a.output:
        raise ValueError("Required argument: -output <name>")
    job = JobConf(conf)
    job.set_job_name("streamjob")
    for d in a.jobconf + a.defines:       # -jobconf is the deprecated spelling of -D
        k, _, v = d.partition("=")
        job.set(k.strip(), v)
    if a.additionalconfspec:
        job.add_resource(a.additionalconfspec)
    if a.dfs:
        job.set("fs.default.name", a.dfs)
    if a.jt:
        job.set("mapred.job.tracker", a.jt)
    FileInputFormat.setInputPaths(job, *a.input)
    job.set_int("stream.numinputspecs", len(a.input))
    FileOutputFormat.setOutputPath(job, a.output)

    # input format: -inputformat, else StreamInputFormat when -inputreader is
    # given, else TextInputFormat (StreamJob.setJobConf)
    if a.inputformat:
        fmt = _INPUT_FORMATS.get(_short(a.inputformat), _class_spec(a.inputformat))
    elif a.inputreader:
        fmt = StreamInputFormat
    else:
        fmt = TextInputFormat
    job.set_input_format(fmt)
    if a.inputreader:
        parts = a.inputreader.split(",")
        reader_class(parts[0])      # fail early: -inputreader: class not found
        job.set("stream.recordreader.class", parts[0])
        for kv in parts[1:]:
            k, _, v = kv.partition("=")
            job.set(f"stream.recordreader.{k}", v)

    # record encodings (-io and the IdentifierResolver)
    if a.io:
        for key in ("stream.map.input", "stream.map.output", "stream.reduce.input",
                    "stream.reduce.output"):
            job.set(key, a.io)
    rcls = job.get_class("stream.io.identifier.resolver.class") or sio.IdentifierResolver
    res = rcls()
    res.resolve(job.get("stream.map.input", sio.TEXT_ID))
    job.set_class("stream.map.input.writer.class", res.input_writer_class)
    res.resolve(job.get("stream.reduce.input", sio.TEXT_ID))
    job.set_class("stream.reduce.input.writer.class", res.input_writer_class)
    res.resolve(job.get("stream.map.output", sio.TEXT_ID))
    job.set_class("stream.map.output.reader.class", res.output_reader_class)
    job.set_map_output_key_class(res.output_key_class)
    job.set_map_output_value_class(res.output_value_class)
    res.resolve(job.get("stream.reduce.output", sio.TEXT_ID))
    job.set_class("stream.reduce.output.reader.class", res.output_reader_class)
    job.set_output_key_class(res.output_key_class)
    job.set_output_value_class(res.output_value_class)

    if a.outputformat:
        job.set("mapred.output.format.class", _class_spec(a.outputformat))
    if a.lazyOutput:
        # LazyOutputFormat: part files only for tasks that emit records
        job.set("mapred.lazy.output.format.class",
                job.get("mapred.output.format.class") or "hbmr.mapred.formats:TextOutputFormat")
        job.set("mapred.output.format.class", "hbmr.mapred.lib.lazy:LazyOutputFormat")
    if a.partitioner:
        job.set("mapred.partitioner.class", _class_spec(a.partitioner))

    if a.file:
        # -file: shipped next to the command (the task's working directory)
        work = os.path.dirname(os.path.abspath(a.file[0]))
        job.set("stream.work.dir", work)
    cache = [os.path.abspath(f) for f in a.file] + list(a.cacheFile)
    if cache:
        job.set("mapred.cache.files", ",".join(cache))
        if a.cacheFile:
            job.set_boolean("mapred.create.symlink", True)
    if a.cacheArchive:
        job.set("mapred.cache.archives", ",".join(a.cacheArchive))
        job.set_boolean("mapred.create.symlink", True)
    if a.cmdenv:
        job.set("stream.addenvironment", " ".join(a.cmdenv))
    if a.mapdebug:
        job.set("mapred.map.task.debug.script", a.mapdebug)
    if a.reducedebug:
        job.set("mapred.reduce.task.debug.script", a.reducedebug)

    mapper = a.mapper or "cat"
    if _is_class(mapper):
        job.set("mapred.mapper.class", mapper)
    else:
        job.set("stream.map.streamprocessor", mapper)
        job.set_map_runner_class(PipeMapRunner)
    reducer = a.reducer
    if reducer is None or reducer == "NONE":
        job.set_num_reduce_tasks(0 if reducer == "NONE" or a.numReduceTasks == 0 else
                                 (a.numReduceTasks if a.numReduceTasks is not None else 1))
        if reducer is None:
            job.set_reducer_class("hbmr.mapred.lib.basic:IdentityReducer")
    elif reducer.lower() == "aggregate":
        job.set_reducer_class("hbmr.mapred.lib.aggregate:ValueAggregatorReducer")
        job.set_combiner_class("hbmr.mapred.lib.aggregate:ValueAggregatorCombiner")
    elif _is_class(reducer):
        job.set("mapred.reducer.class", reducer)
    else:
        job.set("stream.reduce.streamprocessor", reducer)
        job.set_reducer_class(PipeReducer)
    if a.combiner:
        if _is_class(a.combiner):
            job.set("mapred.combiner.class", a.combiner)
        else:
            job.set("stream.combine.streamprocessor", a.combiner)
            job.set_combiner_class(PipeCombiner)
    if a.numReduceTasks is not None and reducer not in (None, "NONE"):
        job.set_num_reduce_tasks(a.numReduceTasks)
    if a.verbose:
        job.set_boolean("stream.debug", True)
    return job


def main(argv=None, cluster=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or "-help" in argv or "-info" in argv:
        print("Usage: hbmr streaming [options]\n" + usage())
        return 0 if argv else 1
    job = stream_job_conf(argv)
    rj = JobClient.runJob(job, cluster=cluster, verbose=True)
    return 0 if rj.isSuccessful() else 1


__all__ = ["stream_job_conf", "main", "usage", "Text"]
