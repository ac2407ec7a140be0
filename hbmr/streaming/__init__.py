"""Hadoop Streaming: map/reduce with any executable over stdin/stdout
(hadoop-1.0.3 contrib/streaming: StreamJob, PipeMapRed, PipeMapper,
PipeReducer, StreamInputFormat, StreamXmlRecordReader, AutoInputFormat,
DumpTypedBytes, LoadTypedBytes, streaming/io/*, typedbytes/*).

  hbmr streaming -input IN -output OUT -mapper CMD [-reducer CMD|NONE] ...

Modules: :mod:`.job` (command line → JobConf), :mod:`.pipe` (the task side),
:mod:`.io` (text / rawbytes / typedbytes record encodings), :mod:`.formats`
(StreamInputFormat, StreamXmlRecordReader, AutoInputFormat), :mod:`.dumptb`
(``hbmr dumptb`` / ``hbmr loadtb``); the typed bytes codec is
:mod:`hbmr.typedbytes`.
"""
from .formats import AutoInputFormat, StreamInputFormat, StreamXmlRecordReader
from .io import IdentifierResolver, split_key_value
from .job import main, stream_job_conf, usage
from .pipe import PipeCombiner, PipeMapRunner, PipeReducer

__all__ = ["main", "stream_job_conf", "usage", "PipeMapRunner", "PipeReducer", "PipeCombiner",
           "StreamInputFormat", "StreamXmlRecordReader", "AutoInputFormat", "IdentifierResolver",
           "split_key_value"]
