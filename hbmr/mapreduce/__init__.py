"""The new ("mapreduce") API: Job + context-object Mapper/Reducer.

See :mod:`hbmr.mapreduce.api` and :mod:`hbmr.mapreduce.job`."""
from .api import (Counter, InputFormat, InputSplit, JobContext, MapContext, Mapper,  # noqa: F401
                  OutputCommitter, OutputFormat, Partitioner, RecordReader, RecordWriter,
                  ReduceContext, Reducer, TaskAttemptContext)
from .job import Job  # noqa: F401
