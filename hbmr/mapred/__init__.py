"""The MapReduce layer: old-style API, job configuration, runners, control plane."""
from .api import (GpuMapper, InputFormat, InputSplit, MapRunnable, Mapper, OutputCollector,  # noqa: F401
                  OutputFormat, Partitioner, RecordReader, RecordWriter, Reducer, Reporter)
from .counters import Counters  # noqa: F401
from .formats import (FileInputFormat, FileOutputFormat, FileSplit, KeyValueTextInputFormat,  # noqa: F401
                      MapFileOutputFormat, NLineInputFormat, NullOutputFormat, SequenceFileAsTextInputFormat,
                      SequenceFileInputFormat, SequenceFileOutputFormat, TextInputFormat,
                      TextOutputFormat)
from .jobclient import JobClient, RunningJob  # noqa: F401
from .jobconf import JobConf  # noqa: F401
