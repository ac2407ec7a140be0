"""Job: the new-API job handle (hadoop-1.0.3 mapreduce/Job.java).

Configures through setters, submits with ``submit()`` / ``waitForCompletion()``
and then reports state, progress and counters.  Translates to a JobConf whose
old-API slots hold the adapters of :mod:`hbmr.mapreduce.adapters`.
"""
from __future__ import annotations

from ..mapred.jobclient import JobClient
from ..mapred.jobconf import JobConf
from ..utils.reflection import class_name
from . import adapters as A


class Job:
    DEFINE, RUNNING = "DEFINE", "RUNNING"

    def __init__(self, conf=None, jobName=None, cluster=None):  # noqa: N803
        self.conf = JobConf(conf) if conf is not None else JobConf()
        if jobName:
            self.conf.set_job_name(jobName)
        self.cluster = cluster
        self.state = Job.DEFINE
        self._rj = None
        c = self.conf
        c.set_map_runner_class(A.NewMapperRunner)
        c.set_reducer_class(A.NewReducerAdapter)
        c.set_partitioner_class(A.NewPartitionerAdapter)
        c.set_input_format(A.NewInputFormatAdapter)
        c.set_output_format(A.NewOutputFormatAdapter)
        for key, default in ((A.MAP_KEY, "hbmr.mapreduce.api:Mapper"),
                             (A.REDUCE_KEY, "hbmr.mapreduce.api:Reducer"),
                             (A.PARTITION_KEY, "hbmr.mapreduce.lib.partition:HashPartitioner"),
                             (A.INPUT_KEY, "hbmr.mapreduce.lib.input:TextInputFormat"),
                             (A.OUTPUT_KEY, "hbmr.mapreduce.lib.output:TextOutputFormat")):
            if c.get(key) is None:
                c.set(key, default)

    @classmethod
    def getInstance(cls, conf=None, jobName=None):  # noqa: N802
        return cls(conf, jobName)

    def _check_define(self):
        if self.state != Job.DEFINE:
            raise RuntimeError("Job in state RUNNING instead of DEFINE")

    # -- configuration -----------------------------------------------------------------
    def getConfiguration(self):  # noqa: N802
        return self.conf

    def setJobName(self, name):  # noqa: N802
        self._check_define()
        self.conf.set_job_name(name)

    def getJobName(self):  # noqa: N802
        return self.conf.get_job_name()

    def setJarByClass(self, cls):  # noqa: N802
        self.conf.set("mapred.jar.class", class_name(cls))

    def setMapperClass(self, cls):  # noqa: N802
        self._check_define()
        self.conf.set(A.MAP_KEY, class_name(cls))

    def setReducerClass(self, cls):  # noqa: N802
        self._check_define()
        self.conf.set(A.REDUCE_KEY, class_name(cls))

    def setCombinerClass(self, cls):  # noqa: N802
        self._check_define()
        self.conf.set(A.COMBINE_KEY, class_name(cls))
        self.conf.set_combiner_class(A.NewCombinerAdapter)

    def setPartitionerClass(self, cls):  # noqa: N802
        self._check_define()
        self.conf.set(A.PARTITION_KEY, class_name(cls))

    def setInputFormatClass(self, cls):  # noqa: N802
        self._check_define()
        self.conf.set(A.INPUT_KEY, class_name(cls))

    def setOutputFormatClass(self, cls):  # noqa: N802
        self._check_define()
        self.conf.set(A.OUTPUT_KEY, class_name(cls))

    def setOutputKeyClass(self, cls):  # noqa: N802
        self.conf.set_output_key_class(cls)

    def setOutputValueClass(self, cls):  # noqa: N802
        self.conf.set_output_value_class(cls)

    def setMapOutputKeyClass(self, cls):  # noqa: N802
        self.conf.set_map_output_key_class(cls)

    def setMapOutputValueClass(self, cls):  # noqa: N802
        self.conf.set_map_output_value_class(cls)

    def setSortComparatorClass(self, cls):  # noqa: N802
        self.conf.set_output_key_comparator_class(cls)

    def setGroupingComparatorClass(self, cls):  # noqa: N802
        self.conf.set_output_value_grouping_comparator(cls)

    def setNumReduceTasks(self, n):  # noqa: N802
        self._check_define()
        self.conf.set_num_reduce_tasks(n)

    def getNumReduceTasks(self):  # noqa: N802
        return self.conf.get_num_reduce_tasks()

    def setSpeculativeExecution(self, b):  # noqa: N802
        self.conf.set_speculative_execution(b)

    def setGPUExecutable(self, path):  # noqa: N802
        """hbmr: a Pipes GPU binary for the maps (the job is then GPU-capable)."""
        self.conf.set_gpu_executable(path)

    # -- lifecycle ----------------------------------------------------------------------
    def submit(self):
        self._check_define()
        self._rj = JobClient(self.conf, cluster=self.cluster).submitJob(self.conf)
        self.state = Job.RUNNING
        return self._rj

    def waitForCompletion(self, verbose=False) -> bool:  # noqa: N802
        if self.state == Job.DEFINE:
            self.submit()
        client = JobClient(self.conf, cluster=self.cluster)
        return client.monitor_and_print_job(self.conf, self._rj, verbose=verbose)

    def _need(self):
        if self._rj is None:
            raise RuntimeError("Job not submitted")
        return self._rj

    def isComplete(self):  # noqa: N802
        return self._need().isComplete()

    def isSuccessful(self):  # noqa: N802
        return self._need().isSuccessful()

    def mapProgress(self):  # noqa: N802
        return self._need().mapProgress()

    def reduceProgress(self):  # noqa: N802
        return self._need().reduceProgress()

    def getCounters(self):  # noqa: N802
        return self._need().getCounters()

    def getJobID(self):  # noqa: N802
        return self._need().getID()

    def killJob(self):  # noqa: N802
        self._need().killJob()

    def getTaskReports(self, is_map=True):  # noqa: N802
        return self._need().getTaskReports(is_map)
