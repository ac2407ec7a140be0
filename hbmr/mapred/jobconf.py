"""JobConf: the job description (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/JobConf.java).

Adds the MapReduce defaults (mapred-default.xml / mapred-site.xml) on top of
:class:`hbmr.conf.Configuration` and typed accessors for every job property the
runtime reads.  GPU additions from the fork:

* ``get/setGPUMapRunnerClass`` (JobConf.java:974-1002) — one key, typo accepted;
* ``set/getGPUExecutable`` / ``set/getCPUExecutable`` (pipes Submitter.java:83-120);
* ``setNumGPUMapSlots``-style tracker keys live on the tracker conf.
"""
from __future__ import annotations

import getpass
import os

from ..conf.configuration import Configuration
from ..utils.reflection import class_name, load_class

Configuration.add_default_resource("mapred-default.xml")
Configuration.add_default_resource("mapred-site.xml")


_USER = None


def _login_user():
    global _USER
    if _USER is None:
        try:
            _USER = getpass.getuser()
        except Exception:  # noqa: BLE001
            _USER = "unknown"
    return _USER


class JobConf(Configuration):
    def __init__(self, conf=None, job_class=None):
        if isinstance(conf, Configuration):
            super().__init__(conf)
        else:
            super().__init__()
        if job_class is not None:
            self.set("mapred.job.class", class_name(job_class))

    # -- identity --------------------------------------------------------------
    def get_job_name(self):
        return self.get("mapred.job.name", "")

    def set_job_name(self, name):
        self.set("mapred.job.name", name)

    getJobName, setJobName = get_job_name, set_job_name  # noqa: N815

    def get_user(self):
        return self.get("user.name") or os.environ.get("USER") or _login_user()

    def set_user(self, u):
        self.set("user.name", u)

    getUser, setUser = get_user, set_user  # noqa: N815

    def get_queue_name(self):
        return self.get("mapred.job.queue.name", "default")

    def set_queue_name(self, q):
        self.set("mapred.job.queue.name", q)

    # -- classes ---------------------------------------------------------------
    def _cls(self, key, default):
        return self.get_class(key, default)

    def get_mapper_class(self):
        return self._cls("mapred.mapper.class", "hbmr.mapred.lib.basic:IdentityMapper")

    def set_mapper_class(self, c):
        self.set_class("mapred.mapper.class", c)

    def get_reducer_class(self):
        return self._cls("mapred.reducer.class", "hbmr.mapred.lib.basic:IdentityReducer")

    def set_reducer_class(self, c):
        self.set_class("mapred.reducer.class", c)

    def get_combiner_class(self):
        return self._cls("mapred.combiner.class", None)

    def set_combiner_class(self, c):
        self.set_class("mapred.combiner.class", c)

    def get_partitioner_class(self):
        return self._cls("mapred.partitioner.class", "hbmr.mapred.lib.basic:HashPartitioner")

    def set_partitioner_class(self, c):
        self.set_class("mapred.partitioner.class", c)

    def get_map_runner_class(self):
        return self._cls("mapred.map.runner.class", "hbmr.mapred.maprunner:MapRunner")

    def set_map_runner_class(self, c):
        self.set_class("mapred.map.runner.class", c)

    def get_gpu_map_runner_class(self):
        """GPU map runner (JobConf.getGPUMapRunnerClass). Reads the canonical key;
        the reference's misspelled getter key is aliased to it."""
        return self._cls("mapred.map.runner.gpu.class", "hbmr.pipes.runner:PipesGPUMapRunner")

    def set_gpu_map_runner_class(self, c):
        self.set_class("mapred.map.runner.gpu.class", c)

    def get_input_format(self):
        return self._cls("mapred.input.format.class", "hbmr.mapred.formats:TextInputFormat")

    def set_input_format(self, c):
        self.set_class("mapred.input.format.class", c)

    def get_output_format(self):
        return self._cls("mapred.output.format.class", "hbmr.mapred.formats:TextOutputFormat")

    def set_output_format(self, c):
        self.set_class("mapred.output.format.class", c)

    def get_output_committer(self):
        return self._cls("mapred.output.committer.class",
                         "hbmr.mapred.committer:FileOutputCommitter")

    def set_output_committer(self, c):
        self.set_class("mapred.output.committer.class", c)

    # key/value types
    def get_output_key_class(self):
        return self._cls("mapred.output.key.class", "hbmr.io.writable:LongWritable")

    def set_output_key_class(self, c):
        self.set_class("mapred.output.key.class", c)

    def get_output_value_class(self):
        return self._cls("mapred.output.value.class", "hbmr.io.writable:Text")

    def set_output_value_class(self, c):
        self.set_class("mapred.output.value.class", c)

    def get_map_output_key_class(self):
        """Writable class, or a serializer adapter for plain types (io.serializations)."""
        from ..io.serializer import adapter_for
        c = self._cls("mapred.mapoutput.key.class", None)
        return adapter_for(c if c is not None else self.get_output_key_class(), self)

    def set_map_output_key_class(self, c):
        self.set_class("mapred.mapoutput.key.class", c)

    def get_map_output_value_class(self):
        from ..io.serializer import adapter_for
        c = self._cls("mapred.mapoutput.value.class", None)
        return adapter_for(c if c is not None else self.get_output_value_class(), self)

    def set_map_output_value_class(self, c):
        self.set_class("mapred.mapoutput.value.class", c)

    def get_output_key_comparator(self):
        """Returns a sort-key function over serialised map-output keys."""
        c = self._cls("mapred.output.key.comparator.class", None)
        if c is not None:
            from ..utils.reflection import new_instance
            return new_instance(c, self).sort_key if isinstance(c, type) else c
        return self.get_map_output_key_class().raw_sort_key

    def set_output_key_comparator_class(self, c):
        self.set_class("mapred.output.key.comparator.class", c)

    def get_output_value_grouping_comparator(self):
        c = self._cls("mapred.output.value.groupfn.class", None)
        if c is not None:
            from ..utils.reflection import new_instance
            return new_instance(c, self).sort_key if isinstance(c, type) else c
        return self.get_output_key_comparator()

    def set_output_value_grouping_comparator(self, c):
        self.set_class("mapred.output.value.groupfn.class", c)

    # -- counts ------------------------------------------------------------------
    def get_num_map_tasks(self):
        return self.get_int("mapred.map.tasks", 1)

    def set_num_map_tasks(self, n):
        self.set_int("mapred.map.tasks", n)

    def get_num_reduce_tasks(self):
        return self.get_int("mapred.reduce.tasks", 1)

    def set_num_reduce_tasks(self, n):
        self.set_int("mapred.reduce.tasks", n)

    def get_max_map_attempts(self):
        return self.get_int("mapred.map.max.attempts", 4)

    def set_max_map_attempts(self, n):
        self.set_int("mapred.map.max.attempts", n)

    def get_max_reduce_attempts(self):
        return self.get_int("mapred.reduce.max.attempts", 4)

    def set_max_reduce_attempts(self, n):
        self.set_int("mapred.reduce.max.attempts", n)

    def get_map_speculative_execution(self):
        return self.get_boolean("mapred.map.tasks.speculative.execution", True)

    def set_map_speculative_execution(self, b):
        self.set_boolean("mapred.map.tasks.speculative.execution", b)

    def get_reduce_speculative_execution(self):
        return self.get_boolean("mapred.reduce.tasks.speculative.execution", True)

    def set_reduce_speculative_execution(self, b):
        self.set_boolean("mapred.reduce.tasks.speculative.execution", b)

    def set_speculative_execution(self, b):
        self.set_map_speculative_execution(b)
        self.set_reduce_speculative_execution(b)

    def get_max_task_failures_per_tracker(self):
        return self.get_int("mapred.max.tracker.failures", 4)

    def get_compress_map_output(self):
        return self.get_boolean("mapred.compress.map.output", False)

    def set_compress_map_output(self, b):
        self.set_boolean("mapred.compress.map.output", b)

    def get_working_directory(self):
        return self.get("mapred.working.dir") or os.getcwd()

    def set_working_directory(self, d):
        self.set("mapred.working.dir", str(d))

    # -- pipes / GPU executables (Submitter.java:83-120, 329-379) -------------------
    def get_cpu_executable(self):
        return self.get("hadoop.pipes.executable")

    def set_cpu_executable(self, path):
        self.set("hadoop.pipes.executable", str(path))

    def get_gpu_executable(self):
        return self.get("hadoop.pipes.gpu.executable")

    def set_gpu_executable(self, path):
        self.set("hadoop.pipes.gpu.executable", str(path))

    def is_gpu_capable(self) -> bool:
        """A job can use GPU slots if it names a GPU executable or an in-process
        GPU mapper (hbmr's split-level GpuMapper interface)."""
        return bool(self.get_gpu_executable()) or self.get("hbmr.gpu.mapper.class") is not None

    def get_gpu_mapper_class(self):
        return self._cls("hbmr.gpu.mapper.class", None)

    def set_gpu_mapper_class(self, c):
        self.set_class("hbmr.gpu.mapper.class", c)

    # -- profiling (JobConf.java:1482-1541) ------------------------------------------
    def get_profile_enabled(self):
        return self.get_boolean("mapred.task.profile", False)

    def set_profile_enabled(self, b):
        self.set_boolean("mapred.task.profile", b)

    def get_profile_task_range(self, is_map: bool):
        return self.get("mapred.task.profile.maps" if is_map else "mapred.task.profile.reduces",
                        "0-2")

    # camelCase aliases used by ported code
    getMapperClass, setMapperClass = get_mapper_class, set_mapper_class  # noqa: N815
    getReducerClass, setReducerClass = get_reducer_class, set_reducer_class  # noqa: N815
    getCombinerClass, setCombinerClass = get_combiner_class, set_combiner_class  # noqa: N815
    getPartitionerClass, setPartitionerClass = get_partitioner_class, set_partitioner_class  # noqa: N815
    getMapRunnerClass, setMapRunnerClass = get_map_runner_class, set_map_runner_class  # noqa: N815
    getGPUMapRunnerClass, setGPUMapRunnerClass = get_gpu_map_runner_class, set_gpu_map_runner_class  # noqa: N815
    getInputFormat, setInputFormat = get_input_format, set_input_format  # noqa: N815
    getOutputFormat, setOutputFormat = get_output_format, set_output_format  # noqa: N815
    getOutputKeyClass, setOutputKeyClass = get_output_key_class, set_output_key_class  # noqa: N815
    getOutputValueClass, setOutputValueClass = get_output_value_class, set_output_value_class  # noqa: N815
    getMapOutputKeyClass, setMapOutputKeyClass = get_map_output_key_class, set_map_output_key_class  # noqa: N815
    getMapOutputValueClass, setMapOutputValueClass = get_map_output_value_class, set_map_output_value_class  # noqa: N815
    setOutputKeyComparatorClass = set_output_key_comparator_class  # noqa: N815
    setOutputValueGroupingComparator = set_output_value_grouping_comparator  # noqa: N815
    getNumMapTasks, setNumMapTasks = get_num_map_tasks, set_num_map_tasks  # noqa: N815
    getNumReduceTasks, setNumReduceTasks = get_num_reduce_tasks, set_num_reduce_tasks  # noqa: N815
    getMaxMapAttempts, setMaxMapAttempts = get_max_map_attempts, set_max_map_attempts  # noqa: N815
    setSpeculativeExecution = set_speculative_execution  # noqa: N815
    setMapSpeculativeExecution = set_map_speculative_execution  # noqa: N815
    setReduceSpeculativeExecution = set_reduce_speculative_execution  # noqa: N815
    setCompressMapOutput = set_compress_map_output  # noqa: N815
    getGPUExecutable, setGPUExecutable = get_gpu_executable, set_gpu_executable  # noqa: N815
    getCPUExecutable, setCPUExecutable = get_cpu_executable, set_cpu_executable  # noqa: N815


def as_jobconf(conf) -> JobConf:
    return conf if isinstance(conf, JobConf) else JobConf(conf)


def load_cls(name):
    return load_class(name)
