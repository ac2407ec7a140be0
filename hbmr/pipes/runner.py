"""Pipes map runners, reducer, partitioner and input format
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/pipes/{PipesMapRunner,
PipesGPUMapRunner,PipesReducer,PipesPartitioner,PipesNonJavaInputFormat}.java).

* :class:`PipesMapRunner`    – CPU attempt: runs ``hadoop.pipes.executable``;
* :class:`PipesGPUMapRunner` – GPU attempt: runs ``hadoop.pipes.gpu.executable``
  with the attempt's device id (argv[1] + HBMR_GPU_DEVICE);
* :class:`PipesReducer`      – one child per reduce task (CPU executable, or the
  GPU executable in CPU mode for GPU-only jobs — the reference crashed on those,
  SURVEY.md B3);
* :class:`PipesPartitioner`  – honours PARTITIONED_OUTPUT from the child, else
  delegates to the job's Java-side partitioner;
* :class:`PipesNonJavaInputFormat` – the child reads its split itself.
"""
from __future__ import annotations

import os
import threading

from ..mapred import counters as C
from ..mapred.api import InputFormat, MapRunnable, Partitioner, RecordReader, Reducer
from ..mapred.formats import FileSplit
from ..utils.reflection import load_class, new_instance
from .application import POOL, Application
from .protocol import frame_of_serialized, frame_parts_of_serialized

JAVA_RR = "hadoop.pipes.java.recordreader"
JAVA_MAPPER = "hadoop.pipes.java.mapper"
JAVA_REDUCER = "hadoop.pipes.java.reducer"
JAVA_RW = "hadoop.pipes.java.recordwriter"
JAVA_PARTITIONER = "hadoop.pipes.partitioner"
# keep Pipes children alive between tasks (hbmr/pipes/application.py ChildPool)
REUSE = "hbmr.pipes.child.reuse"
IDLE = "hbmr.pipes.child.idle.s"


def _work_dir(job, suffix):
    """The Pipes child's working directory (its cwd: core dumps land here; the
    task debug script looks for them, TaskTracker._run_debug_script).  Not the
    task's output work dir, whose contents are committed as job output."""
    import tempfile
    base = job.get("hbmr.local.scratch") or tempfile.gettempdir()
    d = os.path.join(base, f"_pipes_{job.get('mapred.task.id', 'task')}_{suffix}")
    os.makedirs(d, exist_ok=True)
    return d


def _split_bytes(reporter):
    sp = reporter.getInputSplit() if reporter is not None else None
    if sp is None:
        return b""
    return sp.serialize() if hasattr(sp, "serialize") else bytes(sp)


class PipesMapRunner(MapRunnable):
    run_on_gpu = False

    def configure(self, job):
        self.job = job

    def executable(self):
        return self.job.get_cpu_executable() or self.job.get_gpu_executable()

    def device(self):
        return -1

    def run(self, reader, output, reporter):
        job = self.job
        partitioner = None
        # the task's MapOutputBuffer owns a PipesPartitioner when the job uses one
        part = getattr(output, "partitioner", None)
        if isinstance(part, PipesPartitioner):
            partitioner = part
        from ..utils.trace import TRACE
        reuse = job.get_boolean(REUSE, False)
        key = (self.executable(), self.device(), "map")
        split = _split_bytes(reporter)
        # an idle child that already mapped this split (a GPU binary keeps it
        # resident in HBM) is preferred over the most recently idle one
        app = POOL.acquire(key, split) if reuse else None
        if TRACE.on:
            TRACE.instant("pipes.map.child", reused=app is not None)
        if app is not None:
            app.begin_task(job, output, reporter, job.get_map_output_key_class(),
                           job.get_map_output_value_class(), partitioner)
        else:
            app = Application(job, output, reporter, job.get_map_output_key_class(),
                              job.get_map_output_value_class(), self.executable(),
                              run_on_gpu=self.run_on_gpu, gpu_device_id=self.device(),
                              partitioner=partitioner, work_dir=_work_dir(job, "map"),
                              reuse=reuse)
        ok = False
        try:
            is_java_input = job.get_boolean(JAVA_RR, False)
            if is_java_input:
                kc, vc = None, None
                n = 0
                down = app.downlink
                first = reader.next()
                if first is not None:
                    kc, vc = type(first[0]), type(first[1])
                    down.set_input_types(kc.java_name(), vc.java_name())
                down.run_map(split, job.get_num_reduce_tasks(), True)
                kv = first
                while kv is not None:
                    down.map_item(kv[0], kv[1])
                    n += 1
                    if (n & 1023) == 0:
                        reporter.progress()
                    kv = reader.next()
                down.end_of_input()
                reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, n)
            else:
                app.downlink.run_map(split, job.get_num_reduce_tasks(), False)
                app.downlink.flush()
            app.wait_for_finish()
            ok = True
            if TRACE.on:
                TRACE.instant("pipes.map.done", records=app.handler.records)
        except BaseException:
            app.abort()
            raise
        finally:
            if ok and reuse:
                POOL.release(key, app, job.get_float(IDLE, 30.0), split=split)
            else:
                app.cleanup()


class PipesGPUMapRunner(PipesMapRunner):
    """GPU attempt: the GPU executable, told which device the scheduler chose.
    Child-read input (the common GPU shape: the binary loads its split) goes
    to the device's shared child with several maps in flight (hbmr/pipes/
    mux.py, ``hbmr.pipes.gpu.mux``); Java-fed input keeps a child per map."""
    run_on_gpu = True

    def executable(self):
        return self.job.get_gpu_executable()

    def device(self):
        return self.job.get_int("hbmr.task.gpu.device", 0)

    def run(self, reader, output, reporter):
        from . import mux
        job = self.job
        if job.get_boolean(JAVA_RR, False) or not job.get_boolean(mux.MUX, True):
            return super().run(reader, output, reporter)
        part = getattr(output, "partitioner", None)
        partitioner = part if isinstance(part, PipesPartitioner) else None
        pre = mux.PRELAUNCHED.pop(job.get("mapred.task.id"), None)
        if pre is not None:
            # sent to the child by the TaskTracker at launch: take over its
            # messages (those that came already are replayed here)
            child, t = pre
            from .application import OutputHandler
            h = OutputHandler(output, reporter, job.get_map_output_key_class(),
                              job.get_map_output_value_class(), partitioner)
            t.handler.attach(h)
            t.handler = h
            child.wait(t)
            return
        # (the work dir is made only when a child is started: one per child,
        # not a directory per map)
        child = mux.REGISTRY.get(job, self.executable(), self.device(),
                                 lambda: _work_dir(job, f"gpumux{self.device()}"),
                                 job.get_int(mux.DEPTH, 8))
        t = child.submit(job, output, reporter, job.get_map_output_key_class(),
                         job.get_map_output_value_class(), partitioner, _split_bytes(reporter),
                         job.get_num_reduce_tasks())
        child.wait(t)


class PipesReducer(Reducer):
    def configure(self, job):
        self.job = job
        self.app = None
        self.collector = None

    def _start(self, output, reporter):
        job = self.job
        exe = job.get_cpu_executable() or job.get_gpu_executable()
        self.reuse = job.get_boolean(REUSE, False)
        self.key = (exe, -1, "reduce")
        self.app = POOL.acquire(self.key) if self.reuse else None
        if self.app is not None:
            self.app.begin_task(job, output, reporter, job.get_output_key_class(),
                                job.get_output_value_class())
        else:
            self.app = Application(job, output, reporter, job.get_output_key_class(),
                                   job.get_output_value_class(), exe,
                                   work_dir=_work_dir(job, "reduce"), reuse=self.reuse)
        # piped output: the child's records come back up and the framework's
        # OutputFormat writes them; otherwise the child's own RecordWriter does
        piped_output = job.get_boolean(JAVA_RW, False)
        self.app.downlink.run_reduce(job.get_int("mapred.task.partition", 0), piped_output)

    def reduce(self, key, values, output, reporter):
        if self.app is None:
            self.reporter = reporter
            self._start(output, reporter)
        d = self.app.downlink
        d.reduce_key(key)
        for v in values:
            d.reduce_value(v)
        reporter.progress()

    def raw_reduce(self, key_class, value_class):
        """``reduce`` over serialised records (ReduceTask's native merge path):
        each key group goes down as one write of ready-made frames, no
        Writable built per value; None when a class's frame needs its object."""
        kf, vf = frame_of_serialized(key_class), frame_of_serialized(value_class)
        if kf is None or vf is None:
            return None
        vp = frame_parts_of_serialized(value_class)

        def reduce_raw(kb, vbs, output, reporter):
            if self.app is None:
                self.reporter = reporter
                self._start(output, reporter)
            d = self.app.downlink
            if vp is not None and sum(map(len, vbs)) >= (1 << 20):
                # large values (K-Means partials blocks): written in place
                d.reduce_group_parts(kf(kb), [vp(v) for v in vbs])
            else:
                d.reduce_group(kf(kb), [vf(v) for v in vbs])
            reporter.progress()
        return reduce_raw

    def close(self):
        if self.app is None:
            # no input: still let the child run setup/teardown
            self._start(_NullCollector(), None)
        ok = False
        try:
            self.app.downlink.end_of_input()
            self.app.wait_for_finish()
            ok = True
        except BaseException:
            self.app.abort()
            raise
        finally:
            if ok and self.reuse:
                POOL.release(self.key, self.app, self.job.get_float(IDLE, 30.0))
            else:
                self.app.cleanup()


class _NullCollector:
    def collect(self, k, v):
        pass


class PipesPartitioner(Partitioner):
    """Partition chosen by the child (PARTITIONED_OUTPUT) for the next collect, else
    the Java-side partitioner named by ``hadoop.pipes.partitioner``."""
    _tl = threading.local()

    def configure(self, job):
        self.delegate = new_instance(job.get(JAVA_PARTITIONER,
                                             "hbmr.mapred.lib.basic:HashPartitioner"), job)

    def set_next(self, part):
        PipesPartitioner._tl.part = part

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        p = getattr(PipesPartitioner._tl, "part", None)
        if p is not None:
            PipesPartitioner._tl.part = None
            return p
        return self.delegate.getPartition(key, value, num_partitions)


class _DummyReader(RecordReader):
    """Progress-only reader: the child reads the split itself."""

    def __init__(self, split):
        self.split = split
        self.done = False

    def next(self):
        if self.done:
            return None
        self.done = True
        return None

    def getProgress(self):  # noqa: N802
        return 1.0 if self.done else 0.0


class PipesNonJavaInputFormat(InputFormat):
    def getSplits(self, job, num_splits):  # noqa: N802
        inner = load_class(job.get("mapred.pipes.user.inputformat",
                                   "hbmr.mapred.formats:TextInputFormat"))()
        return inner.getSplits(job, num_splits)

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return _DummyReader(split)


_ = FileSplit
