"""Map runners (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/MapRunner.java,
lib/MultithreadedMapRunner.java): drive a Mapper over a RecordReader."""
from __future__ import annotations

import concurrent.futures as cf
import threading

from ..utils.reflection import new_instance
from . import counters as C
from .api import MapRunnable


class MapRunner(MapRunnable):
    def configure(self, job):
        self.job = job
        self.mapper = new_instance(job.get_mapper_class(), job)

    def run(self, reader, output, reporter):
        m = self.mapper
        n = 0
        try:
            while True:
                kv = reader.next()
                if kv is None:
                    break
                n += 1
                m.map(kv[0], kv[1], output, reporter)
                if (n & 1023) == 0:
                    reporter.progress()
        finally:
            reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, n)
            m.close()


class MultithreadedMapRunner(MapRunnable):
    """Runs ``mapred.map.multithreadedrunner.threads`` mapper calls concurrently
    (useful when map() releases the GIL, e.g. native or I/O-bound mappers)."""

    def configure(self, job):
        self.job = job
        self.threads = job.get_int("mapred.map.multithreadedrunner.threads", 10)
        self.mapper = new_instance(job.get_mapper_class(), job)

    def run(self, reader, output, reporter):
        lock = threading.Lock()

        class _SyncOut:
            def collect(self_inner, k, v):
                with lock:
                    output.collect(k, v)

        out = _SyncOut()
        n = 0
        with cf.ThreadPoolExecutor(self.threads) as ex:
            futs = []
            while True:
                kv = reader.next()
                if kv is None:
                    break
                n += 1
                futs.append(ex.submit(self.mapper.map, kv[0], kv[1], out, reporter))
                if len(futs) > 4 * self.threads:
                    for f in futs:
                        f.result()
                    futs = []
            for f in futs:
                f.result()
        reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, n)
        self.mapper.close()
