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
        from .skipbadrecords import SkipLog, record_skip, skipping_limit
        m = self.mapper
        n = 0
        skip_max = skipping_limit(self.job, True)
        skipped = 0
        skiplog = None
        try:
            while True:
                kv = reader.next()
                if kv is None:
                    break
                n += 1
                if skip_max:
                    # skipping mode (SkipBadRecords): a record whose map() fails
                    # is logged and skipped instead of failing the attempt
                    try:
                        m.map(kv[0], kv[1], output, reporter)
                    except Exception:  # noqa: BLE001
                        skipped += 1
                        if skipped > skip_max:
                            raise
                        record_skip(reporter, True)
                        if skiplog is None:
                            skiplog = SkipLog(self.job, type(kv[0]), type(kv[1]))
                        skiplog.add(kv[0], kv[1])
                else:
                    m.map(kv[0], kv[1], output, reporter)
                if (n & 1023) == 0:
                    reporter.progress()
        finally:
            reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, n)
            if skiplog is not None:
                skiplog.close()
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
