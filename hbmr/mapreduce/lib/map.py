"""New-API library mappers (mapreduce/lib/map/*.java)."""
from __future__ import annotations

import concurrent.futures as cf
import threading

from ...io.writable import IntWritable, Text
from ...utils.reflection import new_instance
from .. import api


class TokenCounterMapper(api.Mapper):
    """(token, 1) per whitespace-separated token of the value."""

    def map(self, key, value, context):
        one = IntWritable(1)
        for tok in str(value).split():
            context.write(Text(tok), one)


class InverseMapper(api.Mapper):
    def map(self, key, value, context):
        context.write(value, key)


class MultithreadedMapper(api.Mapper):
    """Runs ``mapreduce.mapper.multithreadedmapper.mapclass`` in
    ``mapreduce.mapper.multithreadedmapper.threads`` threads sharing the input
    (useful for mappers that release the GIL: native calls, I/O)."""

    CLASS_KEY = "mapreduce.mapper.multithreadedmapper.mapclass"
    THREADS_KEY = "mapreduce.mapper.multithreadedmapper.threads"

    @staticmethod
    def setMapperClass(job, cls):  # noqa: N802
        from ...utils.reflection import class_name
        job.getConfiguration().set(MultithreadedMapper.CLASS_KEY, class_name(cls))

    @staticmethod
    def setNumberOfThreads(job, n):  # noqa: N802
        job.getConfiguration().set_int(MultithreadedMapper.THREADS_KEY, n)

    def run(self, context):
        conf = context.getConfiguration()
        cls = conf.get_class(self.CLASS_KEY, "hbmr.mapreduce.api:Mapper")
        n = conf.get_int(self.THREADS_KEY, 10)
        lock = threading.Lock()

        class _Sub(api.MapContext):
            def nextKeyValue(self_inner):  # noqa: N805
                with lock:
                    ok = context.nextKeyValue()
                    self_inner._kv = (context.getCurrentKey(), context.getCurrentValue()) \
                        if ok else None
                return ok

            def write(self_inner, k, v):  # noqa: N805
                with lock:
                    context.write(k, v)

        def one():
            sub = _Sub(conf, context.getTaskAttemptID(), context.reporter, None, None,
                       context.getInputSplit())
            new_instance(cls, conf).run(sub)

        with cf.ThreadPoolExecutor(n) as ex:
            for f in [ex.submit(one) for _ in range(n)]:
                f.result()
