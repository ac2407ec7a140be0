"""ChainMapper / ChainReducer (hadoop-1.0.3 mapred/lib/{ChainMapper,ChainReducer,
Chain}.java): several mappers (and a reducer followed by mappers) run inside one
task, each one's output feeding the next's map() — no intermediate files.

Per-link configuration overrides are stored as ``chain.mapper.<i>.conf.<key>``
(``chain.reducer.mapper.<i>...`` after the reducer); each link sees the job
conf with its overrides applied.
"""
from __future__ import annotations

from ...utils.reflection import class_name, new_instance
from ..api import Mapper, OutputCollector, Reducer

_MAP = "chain.mapper"
_RMAP = "chain.reducer.mapper"
_RED = "chain.reducer.class"


def _add(job, prefix, klass, conf_overrides):
    n = job.get_int(f"{prefix}.size", 0)
    job.set(f"{prefix}.{n}.class", class_name(klass))
    for k, v in (conf_overrides or {}).items():
        job.set(f"{prefix}.{n}.conf.{k}", str(v))
    job.set_int(f"{prefix}.size", n + 1)


def _link_conf(job, prefix, i):
    from ..jobconf import JobConf
    c = JobConf(job)
    pre = f"{prefix}.{i}.conf."
    for k, v in job.to_dict().items():
        if k.startswith(pre):
            c.set(k[len(pre):], v)
    return c


def _build(job, prefix):
    out = []
    for i in range(job.get_int(f"{prefix}.size", 0)):
        c = _link_conf(job, prefix, i)
        out.append(new_instance(job.get_class(f"{prefix}.{i}.class"), c))
    return out


class _Link(OutputCollector):
    def __init__(self, mapper, nxt, reporter):
        self.mapper, self.nxt, self.rep = mapper, nxt, reporter

    def collect(self, key, value):
        self.mapper.map(key, value, self.nxt, self.rep)


def _chain(mappers, final, reporter):
    out = final
    for m in reversed(mappers):
        out = _Link(m, out, reporter)
    return out


class ChainMapper(Mapper):
    @staticmethod
    def addMapper(job, klass, in_key=None, in_val=None, out_key=None, out_val=None,  # noqa: N802
                  by_value=True, mapper_conf=None):
        job.set_mapper_class(ChainMapper)
        _add(job, _MAP, klass, mapper_conf)
        if out_key is not None:
            job.set_map_output_key_class(out_key)
        if out_val is not None:
            job.set_map_output_value_class(out_val)

    def configure(self, job):
        self.mappers = _build(job, _MAP)

    def map(self, key, value, output, reporter):
        if not self.mappers:
            output.collect(key, value)
            return
        head = self.mappers[0]
        head.map(key, value, _chain(self.mappers[1:], output, reporter), reporter)

    def close(self):
        for m in self.mappers:
            m.close()


class ChainReducer(Reducer):
    @staticmethod
    def setReducer(job, klass, in_key=None, in_val=None, out_key=None, out_val=None,  # noqa: N802
                   by_value=True, reducer_conf=None):
        job.set_reducer_class(ChainReducer)
        job.set(_RED, class_name(klass))
        for k, v in (reducer_conf or {}).items():
            job.set(f"{_RED}.conf.{k}", str(v))
        if out_key is not None:
            job.set_output_key_class(out_key)
        if out_val is not None:
            job.set_output_value_class(out_val)

    @staticmethod
    def addMapper(job, klass, in_key=None, in_val=None, out_key=None, out_val=None,  # noqa: N802
                  by_value=True, mapper_conf=None):
        _add(job, _RMAP, klass, mapper_conf)
        if out_key is not None:
            job.set_output_key_class(out_key)
        if out_val is not None:
            job.set_output_value_class(out_val)

    def configure(self, job):
        from ..jobconf import JobConf
        c = JobConf(job)
        pre = f"{_RED}.conf."
        for k, v in job.to_dict().items():
            if k.startswith(pre):
                c.set(k[len(pre):], v)
        self.reducer = new_instance(job.get_class(_RED), c)
        self.mappers = _build(job, _RMAP)

    def reduce(self, key, values, output, reporter):
        self.reducer.reduce(key, values, _chain(self.mappers, output, reporter), reporter)

    def close(self):
        self.reducer.close()
        for m in self.mappers:
            m.close()
