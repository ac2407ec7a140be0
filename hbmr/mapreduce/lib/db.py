"""New-API database formats (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapreduce/lib/db/):
DBInputFormat, DataDrivenDBInputFormat (+ its splitters) and DBOutputFormat
over the same ``mapred.jdbc.*`` keys and DB-API connection as
:mod:`hbmr.mapred.lib.db` (JDBC → Python DB-API; ``sqlite3`` built in)."""
from __future__ import annotations

from ...mapred.lib import db as _db
from ...utils.reflection import class_name
from .. import api
from ..adapters import OldWriterAsNew
from .input import _OldFormatReader

DBConfiguration = _db.DBConfiguration
DBWritable = _db.DBWritable
DBInputSplit = _db.DBInputSplit


def _conf(job):
    return job.getConfiguration() if hasattr(job, "getConfiguration") else job


def _keep_adapter(conf, fn):
    """Run an old-API ``set_input`` without letting it replace the job's
    new-API input adapter in ``mapred.input.format.class``."""
    prev = conf.get("mapred.input.format.class")
    fn()
    if prev is not None:
        conf.set("mapred.input.format.class", prev)


class DBInputFormat(api.InputFormat):
    """LIMIT/OFFSET splits of an ordered table or query (DBInputFormat.java)."""
    _old = _db.DBInputFormat

    @classmethod
    def setInput(cls, job, input_class, table_or_query, conditions_or_count=None,  # noqa: N802
                 order_by=None, *fields):
        """``setInput(job, cls, table, conditions, orderBy, *fields)`` or
        ``setInput(job, cls, inputQuery, inputCountQuery)`` (the two Java
        overloads: a query is told apart by its SELECT)."""
        conf = _conf(job)
        if table_or_query.lstrip().upper().startswith("SELECT"):
            _keep_adapter(conf, lambda: _db.DBInputFormat.set_input(
                conf, input_class, query=table_or_query, count_query=conditions_or_count))
        else:
            _keep_adapter(conf, lambda: _db.DBInputFormat.set_input(
                conf, input_class, table=table_or_query, conditions=conditions_or_count,
                order_by=order_by, fields=list(fields)))
        conf.set("mapreduce.inputformat.class", class_name(cls))

    def getSplits(self, context):  # noqa: N802
        conf = _conf(context)
        return self._old().getSplits(conf, conf.get_num_map_tasks())

    def createRecordReader(self, split, context):  # noqa: N802
        return _OldFormatReader(self._old())


class DataDrivenDBInputFormat(DBInputFormat):
    """WHERE-range splits over the split-by column's bounds
    (DataDrivenDBInputFormat.java): ``setInput(job, cls, table, conditions,
    splitBy, *fields)`` or ``setInput(job, cls, inputQuery, boundingQuery)``
    (the query must contain ``$CONDITIONS``)."""
    _old = _db.DataDrivenDBInputFormat

    @classmethod
    def setInput(cls, job, input_class, table_or_query, conditions_or_bounding=None,  # noqa: N802
                 split_by=None, *fields):
        conf = _conf(job)
        if table_or_query.lstrip().upper().startswith("SELECT"):
            _keep_adapter(conf, lambda: _db.DBInputFormat.set_input(
                conf, input_class, query=table_or_query))
            if conditions_or_bounding:
                conf.set(_db.INPUT_BOUNDING_QUERY, conditions_or_bounding)
        else:
            _keep_adapter(conf, lambda: _db.DBInputFormat.set_input(
                conf, input_class, table=table_or_query, conditions=conditions_or_bounding,
                order_by=split_by, fields=list(fields)))
        conf.set("mapreduce.inputformat.class", class_name(cls))


class DBOutputFormat(api.OutputFormat):
    """Batched INSERTs of the output keys (DBWritable), committed on close."""

    @staticmethod
    def setOutput(job, table, *fields):  # noqa: N802
        conf = _conf(job)
        conf.set(_db.OUTPUT_TABLE, table)
        conf.set_strings(_db.OUTPUT_FIELDS, list(fields))
        conf.set("mapreduce.outputformat.class", class_name(DBOutputFormat))

    def checkOutputSpecs(self, context):  # noqa: N802
        _db.DBOutputFormat().checkOutputSpecs(None, _conf(context))

    def getRecordWriter(self, context):  # noqa: N802
        return OldWriterAsNew(_db.DBRecordWriter(_conf(context)), getattr(context, "reporter", None))


# -- DBSplitter family (DBSplitter.java and its subclasses) -------------------------
class DBSplitter:
    """``split(conf, lo, hi, col) -> [DBInputSplit]`` over [lo, hi]."""

    def points(self, lo, hi, n):
        raise NotImplementedError

    def split(self, conf, lo, hi, col):
        n = max(1, _conf(conf).get_int("mapred.map.tasks", 1))
        pts = self.points(lo, hi, n)
        out = []
        for i, (a, b) in enumerate(zip(pts, pts[1:])):
            op = "<=" if i == len(pts) - 2 else "<"
            out.append(DBInputSplit(0, 0, f"{col} >= {{ph}} AND {col} {op} {{ph}}", (a, b)))
        return out or [DBInputSplit(0, 0, f"{col} = {{ph}}", (pts[0],))]


class IntegerSplitter(DBSplitter):
    def points(self, lo, hi, n):
        return _db._split_points(int(lo), int(hi), n)


class FloatSplitter(DBSplitter):
    def points(self, lo, hi, n):
        return _db._split_points(float(lo), float(hi), n)


class BigDecimalSplitter(FloatSplitter):
    pass


class TextSplitter(DBSplitter):
    def points(self, lo, hi, n):
        return _db._text_points(str(lo), str(hi), n)


class BooleanSplitter(DBSplitter):
    def points(self, lo, hi, n):
        return [False, True] if lo != hi else [bool(lo)]
