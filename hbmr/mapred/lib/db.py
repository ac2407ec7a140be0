"""Database input/output formats (mapred.lib.db and mapreduce.lib.db).

Behaviour from hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/lib/db/
(DBConfiguration keys ``mapred.jdbc.*``, DBInputFormat with LIMIT/OFFSET
splits over an ORDER BY, DBRecordReader yielding (LongWritable row index,
DBWritable), DBOutputFormat batching ``INSERT INTO t (f…) VALUES (?…)`` and
committing on close) and mapreduce/lib/db/DataDrivenDBInputFormat.java with
its IntegerSplitter/FloatSplitter/TextSplitter (splits are WHERE ranges over
``mapred.jdbc.input.bounding.query`` / the split-by column's MIN/MAX).

JDBC becomes Python DB-API 2.0: ``mapred.jdbc.driver.class`` names the DB-API
module (``sqlite3`` is built in) and ``mapred.jdbc.url`` is its connect
argument; ``DBWritable`` is ``read_fields(row_tuple)`` /
``write_fields() -> tuple``.
"""
from __future__ import annotations

import importlib
import json

from ...io.writable import LongWritable
from ...utils.reflection import class_name, load_class
from ..api import InputFormat, InputSplit, OutputFormat, RecordReader, RecordWriter

DRIVER_CLASS = "mapred.jdbc.driver.class"
URL = "mapred.jdbc.url"
USERNAME = "mapred.jdbc.username"
PASSWORD = "mapred.jdbc.password"
INPUT_TABLE = "mapred.jdbc.input.table.name"
INPUT_FIELDS = "mapred.jdbc.input.field.names"
INPUT_CONDITIONS = "mapred.jdbc.input.conditions"
INPUT_ORDER_BY = "mapred.jdbc.input.orderby"
INPUT_QUERY = "mapred.jdbc.input.query"
INPUT_COUNT_QUERY = "mapred.jdbc.input.count.query"
INPUT_BOUNDING_QUERY = "mapred.jdbc.input.bounding.query"
INPUT_CLASS = "mapred.jdbc.input.class"
OUTPUT_TABLE = "mapred.jdbc.output.table.name"
OUTPUT_FIELDS = "mapred.jdbc.output.field.names"


class DBWritable:
    """Row ↔ object mapping (DBWritable.java: readFields(ResultSet) / write(PreparedStatement))."""

    def read_fields(self, row: tuple) -> None:
        raise NotImplementedError

    def write_fields(self) -> tuple:
        raise NotImplementedError

    readFields = read_fields  # noqa: N815


class DBConfiguration:
    @staticmethod
    def configure_db(job, driver="sqlite3", url=":memory:", user=None, password=None):
        job.set(DRIVER_CLASS, driver)
        job.set(URL, url)
        if user is not None:
            job.set(USERNAME, user)
        if password is not None:
            job.set(PASSWORD, password)

    configureDB = configure_db  # noqa: N815

    @staticmethod
    def connect(job):
        mod = importlib.import_module(job.get(DRIVER_CLASS, "sqlite3"))
        url = job.get(URL)
        user, pw = job.get(USERNAME), job.get(PASSWORD)
        if user is not None:
            return mod.connect(url, user=user, password=pw)
        return mod.connect(url)


def _ph(job):
    mod = importlib.import_module(job.get(DRIVER_CLASS, "sqlite3"))
    return "%s" if getattr(mod, "paramstyle", "qmark") in ("format", "pyformat") else "?"


# ---------------------------------------------------------------- DBInputFormat
class DBInputSplit(InputSplit):
    """Rows [start, end) of the ordered query (DBInputFormat.DBInputSplit)."""

    def __init__(self, start=0, end=0, where=None, params=()):
        self.start, self.end, self.where, self.params = start, end, where, tuple(params)

    def getLength(self):  # noqa: N802
        return self.end - self.start

    def getLocations(self):  # noqa: N802
        return []

    def serialize(self) -> bytes:
        return json.dumps([self.start, self.end, self.where, list(self.params)]).encode()

    @classmethod
    def deserialize(cls, raw):
        s, e, w, p = json.loads(raw)
        return cls(s, e, w, p)


class DBRecordReader(RecordReader):
    def __init__(self, split, job, select, params=()):
        self.split, self.job = split, job
        self.cls = load_class(job.get(INPUT_CLASS))
        self.conn = DBConfiguration.connect(job)
        self.cur = self.conn.cursor()
        self.cur.execute(select, params)
        self.pos = 0

    def next(self):
        row = self.cur.fetchone()
        if row is None:
            return None
        obj = self.cls()
        obj.read_fields(tuple(row))
        key = LongWritable(self.split.start + self.pos)
        self.pos += 1
        return key, obj

    def getPos(self):  # noqa: N802
        return self.pos

    def getProgress(self):  # noqa: N802
        return self.pos / max(1, self.split.getLength())

    def close(self):
        self.cur.close()
        self.conn.close()


class DBInputFormat(InputFormat):
    @staticmethod
    def set_input(job, input_class, table=None, conditions=None, order_by=None, fields=None,
                  query=None, count_query=None):
        from ..formats import FileInputFormat  # noqa: F401 (keep the old-API import surface)
        job.set_input_format(DBInputFormat)
        job.set(INPUT_CLASS, class_name(input_class))
        if query is not None:
            job.set(INPUT_QUERY, query)
            if count_query is not None:
                job.set(INPUT_COUNT_QUERY, count_query)
            return
        job.set(INPUT_TABLE, table)
        job.set_strings(INPUT_FIELDS, list(fields or []))
        if conditions:
            job.set(INPUT_CONDITIONS, conditions)
        if order_by:
            job.set(INPUT_ORDER_BY, order_by)

    setInput = set_input  # noqa: N815

    def _base_query(self, job):
        q = job.get(INPUT_QUERY)
        if q:
            return q
        fields = ", ".join(job.get_strings(INPUT_FIELDS) or ["*"])
        q = f"SELECT {fields} FROM {job.get(INPUT_TABLE)}"
        if job.get(INPUT_CONDITIONS):
            q += f" WHERE ({job.get(INPUT_CONDITIONS)})"
        if job.get(INPUT_ORDER_BY):
            q += f" ORDER BY {job.get(INPUT_ORDER_BY)}"
        return q

    def _count(self, job):
        q = job.get(INPUT_COUNT_QUERY)
        if not q:
            if job.get(INPUT_QUERY):
                q = f"SELECT COUNT(*) FROM ({job.get(INPUT_QUERY)}) AS hbmr_cnt"
            else:
                q = f"SELECT COUNT(*) FROM {job.get(INPUT_TABLE)}"
                if job.get(INPUT_CONDITIONS):
                    q += f" WHERE {job.get(INPUT_CONDITIONS)}"
        conn = DBConfiguration.connect(job)
        try:
            cur = conn.cursor()
            cur.execute(q)
            return int(cur.fetchone()[0])
        finally:
            conn.close()

    def getSplits(self, job, num_splits):  # noqa: N802
        n = self._count(job)
        chunks = max(1, num_splits)
        size = n // chunks
        out = []
        for i in range(chunks):
            start = i * size
            end = n if i == chunks - 1 else start + size
            out.append(DBInputSplit(start, end))
        return out

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        q = f"{self._base_query(job)} LIMIT {split.end - split.start} OFFSET {split.start}"
        return DBRecordReader(split, job, q)


# ------------------------------------------------------- DataDrivenDBInputFormat
def _split_points(lo, hi, n):
    """IntegerSplitter / FloatSplitter: n+1 boundaries covering [lo, hi]."""
    if isinstance(lo, int) and isinstance(hi, int):
        step = max(1, (hi - lo) // n) if hi > lo else 1
        pts = list(range(lo, hi, step))
        if not pts or pts[-1] != hi:
            pts.append(hi)
        return pts
    lo, hi = float(lo), float(hi)
    if hi <= lo:
        return [lo, hi]
    return [lo + (hi - lo) * i / n for i in range(n)] + [hi]


def _text_points(lo: str, hi: str, n):
    """TextSplitter: split the string range as base-65536 fractions of the common prefix."""
    p = 0
    while p < min(len(lo), len(hi)) and lo[p] == hi[p]:
        p += 1
    prefix = lo[:p]

    def to_num(s):
        v = 0.0
        for i, ch in enumerate(s[:8]):
            v += ord(ch) / 65536.0 ** (i + 1)
        return v

    def to_str(v):
        out = []
        for _ in range(8):
            v *= 65536.0
            c = int(v)
            out.append(chr(c))
            v -= c
            if v <= 0:
                break
        return "".join(out).rstrip("\0")

    a, b = to_num(lo[p:]), to_num(hi[p:])
    mids = [prefix + to_str(a + (b - a) * i / n) for i in range(1, n)]
    return [lo] + sorted(set(m for m in mids if lo < m < hi)) + [hi]


class DataDrivenDBInputFormat(DBInputFormat):
    SPLIT_BY = "mapred.jdbc.input.split.by"   # hbmr key (the reference takes the ORDER BY column)

    def getSplits(self, job, num_splits):  # noqa: N802
        col = job.get(self.SPLIT_BY) or job.get(INPUT_ORDER_BY)
        q = job.get(INPUT_BOUNDING_QUERY) or \
            f"SELECT MIN({col}), MAX({col}) FROM {job.get(INPUT_TABLE)}" + \
            (f" WHERE ({job.get(INPUT_CONDITIONS)})" if job.get(INPUT_CONDITIONS) else "")
        conn = DBConfiguration.connect(job)
        try:
            cur = conn.cursor()
            cur.execute(q)
            lo, hi = cur.fetchone()
        finally:
            conn.close()
        if lo is None:
            return [DBInputSplit(0, 0, f"{col} IS NULL")]
        n = max(1, num_splits)
        pts = _text_points(lo, hi, n) if isinstance(lo, str) else _split_points(lo, hi, n)
        out = []
        for i, (a, b) in enumerate(zip(pts, pts[1:])):
            last = i == len(pts) - 2
            where = f"{col} >= {{ph}} AND {col} {'<=' if last else '<'} {{ph}}"
            out.append(DBInputSplit(0, 0, where, (a, b)))
        if len(pts) == 1:
            out.append(DBInputSplit(0, 0, f"{col} = {{ph}}", (pts[0],)))
        return out

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        if job.get(INPUT_QUERY):
            # a free-form query carries the split's range at ``$CONDITIONS``
            # (DataDrivenDBRecordReader.getSelectQuery)
            q = job.get(INPUT_QUERY).replace("$CONDITIONS",
                                             f"( {split.where.format(ph=_ph(job))} )")
            return DBRecordReader(split, job, q, split.params)
        fields = ", ".join(job.get_strings(INPUT_FIELDS) or ["*"])
        conds = [split.where.format(ph=_ph(job))]
        if job.get(INPUT_CONDITIONS):
            conds.append(f"({job.get(INPUT_CONDITIONS)})")
        q = f"SELECT {fields} FROM {job.get(INPUT_TABLE)} WHERE {' AND '.join(conds)}"
        if job.get(INPUT_ORDER_BY):
            q += f" ORDER BY {job.get(INPUT_ORDER_BY)}"
        return DBRecordReader(split, job, q, split.params)


# ---------------------------------------------------------------- DBOutputFormat
class DBRecordWriter(RecordWriter):
    BATCH = 1000

    def __init__(self, job):
        self.conn = DBConfiguration.connect(job)
        fields = job.get_strings(OUTPUT_FIELDS) or []
        ph = _ph(job)
        cols = f" ({', '.join(fields)})" if fields else ""
        n = len(fields)
        self.sql = f"INSERT INTO {job.get(OUTPUT_TABLE)}{cols} VALUES " \
                   f"({', '.join([ph] * n) if n else '{vals}'})"
        self.rows = []

    def write(self, key, value):
        row = tuple(key.write_fields())
        if "{vals}" in self.sql:
            self.sql = self.sql.replace("{vals}", ", ".join(["?"] * len(row)))
        self.rows.append(row)
        if len(self.rows) >= self.BATCH:
            self._flush()

    def _flush(self):
        if self.rows:
            cur = self.conn.cursor()
            cur.executemany(self.sql, self.rows)
            self.rows = []

    def close(self, reporter=None):
        try:
            self._flush()
            self.conn.commit()
        except Exception:
            self.conn.rollback()
            raise
        finally:
            self.conn.close()


class DBOutputFormat(OutputFormat):
    """Writes reduce-output keys (DBWritable) into a table; values are ignored."""

    @staticmethod
    def set_output(job, table, *fields):
        job.set_output_format(DBOutputFormat)
        job.set(OUTPUT_TABLE, table)
        job.set_strings(OUTPUT_FIELDS, list(fields))

    setOutput = set_output  # noqa: N815

    def checkOutputSpecs(self, fs, job):  # noqa: N802
        if not job.get(OUTPUT_TABLE):
            raise ValueError("DBOutputFormat needs mapred.jdbc.output.table.name")

    def getRecordWriter(self, fs, job, name, progress=None):  # noqa: N802
        return DBRecordWriter(job)
