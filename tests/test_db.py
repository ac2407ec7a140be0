"""mapred.lib.db: DBInputFormat / DataDrivenDBInputFormat / DBOutputFormat over
DB-API (sqlite3), mirroring the reference's TestDBJob / TestDBInputFormat."""
from __future__ import annotations

import sqlite3

import pytest

from hbmr.io.writable import Text
from hbmr.mapred import JobClient, JobConf
from hbmr.mapred.api import Mapper, Reducer
from hbmr.mapred.lib import db


class Employee(db.DBWritable):
    def read_fields(self, row):
        self.id, self.name, self.dept, self.salary = row

    def write_fields(self):
        return (self.id, self.name, self.dept, self.salary)


class DeptTotal(db.DBWritable):
    def __init__(self, dept=None, total=0.0, n=0):
        self.dept, self.total, self.n = dept, total, n

    def read_fields(self, row):
        self.dept, self.total, self.n = row

    def write_fields(self):
        return (self.dept, self.total, self.n)


class DeptMapper(Mapper):
    def map(self, key, value, output, reporter):
        output.collect(Text(value.dept), Text(f"{value.salary}"))


class DeptReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        xs = [float(str(v)) for v in values]
        output.collect(DeptTotal(str(key), sum(xs), len(xs)), None)


def _db(path, n=200):
    con = sqlite3.connect(path)
    con.execute("CREATE TABLE emp (id INTEGER, name TEXT, dept TEXT, salary REAL)")
    con.executemany("INSERT INTO emp VALUES (?,?,?,?)",
                    [(i, f"e{i:03d}", f"d{i % 7}", 1000.0 + i) for i in range(n)])
    con.execute("CREATE TABLE totals (dept TEXT, total REAL, n INTEGER)")
    con.commit()
    con.close()


def _expected(n=200):
    exp = {}
    for i in range(n):
        d = f"d{i % 7}"
        t, c = exp.get(d, (0.0, 0))
        exp[d] = (t + 1000.0 + i, c + 1)
    return exp


@pytest.mark.parametrize("fmt", ["limit-offset", "data-driven"])
def test_db_to_db_job(tmp_path, fmt):
    path = str(tmp_path / "x.db")
    _db(path)
    job = JobConf()
    db.DBConfiguration.configure_db(job, "sqlite3", path)
    db.DBInputFormat.set_input(job, Employee, table="emp", order_by="id",
                               fields=["id", "name", "dept", "salary"])
    if fmt == "data-driven":
        job.set_input_format(db.DataDrivenDBInputFormat)
    db.DBOutputFormat.set_output(job, "totals", "dept", "total", "n")
    job.set_mapper_class(DeptMapper)
    job.set_reducer_class(DeptReducer)
    job.set_map_output_key_class(Text)
    job.set_map_output_value_class(Text)
    job.set_num_map_tasks(4)
    job.set_num_reduce_tasks(2)
    rj = JobClient.runJob(job, verbose=False)
    cs = rj.getCounters()
    assert cs.get("org.apache.hadoop.mapred.Task$Counter", "MAP_INPUT_RECORDS") == 200
    con = sqlite3.connect(path)
    got = {d: (t, n) for d, t, n in con.execute("SELECT dept, total, n FROM totals")}
    con.close()
    assert got == _expected()


def test_splits_cover_all_rows(tmp_path):
    path = str(tmp_path / "y.db")
    _db(path, n=103)
    job = JobConf()
    db.DBConfiguration.configure_db(job, "sqlite3", path)
    db.DBInputFormat.set_input(job, Employee, table="emp", order_by="id",
                               fields=["id", "name", "dept", "salary"], conditions="salary > 1010")
    for fmt in (db.DBInputFormat(), db.DataDrivenDBInputFormat()):
        seen = []
        for sp in fmt.getSplits(job, 5):
            sp = db.DBInputSplit.deserialize(sp.serialize())
            rr = fmt.getRecordReader(sp, job, None)
            seen += [v.id for _, v in rr]
            rr.close()
        assert sorted(seen) == list(range(11, 103)), type(fmt).__name__
    # text column splitting
    job.set(db.DataDrivenDBInputFormat.SPLIT_BY, "name")
    fmt = db.DataDrivenDBInputFormat()
    seen = []
    for sp in fmt.getSplits(job, 4):
        rr = fmt.getRecordReader(sp, job, None)
        seen += [v.name for _, v in rr]
    assert sorted(seen) == [f"e{i:03d}" for i in range(11, 103)]


def test_output_rolls_back_on_error(tmp_path):
    path = str(tmp_path / "z.db")
    _db(path, n=1)
    job = JobConf()
    db.DBConfiguration.configure_db(job, "sqlite3", path)
    db.DBOutputFormat.set_output(job, "totals", "dept", "total", "n")
    w = db.DBOutputFormat().getRecordWriter(None, job, "part-0")
    w.write(DeptTotal("a", 1.0, 1), None)
    w.write(DeptTotal("b", 2.0, 2, ), None)
    w.rows.append(("c",))   # malformed row → executemany fails → rollback
    with pytest.raises(sqlite3.Error):
        w.close()
    con = sqlite3.connect(path)
    assert con.execute("SELECT COUNT(*) FROM totals").fetchone()[0] == 0
    con.close()


from hbmr.mapreduce import Mapper as _NewMapper, Reducer as _NewReducer  # noqa: E402


class NewM(_NewMapper):
    def map(self, key, value, context):
        context.write(Text(value.dept), Text(f"{value.salary}"))


class NewR(_NewReducer):
    def reduce(self, key, values, context):
        xs = [float(str(v)) for v in values]
        context.write(DeptTotal(str(key), sum(xs), len(xs)), None)


@pytest.mark.parametrize("form", ["table", "query"])
def test_new_api_db_job(tmp_path, form):
    """mapreduce.lib.db: DataDrivenDBInputFormat (table form, and a free-form
    query with $CONDITIONS + bounding query) into DBOutputFormat."""
    from hbmr.mapreduce import Job
    from hbmr.mapreduce.lib import db as ndb
    path = str(tmp_path / "n.db")
    _db(path)
    conf = JobConf()
    conf.set("mapred.job.tracker", "local")
    job = Job(conf, "db")
    c = job.getConfiguration()
    ndb.DBConfiguration.configureDB(c, "sqlite3", path)
    if form == "table":
        ndb.DataDrivenDBInputFormat.setInput(job, Employee, "emp", None, "id",
                                             "id", "name", "dept", "salary")
    else:
        ndb.DataDrivenDBInputFormat.setInput(
            job, Employee, "SELECT id, name, dept, salary FROM emp WHERE $CONDITIONS",
            "SELECT MIN(id), MAX(id) FROM emp")
        c.set(db.INPUT_ORDER_BY, "id")
    ndb.DBOutputFormat.setOutput(job, "totals", "dept", "total", "n")
    c.set_num_map_tasks(3)
    job.setMapperClass(NewM)
    job.setReducerClass(NewR)
    job.setMapOutputKeyClass(Text)
    job.setMapOutputValueClass(Text)
    job.setNumReduceTasks(2)
    assert job.waitForCompletion(False)
    con = sqlite3.connect(path)
    got = {d: (t, n) for d, t, n in con.execute("SELECT dept, total, n FROM totals")}
    con.close()
    assert got == _expected()


def test_new_api_splitters():
    from hbmr.mapreduce.lib import db as ndb
    conf = JobConf()
    conf.set_num_map_tasks(4)
    sp = ndb.IntegerSplitter().split(conf, 0, 100, "id")
    assert len(sp) == 4 and sp[0].params[0] == 0 and sp[-1].params[1] == 100
    assert "<=" in sp[-1].where and "<=" not in sp[0].where.split("AND")[1]
    ts = ndb.TextSplitter().split(conf, "aaa", "azz", "name")
    assert ts[0].params[0] == "aaa" and ts[-1].params[1] == "azz"
    assert all(a.params[1] == b.params[0] for a, b in zip(ts, ts[1:]))
