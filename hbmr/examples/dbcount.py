"""DBCountPageView: page views per URL from a database access log, written back
to the database (src/examples/org/apache/hadoop/examples/DBCountPageView.java).

The reference starts an HSQLDB server; hbmr uses a DB-API module instead
(``sqlite3`` by default, a file under ``test.build.data``).  The program
creates ``Access(url, referrer, time)`` and ``Pageview(url, pageview)``,
fills Access with a random-surfer walk over ten linked pages
(DBCountPageView.java:179-236), runs the job (DBInputFormat ordered by url →
(url, 1) → LongSumReducer combiner → PageviewRecord rows through
DBOutputFormat) and checks that the page views add up to the log's rows.

Usage: ``dbcount [driverModule dbUrl]``."""
from __future__ import annotations

import importlib
import os
import random
import sys

from ..io.writable import LongWritable, NullWritable, Text
from ..mapred import JobClient, JobConf
from ..mapred.api import Mapper, Reducer
from ..mapred.lib import LongSumReducer
from ..mapred.lib import db

ACCESS_FIELDS = ("url", "referrer", "time")
PAGEVIEW_FIELDS = ("url", "pageview")
PAGES = ["/a", "/b", "/c", "/d", "/e", "/f", "/g", "/h", "/i", "/j"]
LINKS = [[1, 5, 7], [0, 7, 4, 6], [0, 1, 7, 8], [0, 2, 4, 6, 7, 9], [0, 1],
         [0, 3, 5, 9], [0], [0, 1, 3], [0, 2, 6], [0, 2, 6]]


class AccessRecord(db.DBWritable):
    def read_fields(self, row):
        self.url, self.referrer, self.time = row

    def write_fields(self):
        return (self.url, self.referrer, self.time)


class PageviewRecord(db.DBWritable):
    def __init__(self, url=None, pageview=0):
        self.url, self.pageview = url, pageview

    def read_fields(self, row):
        self.url, self.pageview = row

    def write_fields(self):
        return (self.url, self.pageview)

    def __str__(self):
        return f"{self.url} {self.pageview}"


class PageviewMapper(Mapper):
    ONE = LongWritable(1)

    def map(self, key, value, output, reporter):
        output.collect(Text(value.url), self.ONE)


class PageviewReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(PageviewRecord(str(key), sum(v.get() for v in values)), NullWritable.get())


def _connect(driver, url):
    return importlib.import_module(driver).connect(url)


def initialize(driver, url, seed=None):
    """Drop/create the tables and populate Access (a random surfer)."""
    con = _connect(driver, url)
    try:
        for t in ("Access", "Pageview"):
            try:
                con.execute(f"DROP TABLE {t}")
            except Exception:  # noqa: BLE001 (absent table)
                pass
        con.execute("CREATE TABLE Access (url VARCHAR(100) NOT NULL, referrer VARCHAR(100), "
                    "time BIGINT NOT NULL, PRIMARY KEY (url, time))")
        con.execute("CREATE TABLE Pageview (url VARCHAR(100) NOT NULL, pageview BIGINT NOT NULL, "
                    "PRIMARY KEY (url))")
        rnd = random.Random(seed)
        n = rnd.randrange(50) + 50
        cur, ref, rows = rnd.randrange(len(PAGES)), None, []
        for i in range(n):
            rows.append((PAGES[cur], ref, i))
            if rnd.randrange(100) < 15:               # jump to a random page
                cur, ref = rnd.randrange(len(PAGES)), None
            else:                                     # follow a link
                ref = PAGES[cur]
                cur = LINKS[cur][rnd.randrange(len(LINKS[cur]))]
        con.executemany("INSERT INTO Access(url, referrer, time) VALUES (?, ?, ?)", rows)
        con.commit()
        return n
    finally:
        con.close()


def verify(driver, url) -> bool:
    con = _connect(driver, url)
    try:
        total = con.execute("SELECT COUNT(*) FROM Access").fetchone()[0]
        summed = con.execute("SELECT SUM(pageview) FROM Pageview").fetchone()[0] or 0
        return total == summed and total != 0
    finally:
        con.close()


def make_job(driver, url, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name("Count Pageviews of URLs")
    job.set_mapper_class(PageviewMapper)
    job.set_combiner_class(LongSumReducer)
    job.set_reducer_class(PageviewReducer)
    db.DBConfiguration.configure_db(job, driver, url)
    db.DBInputFormat.set_input(job, AccessRecord, table="Access", order_by="url",
                               fields=list(ACCESS_FIELDS))
    db.DBOutputFormat.set_output(job, "Pageview", *PAGEVIEW_FIELDS)
    job.set_map_output_key_class(Text)
    job.set_map_output_value_class(LongWritable)
    job.set_output_key_class(PageviewRecord)
    job.set_output_value_class(NullWritable)
    return job


def main(argv=None, cluster=None) -> int:
    args = list(sys.argv[1:] if argv is None else argv)
    if len(args) > 1:
        driver, url = args[0], args[1]
    else:
        driver = "sqlite3"
        url = os.path.join(os.environ.get("test.build.data", "."), "URLAccess.db")
    initialize(driver, url)
    JobClient.runJob(make_job(driver, url), cluster=cluster)
    if not verify(driver, url):
        raise RuntimeError("Evaluation was not correct!")
    return 0


if __name__ == "__main__":
    sys.exit(main())
