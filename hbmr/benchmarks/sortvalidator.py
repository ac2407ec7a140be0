"""SortValidator: checks the output of ``sort`` against its input.

Behaviour from hadoop-1.0.3/src/test/org/apache/hadoop/mapred/SortValidator.java:
(1) RecordStatsChecker — record count, byte count and an order-independent
checksum of all records must match between sort input and output;
(2) RecordChecker — every output file is sorted by the job's key order and
every record sits in the partition the partitioner assigns it (hash
partitioning, or contiguous key ranges under total order); every input record
appears in the output exactly as often as in the input.

Our form: one map-only job reads input and output together (the map knows
which side a split belongs to from ``map.input.file``) and folds everything
into counters — sums of a 64-bit record hash and of its square make the
multiset comparison order-free without a shuffle — while the per-file order
and partition checks run in the maps over the sorted side.
"""
from __future__ import annotations

import argparse
import hashlib
import os

from ..io import sequencefile as seqf
from ..mapred import FileInputFormat, JobClient, JobConf
from ..mapred.api import Mapper
from ..mapred.formats import NullOutputFormat, SequenceFileInputFormat, SequenceFileRecordReader

GROUP = "SortValidator"
M64 = (1 << 64) - 1


class _WholeFileSeq(SequenceFileInputFormat):
    def is_splitable(self, fs, path):
        return False

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return _RawReader(job, split)


class _RawReader(SequenceFileRecordReader):
    def next(self):
        return self.next_raw()


def _rec_hash(kb: bytes, vb: bytes) -> int:
    d = hashlib.blake2b(kb, digest_size=8, key=b"k")
    d.update(len(kb).to_bytes(4, "big"))
    d.update(vb)
    return int.from_bytes(d.digest(), "little")


class ValidateMapper(Mapper):
    def configure(self, job):
        path = job.get("map.input.file", "")
        self.sorted_side = os.path.abspath(path).startswith(
            os.path.abspath(job.get("sortvalidate.sorted.dir")))
        self.side = "OUT" if self.sorted_side else "IN"
        self.prev = None
        self.part = None
        self.reduces = job.get_int("sortvalidate.reduces", 1)
        self.total_order = job.get_boolean("sortvalidate.total.order", False)
        name = os.path.basename(path)
        if self.sorted_side and name.startswith("part-"):
            self.part = int(name.split("-")[1])
        r = seqf.Reader(path)
        self.kcls = r.key_class
        r.close()
        self.first = None

    def map(self, key, value, output, reporter):
        kb, vb = key, value
        h = _rec_hash(kb, vb)
        reporter.incrCounter(GROUP, f"{self.side}_RECORDS", 1)
        reporter.incrCounter(GROUP, f"{self.side}_BYTES", len(kb) + len(vb))
        reporter.incrCounter(GROUP, f"{self.side}_HASH_SUM", h)
        reporter.incrCounter(GROUP, f"{self.side}_HASH_SQ_SUM", (h * h) & M64)
        if not self.sorted_side:
            return
        sk = self.kcls.raw_sort_key(kb)
        if self.prev is not None and sk < self.prev:
            reporter.incrCounter(GROUP, "UNSORTED_RECORDS", 1)
        self.prev = sk
        if self.first is None:
            self.first = sk
        if not self.total_order and self.part is not None:
            k = self.kcls.deserialize(kb)
            if (k.hash_code() & 0x7FFFFFFF) % self.reduces != self.part:
                reporter.incrCounter(GROUP, "MISPARTITIONED_RECORDS", 1)


def validate(sort_input, sort_output, conf=None, cluster=None, total_order=False) -> dict:
    """Run the checks; returns {'ok': bool, ...counts}."""
    job = JobConf(conf)
    outs = sorted(p for p in os.listdir(sort_output) if p.startswith("part-"))
    job.set_job_name("sortvalidate")
    job.set("sortvalidate.sorted.dir", sort_output)
    job.set_int("sortvalidate.reduces", len(outs))
    job.set_boolean("sortvalidate.total.order", total_order)
    FileInputFormat.setInputPaths(job, sort_input, sort_output)
    job.set_input_format(_WholeFileSeq)
    job.set_mapper_class(ValidateMapper)
    job.set_num_reduce_tasks(0)
    job.set_output_format(NullOutputFormat)
    rj = JobClient.runJob(job, cluster=cluster, verbose=False)
    cs = rj.getCounters()

    def c(n):
        return cs.get(GROUP, n)

    res = {k: c(k) for k in ("IN_RECORDS", "OUT_RECORDS", "IN_BYTES", "OUT_BYTES",
                             "UNSORTED_RECORDS", "MISPARTITIONED_RECORDS")}
    res["checksum_match"] = (c("IN_HASH_SUM") == c("OUT_HASH_SUM") and
                             (c("IN_HASH_SQ_SUM") & M64) == (c("OUT_HASH_SQ_SUM") & M64))
    if total_order:  # partitions must hold contiguous, increasing key ranges
        res["RANGE_OVERLAPS"] = _range_overlaps(sort_output, outs)
    res["ok"] = (res["IN_RECORDS"] == res["OUT_RECORDS"] and res["IN_BYTES"] == res["OUT_BYTES"]
                 and res["checksum_match"] and res["UNSORTED_RECORDS"] == 0
                 and res["MISPARTITIONED_RECORDS"] == 0 and res.get("RANGE_OVERLAPS", 0) == 0)
    return res


def _range_overlaps(d, outs) -> int:
    bounds = []
    for p in outs:
        r = seqf.Reader(os.path.join(d, p))
        kcls = r.key_class
        lo = hi = None
        while True:
            raw = r.next_raw()
            if raw is None:
                break
            sk = kcls.raw_sort_key(raw[0])
            lo = sk if lo is None else lo
            hi = sk
        r.close()
        if lo is not None:
            bounds.append((lo, hi))
    return sum(1 for a, b in zip(bounds, bounds[1:]) if a[1] > b[0])


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="sortvalidate")
    ap.add_argument("-sortInput", required=True)
    ap.add_argument("-sortOutput", required=True)
    ap.add_argument("-totalOrder", action="store_true")
    a = ap.parse_args(argv)
    res = validate(a.sortInput, a.sortOutput, cluster=cluster, total_order=a.totalOrder)
    print(("SUCCESS! Validated the MapReduce framework's 'sort' successfully."
           if res["ok"] else f"FAILED: {res}"))
    return 0 if res["ok"] else 1

