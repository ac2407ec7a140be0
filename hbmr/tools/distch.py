"""DistCh: change owner / group / permission of many files with a map job.

Behaviour from hadoop-1.0.3/src/tools/org/apache/hadoop/tools/DistCh.java:
arguments ``path:owner:group:permission`` (empty fields leave that attribute
alone, permission in octal), recursive over directories, one file operation
per record split across maps (``-f`` list file, ``-i`` ignore failures),
counters SUCCEED/FAIL.  Applies to the local file system; hbmr.dfs has no
permission model (single-tenant node), so hdfs:// paths are
rejected up front.
"""
from __future__ import annotations

import argparse
import grp
import json
import os
import pwd
import shutil
import tempfile

from ..fs import strip_scheme
from ..mapred import FileInputFormat, JobClient, JobConf
from ..mapred.api import Mapper
from ..mapred.formats import NullOutputFormat
from .distcp import _ChunkInputFormat, _chunks

GROUP = "distch"


def parse_op(spec: str) -> dict:
    parts = spec.split(":")
    if len(parts) != 4:
        raise ValueError(f"bad operation {spec!r} (path:owner:group:permission)")
    path, owner, group, perm = parts
    if perm and not all(c in "01234567" for c in perm):
        raise ValueError(f"bad permission {perm!r}")
    if path.startswith("hdfs://"):
        raise ValueError("hbmr.dfs has no permission model; DistCh works on local paths")
    return {"path": strip_scheme(path), "owner": owner or None, "group": group or None,
            "perm": int(perm, 8) if perm else None}


class ChangeFilesMapper(Mapper):
    def configure(self, job):
        self.ignore = job.get_boolean("distch.ignore.failures", False)

    def map(self, key, value, output, reporter):
        e = json.loads(str(value))
        try:
            if e["perm"] is not None:
                os.chmod(e["path"], e["perm"])
            if e["owner"] is not None or e["group"] is not None:
                uid = pwd.getpwnam(e["owner"]).pw_uid if e["owner"] else -1
                gid = grp.getgrnam(e["group"]).gr_gid if e["group"] else -1
                os.chown(e["path"], uid, gid)
            reporter.incrCounter(GROUP, "SUCCEED", 1)
        except Exception:  # noqa: BLE001
            reporter.incrCounter(GROUP, "FAIL", 1)
            if not self.ignore:
                raise


def change(ops, conf=None, cluster=None, ignore_failures=False, maps=None):
    entries = []
    for spec in ops:
        op = parse_op(spec) if isinstance(spec, str) else spec
        root = op["path"]
        paths = [root] + ([os.path.join(d, n) for d, ds, fs in os.walk(root) for n in ds + fs]
                          if os.path.isdir(root) else [])
        for p in paths:
            entries.append({**op, "path": p, "len": 1})
    job = JobConf(conf)
    work = tempfile.mkdtemp(prefix="distch-")
    try:
        for i, ch in enumerate(_chunks(entries, maps or max(1, min(8, len(entries) // 100 + 1)))):
            with open(os.path.join(work, f"chunk-{i:05d}"), "w") as f:
                for e in ch:
                    f.write(json.dumps(e) + "\n")
        job.set_job_name("distch")
        job.set_boolean("distch.ignore.failures", ignore_failures)
        FileInputFormat.setInputPaths(job, work)
        job.set_input_format(_ChunkInputFormat)
        job.set_mapper_class(ChangeFilesMapper)
        job.set_num_reduce_tasks(0)
        job.set_output_format(NullOutputFormat)
        return JobClient.runJob(job, cluster=cluster, verbose=False)
    finally:
        shutil.rmtree(work, ignore_errors=True)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr distch",
                                 description="distch [-i] [-f list] path:owner:group:permission ...")
    ap.add_argument("-i", action="store_true")
    ap.add_argument("-f", dest="oplist")
    ap.add_argument("ops", nargs="*")
    a = ap.parse_args(argv)
    ops = list(a.ops)
    if a.oplist:
        with open(a.oplist) as f:
            ops += [ln.strip() for ln in f if ln.strip()]
    rj = change(ops, cluster=cluster, ignore_failures=a.i)
    return 0 if rj.isSuccessful() else 1
