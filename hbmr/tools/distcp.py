"""DistCp: parallel copy of file trees as a map-only job.

Behaviour follows hadoop-1.0.3/src/tools/org/apache/hadoop/tools/DistCp.java:
options -update/-overwrite/-delete/-i/-p/-skipcrccheck/-filelimit/-sizelimit/
-log/-m/-f (127-135, 772-850), the "special" root rule (a single source into a
missing destination, or -update/-overwrite, copies the source's *contents*;
1085-1093), skip-if-exists unless -overwrite or the file differs under -update
(404-411, sameFile 1208), per-file copy through a temporary name then rename
(the ``_distcp_tmp_`` dir, 1183-1185), counters COPY/SKIP/FAIL/BYTESCOPIED/
BYTESEXPECTED (126, DistCp_Counter.properties) and map count =
total bytes / distcp.bytes.per.map capped by distcp.max.map.tasks (949-957).

Not a translation: the file list is cut into byte-balanced chunk files up
front (one per map, first-fit-decreasing), so every map gets one
non-splittable chunk and no sync-marker SequenceFile is needed; copies stream
through the FileSystem layer, so ``file://`` ↔ ``hdfs://`` in any direction.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import uuid
import zlib

from ..fs import get_fs, hidden, strip_scheme
from ..io.writable import NullWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf
from ..mapred.api import Mapper
from ..mapred.formats import LineRecordReader, TextInputFormat

NAME = "distcp"
BYTES_PER_MAP = 256 * 1024 * 1024
MAX_MAPS_PER_NODE = 20
BUF = 1 << 20
GROUP = "distcp"

OPTIONS = {  # flag -> property (DistCp.Options)
    "-delete": "distcp.delete",
    "-i": "distcp.ignore.read.failures",
    "-p": "distcp.preserve.status",
    "-overwrite": "distcp.overwrite.always",
    "-update": "distcp.overwrite.ifnewer",
    "-skipcrccheck": "distcp.skip.crc.check",
}


def _join(root: str, rel: str) -> str:
    return root.rstrip("/") + "/" + rel if rel else root


def _crc(fs, path) -> int:
    c = 0
    with fs.open(path) as f:
        while True:
            b = f.read(BUF)
            if not b:
                return c
            c = zlib.crc32(b, c)


def same_file(srcfs, src, dstfs, dst, skip_crc=False) -> bool:
    """True iff dst exists with src's length and (unless skipped) checksum."""
    if not dstfs.exists(dst):
        return False
    s, d = srcfs.get_file_status(src), dstfs.get_file_status(dst)
    if d.is_dir or s.length != d.length:
        return False
    return skip_crc or _crc(srcfs, src) == _crc(dstfs, dst)


class _ChunkInputFormat(TextInputFormat):
    """One whole chunk file per map (the chunks are already byte-balanced)."""

    def is_splitable(self, fs, path):
        return False

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        return LineRecordReader(job, split)


class CopyFilesMapper(Mapper):
    """Copies each listed file; emits SKIP:/FAIL: lines to the log output."""

    def configure(self, job):
        self.dst_root = job.get("distcp.dest.path")
        self.tmp_dir = job.get("distcp.tmp.dir")
        self.update = job.get_boolean(OPTIONS["-update"], False)
        self.overwrite = not self.update and job.get_boolean(OPTIONS["-overwrite"], False)
        self.ignore_failures = job.get_boolean(OPTIONS["-i"], False)
        self.preserve = job.get_boolean(OPTIONS["-p"], False)
        self.skip_crc = job.get_boolean(OPTIONS["-skipcrccheck"], False)
        self.job = job

    def map(self, key, value, output, reporter):
        e = json.loads(str(value))
        src, dst = e["src"], _join(self.dst_root, e["rel"])
        srcfs, dstfs = get_fs(src, self.job), get_fs(dst, self.job)
        if e["dir"]:
            dstfs.mkdirs(dst)
            return
        try:
            if dstfs.exists(dst) and not self.overwrite and not (
                    self.update and not same_file(srcfs, src, dstfs, dst, self.skip_crc)):
                output.collect(NullWritable.get(), Text(f"SKIP: {src}"))
                reporter.incrCounter(GROUP, "SKIP", 1)
                return
            reporter.incrCounter(GROUP, "BYTESEXPECTED", e["len"])
            n = self._copy(srcfs, src, dstfs, dst, reporter)
            if n != e["len"]:
                raise OSError(f"File size not matched: copied {n} bytes to tmp (= {dst}),"
                              f" expected {e['len']} (src = {src})")
            reporter.incrCounter(GROUP, "COPY", 1)
            reporter.incrCounter(GROUP, "BYTESCOPIED", n)
        except Exception as exc:  # noqa: BLE001 - per-file failure is recorded, -i decides
            reporter.incrCounter(GROUP, "FAIL", 1)
            output.collect(NullWritable.get(), Text(f"FAIL: {src} : {exc}"))
            if not self.ignore_failures:
                raise

    def _copy(self, srcfs, src, dstfs, dst, reporter) -> int:
        tmp = _join(self.tmp_dir, uuid.uuid4().hex)
        n = 0
        repl = None
        if self.preserve and hasattr(srcfs, "set_replication"):
            try:
                repl = getattr(srcfs.get_file_status(src), "replication", None)
            except Exception:  # noqa: BLE001
                repl = None
        with srcfs.open(src) as fin, dstfs.create(tmp, overwrite=True) as fout:
            while True:
                b = fin.read(BUF)
                if not b:
                    break
                fout.write(b)
                n += len(b)
                reporter.progress()
        if dstfs.exists(dst):
            dstfs.delete(dst, recursive=False)
        parent = os.path.dirname(dst.rstrip("/"))
        if parent:
            dstfs.mkdirs(parent)
        if not dstfs.rename(tmp, dst):
            raise OSError(f"rename {tmp} -> {dst} failed")
        if repl and hasattr(dstfs, "set_replication"):
            dstfs.set_replication(dst, repl)
        if self.preserve and not dst.startswith("hdfs://") and not src.startswith("hdfs://"):
            st = os.stat(strip_scheme(src))
            os.utime(strip_scheme(dst), (st.st_atime, st.st_mtime))
        return n


def _walk(fs, root_status):
    """(FileStatus, is_dir) of everything below a directory, depth-first."""
    stack = [root_status]
    while stack:
        cur = stack.pop()
        for ch in fs.list_status(cur.path, filter_hidden=False):
            yield ch
            if ch.is_dir:
                stack.append(ch)


def _rel(root: str, path: str) -> str:
    r, p = strip_scheme(root).rstrip("/"), strip_scheme(path)
    return p[len(r):].lstrip("/") if p.startswith(r) else os.path.basename(p)


def build_file_list(srcs, dst, conf, update=False, overwrite=False, skip_crc=False,
                    filelimit=None, sizelimit=None):
    """The copy list: [{src, rel, len, dir}], plus totals (DistCp.setup 1060-1190)."""
    dstfs = get_fs(dst, conf)
    dst_exists = dstfs.exists(dst)
    dst_is_dir = dst_exists and dstfs.is_dir(dst)
    special = (len(srcs) == 1 and not dst_exists) or update or overwrite
    entries, files, nbytes = [], 0, 0
    filelimit = sys.maxsize if filelimit is None else filelimit
    sizelimit = sys.maxsize if sizelimit is None else sizelimit
    for src in srcs:
        srcfs = get_fs(src, conf)
        st = srcfs.get_file_status(src)
        if not st.is_dir:
            if dst_exists and not dst_is_dir and len(srcs) == 1:
                rel = ""  # file onto an existing file path
            elif not dst_exists and len(srcs) == 1:
                rel = ""
            else:
                rel = os.path.basename(src.rstrip("/"))
            children = [(st, rel)]
        else:
            root = src if special else os.path.dirname(src.rstrip("/"))
            children = []
            if not special:
                children.append((st, _rel(root, src)))
            children += [(c, _rel(root, c.path)) for c in _walk(srcfs, st)]
        for c, rel in children:
            if c.is_dir:
                entries.append({"src": c.path, "rel": rel, "len": 0, "dir": True})
                continue
            if hidden(c.path) and os.path.basename(c.path).startswith("_distcp"):
                continue
            target = _join(dst, rel)
            if update and same_file(srcfs, c.path, dstfs, target, skip_crc):
                continue
            if files == filelimit or nbytes + c.length > sizelimit:
                continue
            files += 1
            nbytes += c.length
            entries.append({"src": c.path, "rel": rel, "len": c.length, "dir": False})
    rels = [e["rel"] for e in entries if not e["dir"]]
    dup = {r for r in rels if rels.count(r) > 1} if len(rels) != len(set(rels)) else set()
    if dup:
        raise OSError(f"Duplicated files found at destination: {sorted(dup)[:5]}")
    return entries, files, nbytes


def _chunks(entries, n_maps):
    """First-fit-decreasing by bytes: n_maps chunks of near-equal total size."""
    bins = [[0, []] for _ in range(max(1, n_maps))]
    for e in sorted(entries, key=lambda e: -e["len"]):
        b = min(bins, key=lambda b: b[0])
        b[0] += max(e["len"], 1)
        b[1].append(e)
    return [b[1] for b in bins if b[1]]


def delete_nonexisting(srcs_entries, dst, conf) -> int:
    """-delete: remove destination files absent from the source tree (1178-1181)."""
    dstfs = get_fs(dst, conf)
    if not dstfs.exists(dst) or not dstfs.is_dir(dst):
        return 0
    keep = {e["rel"] for e in srcs_entries}
    n = 0
    for st in list(_walk(dstfs, dstfs.get_file_status(dst))):
        rel = _rel(dst, st.path)
        if rel not in keep and not any(k.startswith(rel + "/") for k in keep):
            if dstfs.exists(st.path):
                dstfs.delete(st.path, recursive=True)
                n += 1
    return n


def copy(srcs, dst, conf=None, cluster=None, update=False, overwrite=False, delete=False,
         ignore_failures=False, preserve=False, skip_crc=False, filelimit=None,
         sizelimit=None, log_dir=None, maps=None, verbose=False):
    """Run DistCp; returns the RunningJob (None if there was nothing to copy)."""
    if isinstance(srcs, str):
        srcs = [srcs]
    if delete and not (update or overwrite):
        raise ValueError("-delete must be specified with -overwrite or -update.")
    if skip_crc and not update:
        raise ValueError("-skipcrccheck is relevant only with the -update option")
    job = JobConf(conf)
    job.set_job_name(f"distcp: {','.join(srcs)} -> {dst}")
    dstfs = get_fs(dst, job)
    entries, nfiles, nbytes = build_file_list(srcs, dst, job, update, overwrite, skip_crc,
                                              filelimit, sizelimit)
    if delete:
        delete_nonexisting(entries, dst, job)
    if nfiles == 0 and not any(e["dir"] for e in entries):
        return None
    dst_exists = dstfs.exists(dst)
    if (len(srcs) > 1 or any(e["rel"] for e in entries)) and not dst_exists:
        dstfs.mkdirs(dst)
    per_map = job.get_long("distcp.bytes.per.map", BYTES_PER_MAP)
    n_maps = maps or min(max(1, nbytes // max(per_map, 1)),
                         job.get_int("distcp.max.map.tasks", MAX_MAPS_PER_NODE * 8))
    n_maps = max(1, min(n_maps, max(1, len(entries))))
    work = tempfile.mkdtemp(prefix="distcp-")
    tmp_dir = _join(dst if dstfs.is_dir(dst) else os.path.dirname(dst.rstrip("/")) or ".",
                    f"_distcp_tmp_{uuid.uuid4().hex[:6]}")
    try:
        dirs = [e for e in entries if e["dir"]]
        files = [e for e in entries if not e["dir"]]
        chunks = _chunks(files, n_maps) or [[]]
        chunks[0] = dirs + chunks[0]  # directories first, created before any file lands
        for i, ch in enumerate(chunks):
            with open(os.path.join(work, f"chunk-{i:05d}"), "w") as f:
                for e in ch:
                    f.write(json.dumps(e) + "\n")
        job.set("distcp.dest.path", dst)
        job.set("distcp.tmp.dir", tmp_dir)
        job.set_long("distcp.total.size", nbytes)
        job.set_int("distcp.src.count", nfiles)
        job.set_boolean(OPTIONS["-update"], update)
        job.set_boolean(OPTIONS["-overwrite"], overwrite and not update)
        job.set_boolean(OPTIONS["-i"], ignore_failures)
        job.set_boolean(OPTIONS["-p"], preserve)
        job.set_boolean(OPTIONS["-skipcrccheck"], skip_crc)
        job.set_boolean("mapred.map.tasks.speculative.execution", False)
        job.set_int("mapred.map.max.attempts", job.get_int("mapred.map.max.attempts", 1)
                    if ignore_failures else job.get_int("mapred.map.max.attempts", 4))
        FileInputFormat.setInputPaths(job, work)
        job.set_input_format(_ChunkInputFormat)
        job.set_mapper_class(CopyFilesMapper)
        job.set_num_map_tasks(len(chunks))
        job.set_num_reduce_tasks(0)
        job.set_output_key_class(NullWritable)
        job.set_output_value_class(Text)
        FileOutputFormat.setOutputPath(job, log_dir or os.path.join(work, "_logs"))
        return JobClient.runJob(job, cluster=cluster, verbose=verbose)
    finally:
        if dstfs.exists(tmp_dir):
            dstfs.delete(tmp_dir, recursive=True)
        import shutil
        shutil.rmtree(work, ignore_errors=True)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr distcp", description="distcp [OPTIONS] <srcurl>* <desturl>")
    for flag in OPTIONS:
        ap.add_argument(flag, action="store_true")
    ap.add_argument("-f", dest="srclist", help="use list at <urilist_uri> as src list")
    ap.add_argument("-log", dest="log")
    ap.add_argument("-m", dest="maps", type=int)
    ap.add_argument("-filelimit", type=int)
    ap.add_argument("-sizelimit", type=int)
    ap.add_argument("paths", nargs="+")
    a = ap.parse_args(argv)
    srcs, dst = a.paths[:-1], a.paths[-1]
    if a.srclist:
        with open(strip_scheme(a.srclist)) as f:
            srcs += [ln.strip() for ln in f if ln.strip()]
    if not srcs:
        ap.error("missing source")
    rj = copy(srcs, dst, cluster=cluster, update=a.update, overwrite=a.overwrite,
              delete=a.delete, ignore_failures=a.i, preserve=a.p, skip_crc=a.skipcrccheck,
              filelimit=a.filelimit, sizelimit=a.sizelimit, log_dir=a.log, maps=a.maps,
              verbose=True)
    return 0 if rj is None or rj.isSuccessful() else 1
