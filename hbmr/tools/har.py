"""Hadoop archives: ``hbmr archive -archiveName NAME.har -p PARENT SRC* DEST`` and
the read-only ``har://`` file system over them.

Behaviour from hadoop-1.0.3/src/tools/org/apache/hadoop/tools/HadoopArchives.java
(VERSION 3 at 78; part files ``part-N`` written by the maps, 593; one reducer
writing ``_index`` lines ``<urlenc path> dir <props> 0 0 <children…>`` /
``<urlenc path> file part-N <start> <len> <props>`` ordered by path hash, and a
``_masterindex`` of ``<startHash> <endHash> <indexStart> <indexEnd>`` ranges,
641-691, 725-778) and src/core/org/apache/hadoop/fs/HarFileSystem.java (the
``har://`` scheme: ``har:///abs/x.har/inner`` over the local FS or
``har://hdfs-<authority>/x.har/inner`` over hbmr.dfs).

Our design: the archive job is a normal hbmr job.  Maps get byte-balanced
chunks (same helper as DistCp), stream each file into their own part file
(written under a temporary name, renamed on close so retries cannot leave
torn parts) and emit ``(hash, index line)``; the single reducer receives the
lines already sorted by hash from the shuffle and writes both index files.
The reader keeps the whole index in a dict (archives index small metadata
only) and serves file bodies as bounded views of the part files.
"""
from __future__ import annotations

import argparse
import io
import json
import os
import shutil
import tempfile
import urllib.parse
import uuid

from ..fs import FileStatus, get_fs, strip_scheme
from ..io.writable import IntWritable, Text
from ..mapred import FileInputFormat, JobClient, JobConf
from ..mapred.api import Mapper, Reducer
from ..mapred.formats import NullOutputFormat
from .distcp import BUF, _ChunkInputFormat, _chunks, _rel, _walk

VERSION = 3
INDEX_BLOCK = 1000  # index lines per _masterindex range


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode over UTF-16 code units, as a signed int."""
    h = 0
    for cu in s.encode("utf-16-be").hex(" ", 2).split():
        h = (31 * h + int(cu, 16)) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


def _enc(s: str) -> str:
    return urllib.parse.quote_plus(s, safe="/")


def _dec(s: str) -> str:
    return urllib.parse.unquote_plus(s)


def _props(st: FileStatus) -> str:
    return _enc(f"{int(st.modification_time * 1000)} 644 hbmr hbmr")


class HarMapper(Mapper):
    def configure(self, job):
        self.job = job
        self.archive = job.get("har.archive.path")
        self.part = f"part-{job.get_int('mapred.task.partition', 0)}"
        self.fs = get_fs(self.archive, job)
        self.tmp = f"{self.archive}/_tmp_{self.part}_{uuid.uuid4().hex[:8]}"
        self.out = None
        self.pos = 0

    def map(self, key, value, output, reporter):
        e = json.loads(str(value))
        path = "/" + e["rel"] if e["rel"] else "/"
        h = IntWritable(java_string_hash(path))
        if e["dir"]:
            kids = " ".join(_enc(c) for c in e["children"])
            output.collect(h, Text(f"{_enc(path)} dir {e['props']} 0 0 {kids}".rstrip()))
            return
        if self.out is None:
            self.out = self.fs.create(self.tmp, overwrite=True)
        start = self.pos
        srcfs = get_fs(e["src"], self.job)
        with srcfs.open(e["src"]) as f:
            while True:
                b = f.read(BUF)
                if not b:
                    break
                self.out.write(b)
                self.pos += len(b)
                reporter.progress()
        output.collect(h, Text(f"{_enc(path)} file {self.part} {start} {self.pos - start} "
                               f"{e['props']}"))

    def close(self):
        if self.out is not None:
            self.out.close()
            dst = f"{self.archive}/{self.part}"
            if self.fs.exists(dst):
                self.fs.delete(dst, recursive=False)
            self.fs.rename(self.tmp, dst)


class HarIndexReducer(Reducer):
    """Single reducer: index lines arrive sorted by hash; write _index/_masterindex."""

    def configure(self, job):
        self.archive = job.get("har.archive.path")
        self.fs = get_fs(self.archive, job)
        self.lines = []  # (hash, line)

    def reduce(self, key, values, output, reporter):
        h = key.get()
        for v in sorted(str(v) for v in values):
            self.lines.append((h, v))

    def close(self):
        index, master = io.BytesIO(), io.BytesIO()
        master.write(f"{VERSION} \n".encode())
        for i in range(0, len(self.lines), INDEX_BLOCK):
            blk = self.lines[i:i + INDEX_BLOCK]
            start = index.tell()
            for _, ln in blk:
                index.write((ln + " \n").encode())
            master.write(f"{blk[0][0]} {blk[-1][0]} {start} {index.tell()} \n".encode())
        for name, buf in (("_index", index), ("_masterindex", master)):
            with self.fs.create(f"{self.archive}/{name}", overwrite=True) as f:
                f.write(buf.getvalue())


def create_archive(name, parent, srcs, dest, conf=None, cluster=None, maps=None,
                   verbose=False):
    """Archive ``srcs`` (relative to ``parent``) into ``dest/name`` (must end .har)."""
    if not name.endswith(".har"):
        raise ValueError(f"Invalid name for archives. {name}")
    job = JobConf(conf)
    archive = dest.rstrip("/") + "/" + name
    fs = get_fs(archive, job)
    if fs.exists(archive):
        raise FileExistsError(f"Invalid Output: {archive}")
    srcs = [s if (s.startswith("/") or "://" in s) else parent.rstrip("/") + "/" + s
            for s in (srcs or [parent])]
    entries, dirs = [], {}

    def add_dir(rel, st):
        if rel not in dirs:
            dirs[rel] = {"src": st.path if st else "", "rel": rel, "dir": True,
                         "children": [], "props": _props(st) if st else _enc("0 755 hbmr hbmr")}
            if rel:
                up = os.path.dirname(rel)
                add_dir(up, None)
                kid = os.path.basename(rel)
                if kid not in dirs[up]["children"]:
                    dirs[up]["children"].append(kid)
        elif st is not None and not dirs[rel]["src"]:
            dirs[rel].update(src=st.path, props=_props(st))

    add_dir("", None)
    for s in srcs:
        sfs = get_fs(s, job)
        st = sfs.get_file_status(s)
        items = [st] + (list(_walk(sfs, st)) if st.is_dir else [])
        for it in items:
            rel = _rel(parent, it.path)
            if it.is_dir:
                add_dir(rel, it)
            else:
                add_dir(os.path.dirname(rel), None)
                kid = os.path.basename(rel)
                up = dirs[os.path.dirname(rel)]
                if kid not in up["children"]:
                    up["children"].append(kid)
                entries.append({"src": it.path, "rel": rel, "dir": False, "len": it.length,
                                "props": _props(it)})
    work = tempfile.mkdtemp(prefix="har-")
    try:
        nbytes = sum(e["len"] for e in entries)
        n_maps = maps or max(1, min(len(entries), nbytes // (256 << 20) + 1))
        chunks = _chunks(entries, n_maps) or [[]]
        chunks[0] = list(dirs.values()) + chunks[0]
        for i, ch in enumerate(chunks):
            with open(os.path.join(work, f"chunk-{i:05d}"), "w") as f:
                for e in ch:
                    f.write(json.dumps(e) + "\n")
        fs.mkdirs(archive)
        job.set_job_name(f"archive {name}")
        job.set("har.archive.path", archive)
        job.set_boolean("mapred.map.tasks.speculative.execution", False)
        FileInputFormat.setInputPaths(job, work)
        job.set_input_format(_ChunkInputFormat)
        job.set_mapper_class(HarMapper)
        job.set_reducer_class(HarIndexReducer)
        job.set_num_map_tasks(len(chunks))
        job.set_num_reduce_tasks(1)
        job.set_map_output_key_class(IntWritable)
        job.set_map_output_value_class(Text)
        job.set_output_format(NullOutputFormat)
        rj = JobClient.runJob(job, cluster=cluster, verbose=verbose)
        for st in fs.list_status(archive, filter_hidden=False):
            if os.path.basename(st.path).startswith("_tmp_"):
                fs.delete(st.path, recursive=False)
        return rj
    except BaseException:
        if fs.exists(archive):
            fs.delete(archive, recursive=True)
        raise
    finally:
        shutil.rmtree(work, ignore_errors=True)


# ---------------------------------------------------------------- har:// read side
class _Slice(io.RawIOBase):
    """Bounded, seekable view [start, start+length) of an underlying stream."""

    def __init__(self, raw, start, length):
        self.raw, self.start, self.length, self.pos = raw, start, length, 0

    def readable(self):
        return True

    def seekable(self):
        return True

    def readinto(self, b):
        n = min(len(b), self.length - self.pos)
        if n <= 0:
            return 0
        self.raw.seek(self.start + self.pos)
        data = self.raw.read(n)
        b[:len(data)] = data
        self.pos += len(data)
        return len(data)

    def seek(self, off, whence=0):
        base = {0: 0, 1: self.pos, 2: self.length}[whence]
        self.pos = max(0, base + off)
        return self.pos

    def tell(self):
        return self.pos

    def close(self):
        if not self.closed:
            self.raw.close()
        super().close()


def split_har_uri(uri: str):
    """har URI → (underlying archive root, path inside the archive)."""
    rest = uri[len("har://"):]
    if rest.startswith("/"):
        under, path = "", rest
    else:
        auth, _, path = rest.partition("/")
        path = "/" + path
        scheme, _, authority = auth.partition("-")
        if scheme != "hdfs":
            raise ValueError(f"unsupported har underlying scheme in {uri!r}")
        under = f"hdfs://{authority}"
    i = path.find(".har")
    while i >= 0 and not (i + 4 == len(path) or path[i + 4] == "/"):
        i = path.find(".har", i + 1)
    if i < 0:
        raise ValueError(f"Invalid har URI (no .har component): {uri}")
    return under + path[:i + 4], path[i + 4:] or "/"


class HarFileSystem:
    """Read-only FileSystem over one archive (HarFileSystem.java)."""

    scheme = "har"

    def __init__(self, uri, conf=None):
        self.archive, _ = split_har_uri(uri)
        self.prefix = uri[:uri.find(".har") + 4]
        self.fs = get_fs(self.archive, conf)
        self.conf = conf
        with self.fs.open(self.archive + "/_masterindex") as f:
            version = int(f.readline().split()[0])
        if version != VERSION:
            raise OSError(f"Invalid version {version} expected {VERSION}")
        self.entries = {}
        with self.fs.open(self.archive + "/_index") as f:
            for raw in f.read().decode().splitlines():
                t = raw.split()
                if not t:
                    continue
                path = _dec(t[0])
                if t[1] == "dir":
                    self.entries[path] = {"dir": True, "props": _dec(t[2]),
                                          "children": [_dec(c) for c in t[5:]]}
                else:
                    self.entries[path] = {"dir": False, "part": t[2], "start": int(t[3]),
                                          "len": int(t[4]), "props": _dec(t[5])}

    def _inner(self, path) -> str:
        p = str(path)
        if p.startswith("har://"):
            p = split_har_uri(p)[1]
        p = "/" + p.strip("/")
        return p

    def _uri(self, inner):
        return self.prefix + ("" if inner == "/" else inner)

    def _entry(self, path):
        e = self.entries.get(self._inner(path))
        if e is None:
            raise FileNotFoundError(path)
        return e

    def get_file_status(self, path) -> FileStatus:
        inner = self._inner(path)
        e = self._entry(inner)
        mtime = int(e["props"].split()[0]) / 1000.0 if e["props"] else 0.0
        return FileStatus(self._uri(inner), 0 if e["dir"] else e["len"], e["dir"],
                          self.fs.get_default_block_size(), mtime)

    getFileStatus = get_file_status  # noqa: N815

    def exists(self, path) -> bool:
        return self._inner(path) in self.entries

    def is_dir(self, path) -> bool:
        e = self.entries.get(self._inner(path))
        return bool(e and e["dir"])

    def list_status(self, path, filter_hidden=True):
        from ..fs import hidden
        inner = self._inner(path)
        e = self._entry(inner)
        if not e["dir"]:
            return [self.get_file_status(inner)]
        base = "" if inner == "/" else inner
        out = [self.get_file_status(f"{base}/{c}") for c in sorted(e["children"])]
        return [s for s in out if not (filter_hidden and hidden(s.path))]

    listStatus = list_status  # noqa: N815

    def listdir(self, path):
        return sorted(self._entry(path)["children"])

    def glob_status(self, pattern):
        import fnmatch
        pat = self._inner(pattern)
        return [self.get_file_status(p) for p in sorted(self.entries) if fnmatch.fnmatch(p, pat)]

    globStatus = glob_status  # noqa: N815

    def open(self, path, buffering=1 << 20):
        e = self._entry(path)
        if e["dir"]:
            raise IsADirectoryError(path)
        raw = self.fs.open(f"{self.archive}/{e['part']}")
        return io.BufferedReader(_Slice(raw, e["start"], e["len"]), max(8192, buffering))

    def get_default_block_size(self):
        return self.fs.get_default_block_size()

    getDefaultBlockSize = get_default_block_size  # noqa: N815

    def _ro(self, *a, **k):
        raise PermissionError("Hadoop archives are read-only")

    create = mkdirs = rename = delete = _ro


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr archive",
                                 description="archive -archiveName NAME -p <parent path> <src>* <dest>")
    ap.add_argument("-archiveName", required=True)
    ap.add_argument("-p", dest="parent", required=True)
    ap.add_argument("-m", dest="maps", type=int)
    ap.add_argument("paths", nargs="+")
    a = ap.parse_args(argv)
    srcs, dest = a.paths[:-1], a.paths[-1]
    create_archive(a.archiveName, strip_scheme(a.parent) if a.parent.startswith("file://")
                   else a.parent, srcs, dest, cluster=cluster, maps=a.maps, verbose=True)
    return 0
