"""FileSystem abstraction (hadoop-1.0.3/src/core/org/apache/hadoop/fs/FileSystem.java).

hbmr targets one 8×MI355X node, so HDFS is replaced by the local file system
(NVMe / page cache); ``file://`` and bare paths resolve to it.  The interface
keeps the Hadoop operations the MapReduce layer uses: listStatus with hidden
file filtering (``_``/``.`` prefixes, as FileInputFormat's hiddenFileFilter),
create/open/rename/delete/mkdirs and block-size metadata for split sizing.
"""
from __future__ import annotations

import glob as _glob
import os
import shutil
import stat
from dataclasses import dataclass

DEFAULT_BLOCK_SIZE = 64 * 1024 * 1024  # dfs.block.size default (hdfs-default.xml:259-260)


class Statistics:
    """Per-thread bytes read/written by scheme (FileSystem.Statistics,
    hadoop-1.0.3/src/core/org/apache/hadoop/fs/FileSystem.java): a task running
    on a thread snapshots them around its run to fill the FileSystemCounters
    (HDFS_BYTES_READ, FILE_BYTES_WRITTEN, ...)."""

    def __init__(self):
        import threading
        self._tl = threading.local()

    def _d(self):
        d = getattr(self._tl, "d", None)
        if d is None:
            d = self._tl.d = {}
        return d

    def add(self, scheme: str, read: int = 0, written: int = 0):
        d = self._d()
        r, w = d.get(scheme, (0, 0))
        d[scheme] = (r + read, w + written)

    def snapshot(self) -> dict:
        return dict(self._d())

    @staticmethod
    def delta(before: dict, after: dict) -> dict:
        out = {}
        for k, (r, w) in after.items():
            r0, w0 = before.get(k, (0, 0))
            if r - r0 or w - w0:
                out[k] = (r - r0, w - w0)
        return out


STATS = Statistics()


def strip_scheme(path) -> str:
    p = str(path)
    if p.startswith("file://"):
        p = p[len("file://"):]
    return p


@dataclass
class FileStatus:
    path: str
    length: int
    is_dir: bool
    block_size: int = DEFAULT_BLOCK_SIZE
    modification_time: float = 0.0

    def getLen(self):  # noqa: N802
        return self.length

    def getPath(self):  # noqa: N802
        return self.path

    def isDir(self):  # noqa: N802
        return self.is_dir

    def getBlockSize(self):  # noqa: N802
        return self.block_size


def hidden(name: str) -> bool:
    base = os.path.basename(name.rstrip("/"))
    return base.startswith("_") or base.startswith(".")


class LocalFileSystem:
    scheme = "file"

    def __init__(self, conf=None):
        self.conf = conf
        bs = conf.get_long("fs.local.block.size", DEFAULT_BLOCK_SIZE) if conf is not None else \
            DEFAULT_BLOCK_SIZE
        self.block_size = bs

    def get_file_status(self, path) -> FileStatus:
        p = strip_scheme(path)
        st = os.stat(p)
        return FileStatus(p, st.st_size, stat.S_ISDIR(st.st_mode), self.block_size, st.st_mtime)

    getFileStatus = get_file_status  # noqa: N815

    def exists(self, path) -> bool:
        return os.path.exists(strip_scheme(path))

    def is_dir(self, path) -> bool:
        return os.path.isdir(strip_scheme(path))

    def list_status(self, path, filter_hidden=True) -> list[FileStatus]:
        p = strip_scheme(path)
        if not os.path.isdir(p):
            return [self.get_file_status(p)]
        out = []
        # one stat per entry (DirEntry.stat follows links like os.stat)
        with os.scandir(p) as it:
            ents = sorted(it, key=lambda e: e.name)
        for e in ents:
            if filter_hidden and hidden(e.name):
                continue
            st = e.stat()
            out.append(FileStatus(os.path.join(p, e.name), st.st_size, stat.S_ISDIR(st.st_mode),
                                  self.block_size, st.st_mtime))
        return out

    listStatus = list_status  # noqa: N815

    def glob_status(self, pattern) -> list[FileStatus]:
        return [self.get_file_status(p) for p in sorted(_glob.glob(strip_scheme(pattern)))]

    globStatus = glob_status  # noqa: N815

    def mkdirs(self, path):
        os.makedirs(strip_scheme(path), exist_ok=True)
        return True

    def create(self, path, overwrite=True):
        p = strip_scheme(path)
        if not overwrite and os.path.exists(p):
            raise FileExistsError(p)
        d = os.path.dirname(p)
        if d:
            os.makedirs(d, exist_ok=True)
        return open(p, "wb")

    def open(self, path):
        return open(strip_scheme(path), "rb")

    def rename(self, src, dst) -> bool:
        s, d = strip_scheme(src), strip_scheme(dst)
        if not os.path.exists(s):
            return False
        parent = os.path.dirname(d)
        if parent:
            os.makedirs(parent, exist_ok=True)
        if os.path.isdir(d):
            d = os.path.join(d, os.path.basename(s.rstrip("/")))
        os.replace(s, d)
        return True

    def delete(self, path, recursive=True) -> bool:
        p = strip_scheme(path)
        if not os.path.exists(p):
            return False
        if os.path.isdir(p):
            if not recursive and os.listdir(p):
                raise OSError(f"{p} is a non-empty directory")
            shutil.rmtree(p)
        else:
            os.remove(p)
        return True

    def get_default_block_size(self):
        return self.block_size

    getDefaultBlockSize = get_default_block_size  # noqa: N815


def is_dfs(path) -> bool:
    """True for paths served by a non-local FileSystem (hdfs://, webhdfs://, har://)."""
    return str(path).startswith(("hdfs://", "webhdfs://", "har://"))


_HAR_CACHE: dict = {}


def get_fs(path=None, conf=None):
    """FileSystem for a path: ``hdfs://authority/...`` → hbmr.dfs, ``webhdfs://host:port/...``
    → its REST API (hbmr.dfs.webhdfs), ``har://...`` →
    a read-only Hadoop archive, else local."""
    p = str(path or "")
    if p.startswith("har://"):
        from ..tools.har import HarFileSystem, split_har_uri
        key = split_har_uri(p)[0]
        fs = _HAR_CACHE.get(key)
        if fs is None:
            fs = _HAR_CACHE[key] = HarFileSystem(p, conf)
        return fs
    if p.startswith("hdfs://"):
        from ..dfs.client import DistributedFileSystem, split_uri
        return DistributedFileSystem(split_uri(p)[0], conf)
    if p.startswith("webhdfs://"):
        from ..dfs.webhdfs import WebHdfsFileSystem, split_uri
        return WebHdfsFileSystem(split_uri(p)[0], conf)
    if "://" in p and not p.startswith("file://"):
        raise ValueError(f"unsupported filesystem scheme in {p!r} (use file:// or hdfs://)")
    return LocalFileSystem(conf)


# -- scheme-dispatching helpers for the MapReduce I/O paths ---------------------------------
def fopen(path, mode="rb", buffering=-1, conf=None):
    """open() for local paths and hdfs:// URIs (read or write, binary)."""
    if is_dfs(path):
        fs = get_fs(path, conf)
        return fs.open(path) if "r" in mode else fs.create(path)
    return open(strip_scheme(path), mode, buffering=buffering)


def mkdirs_fast(path):
    """os.makedirs for the common case that only the last level or two are
    missing: mkdir from the deepest level up as needed, no stat per level
    (os.makedirs stats every parent first)."""
    try:
        os.mkdir(path)
        return
    except FileExistsError:
        if os.path.isdir(path):
            return
        raise
    except FileNotFoundError:
        pass
    mkdirs_fast(os.path.dirname(path))
    try:
        os.mkdir(path)
    except FileExistsError:
        if not os.path.isdir(path):
            raise


def makedirs(path):
    if is_dfs(path):
        get_fs(path).mkdirs(path)
    else:
        os.makedirs(strip_scheme(path), exist_ok=True)


def exists(path) -> bool:
    return get_fs(path).exists(path) if is_dfs(path) else os.path.exists(strip_scheme(path))


def isdir(path) -> bool:
    return get_fs(path).is_dir(path) if is_dfs(path) else os.path.isdir(strip_scheme(path))


def listdir(path) -> list:
    return get_fs(path).listdir(path) if is_dfs(path) else os.listdir(strip_scheme(path))


def rmtree(path):
    if is_dfs(path):
        get_fs(path).delete(path, recursive=True)
    else:
        shutil.rmtree(strip_scheme(path), ignore_errors=True)


def replace(src, dst):
    """Move src over dst (files)."""
    if is_dfs(src):
        fs = get_fs(src)
        if fs.exists(dst):
            fs.delete(dst)
        fs.rename(src, dst)
    else:
        os.replace(strip_scheme(src), strip_scheme(dst))


def walk_files(root) -> list:
    """Relative paths of all files under root."""
    if not is_dfs(root):
        r = strip_scheme(root)
        return [os.path.relpath(os.path.join(d, f), r) for d, _, fs in os.walk(r) for f in fs]
    fs = get_fs(root)
    out, todo = [], [""]
    while todo:
        rel = todo.pop()
        for st in fs.list_status(os.path.join(root, rel) if rel else root, filter_hidden=False):
            name = os.path.join(rel, os.path.basename(st.path.rstrip("/")))
            (todo if st.is_dir else out).append(name)
    return out


def block_hosts(fs, path, start, length) -> list:
    """Hosts of the block holding ``start`` (FileInputFormat.getBlockIndex)."""
    if not hasattr(fs, "get_file_block_locations"):
        return []
    for off, blen, hosts in fs.get_file_block_locations(path, start, max(1, length)):
        if off <= start < off + max(blen, 1):
            return list(hosts)
    return []


FileSystem = LocalFileSystem
