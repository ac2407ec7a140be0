"""DistributedCache: side files and archives shipped to every task
(hadoop-1.0.3 filecache/{DistributedCache,TrackerDistributedCacheManager,
TaskDistributedCacheManager}.java).

A job lists URIs in ``mapred.cache.files`` / ``mapred.cache.archives``
(``path#linkname`` fragments name the symlink).  Each TaskTracker localizes a
job's cache once, into ``<local dir>/<job id>/cache`` (files hard-linked or
copied; archives — zip, tar, tgz, jar — unpacked), and publishes the local
paths in ``mapred.cache.localFiles`` / ``mapred.cache.localArchives`` of the
conf its tasks see; with ``mapred.create.symlink=yes`` the fragment names are
symlinked into the job's working directory.  Localized copies are shared by
every task of the job on that tracker and removed with the job.

(For GPU split jobs the per-iteration side data — e.g. K-Means centroids —
stays resident in HBM instead; see hbmr.models.kmeans.CentroidStore.)
"""
from __future__ import annotations

import os
import shutil
import threading

FILES, ARCHIVES = "mapred.cache.files", "mapred.cache.archives"
LOCAL_FILES, LOCAL_ARCHIVES = "mapred.cache.localFiles", "mapred.cache.localArchives"
SYMLINK = "mapred.create.symlink"


def _strip(uri: str) -> str:
    return uri[5:] if uri.startswith("file:") else uri


def _split(uri: str):
    path, _, frag = uri.partition("#")
    return _strip(path), frag or os.path.basename(_strip(path))


class DistributedCache:
    @staticmethod
    def _add(conf, key, uri):
        old = conf.get(key)
        conf.set(key, (old + "," if old else "") + str(uri))

    @staticmethod
    def addCacheFile(uri, conf):  # noqa: N802
        DistributedCache._add(conf, FILES, uri)

    @staticmethod
    def addCacheArchive(uri, conf):  # noqa: N802
        DistributedCache._add(conf, ARCHIVES, uri)

    @staticmethod
    def setCacheFiles(uris, conf):  # noqa: N802
        conf.set(FILES, ",".join(map(str, uris)))

    @staticmethod
    def setCacheArchives(uris, conf):  # noqa: N802
        conf.set(ARCHIVES, ",".join(map(str, uris)))

    @staticmethod
    def getCacheFiles(conf):  # noqa: N802
        v = conf.get(FILES)
        return v.split(",") if v else []

    @staticmethod
    def getCacheArchives(conf):  # noqa: N802
        v = conf.get(ARCHIVES)
        return v.split(",") if v else []

    @staticmethod
    def getLocalCacheFiles(conf):  # noqa: N802
        v = conf.get(LOCAL_FILES)
        return v.split(",") if v else []

    @staticmethod
    def getLocalCacheArchives(conf):  # noqa: N802
        v = conf.get(LOCAL_ARCHIVES)
        return v.split(",") if v else []

    @staticmethod
    def createSymlink(conf):  # noqa: N802
        conf.set(SYMLINK, "yes")

    @staticmethod
    def addFileToClassPath(path, conf):  # noqa: N802
        """Python analogue: the file/dir is put on sys.path of the tasks."""
        DistributedCache._add(conf, "mapred.job.classpath.files", path)
        DistributedCache.addCacheFile(path, conf)


class TrackerCacheManager:
    """Per-TaskTracker localization (once per job)."""

    def __init__(self, local_dir):
        self.local_dir = local_dir
        self.lock = threading.Lock()
        self.done: dict = {}

    def localize(self, job_id: str, conf) -> None:
        files = DistributedCache.getCacheFiles(conf)
        archives = DistributedCache.getCacheArchives(conf)
        if not files and not archives:
            return
        with self.lock:
            cached = self.done.get(job_id)
            if cached is None:
                cached = self._localize(job_id, files, archives, conf)
                self.done[job_id] = cached
        lf, la = cached
        conf.set(LOCAL_FILES, ",".join(lf))
        conf.set(LOCAL_ARCHIVES, ",".join(la))
        cp = conf.get("mapred.job.classpath.files")
        if cp:
            import sys
            for p in lf:
                if p not in sys.path and any(os.path.basename(p) == os.path.basename(c)
                                             for c in cp.split(",")):
                    sys.path.insert(0, p if os.path.isdir(p) else os.path.dirname(p))

    def _localize(self, job_id, files, archives, conf):
        base = os.path.join(self.local_dir, job_id, "cache")
        work = os.path.join(self.local_dir, job_id, "work")
        os.makedirs(base, exist_ok=True)
        os.makedirs(work, exist_ok=True)
        lf, la = [], []
        for i, uri in enumerate(files):
            src, name = _split(uri)
            dst = os.path.join(base, f"f{i}", os.path.basename(src))
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            if os.path.isdir(src):
                shutil.copytree(src, dst)
            else:
                try:
                    os.link(src, dst)
                except OSError:
                    shutil.copy2(src, dst)
            lf.append(dst)
            self._symlink(conf, work, dst, name)
        for i, uri in enumerate(archives):
            src, name = _split(uri)
            dst = os.path.join(base, f"a{i}")
            fmt = "zip" if src.endswith((".zip", ".jar")) else None
            shutil.unpack_archive(src, dst, format=fmt)
            la.append(dst)
            self._symlink(conf, work, dst, name)
        conf.set("mapred.cache.workdir", work)
        return lf, la

    @staticmethod
    def _symlink(conf, work, target, name):
        if str(conf.get(SYMLINK, "no")).lower() == "yes":
            link = os.path.join(work, name)
            if not os.path.lexists(link):
                os.symlink(target, link)

    def release(self, job_id):
        with self.lock:
            self.done.pop(job_id, None)
        shutil.rmtree(os.path.join(self.local_dir, job_id, "cache"), ignore_errors=True)
