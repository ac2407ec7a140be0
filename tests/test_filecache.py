"""DistributedCache: files and archives localized per tracker, visible to tasks."""
import os
import shutil

import pytest

from hbmr.filecache import DistributedCache
from hbmr.io.writable import Text
from hbmr.mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper
from hbmr.mapred.cluster import LocalCluster


class LookupMapper(Mapper):
    """Maps each word through a dictionary shipped in the cache."""

    def configure(self, job):
        files = DistributedCache.getLocalCacheFiles(job)
        archives = DistributedCache.getLocalCacheArchives(job)
        self.table = dict(line.split("=") for line in open(files[0]).read().split())
        self.extra = open(os.path.join(archives[0], "inner", "note.txt")).read().strip()
        work = job.get("mapred.cache.workdir")
        self.linked = os.path.exists(os.path.join(work, "dict"))

    def map(self, key, value, output, reporter):
        for w in str(value).split():
            output.collect(Text(self.table.get(w, "?")), Text(f"{self.extra}:{self.linked}"))


@pytest.mark.parametrize("where", ["local", "cluster"])
def test_cache_files_and_archives(tmp_path, where):
    (tmp_path / "dict.txt").write_text("a=1\nb=2\n")
    arch_src = tmp_path / "arch" / "inner"
    arch_src.mkdir(parents=True)
    (arch_src / "note.txt").write_text("from-archive\n")
    archive = shutil.make_archive(str(tmp_path / "bundle"), "zip", tmp_path / "arch")
    (tmp_path / "in").mkdir()
    (tmp_path / "in" / "x").write_text("a b c\n")
    job = JobConf()
    FileInputFormat.setInputPaths(job, str(tmp_path / "in"))
    FileOutputFormat.setOutputPath(job, str(tmp_path / "out"))
    job.set_mapper_class(LookupMapper)
    job.set_num_reduce_tasks(0)
    job.set_output_key_class(Text)
    job.set_output_value_class(Text)
    DistributedCache.addCacheFile(f"{tmp_path / 'dict.txt'}#dict", job)
    DistributedCache.addCacheArchive(archive, job)
    DistributedCache.createSymlink(job)
    cl = LocalCluster(JobConf(), num_trackers=2, cpu_slots=1) if where == "cluster" else None
    try:
        JobClient.runJob(job, cluster=cl, verbose=False)
    finally:
        if cl:
            cl.shutdown()
    out = "".join(open(tmp_path / "out" / f).read() for f in os.listdir(tmp_path / "out")
                  if f.startswith("part-"))
    assert sorted(out.split("\n")[:-1]) == ["1\tfrom-archive:True", "2\tfrom-archive:True",
                                            "?\tfrom-archive:True"]
