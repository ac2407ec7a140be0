"""Task child processes (TaskRunner/JvmManager/Child, SURVEY.md §2.2 "Task launch"):
isolation, process reuse (mapred.job.reuse.jvm.num.tasks), crash → retry,
kill on timeout, memory-limit kills (TaskMemoryManagerThread), child env and
per-attempt userlogs."""
import collections
import os

from hbmr.io.writable import LongWritable, Text
from hbmr.mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from hbmr.mapred.cluster import LocalCluster
from hbmr.models import wordcount

JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"


def _words(tmp_path, files=4):
    d = tmp_path / "in"
    d.mkdir()
    cnt = collections.Counter()
    for i in range(files):
        lines = [" ".join(f"w{(i * 3 + j + t) % 11}" for t in range(j % 5)) for j in range(60)]
        (d / f"p{i}").write_text("\n".join(lines) + "\n")
        for ln in lines:
            cnt.update(ln.split())
    return d, cnt


def _read(out):
    res = {}
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            for line in open(os.path.join(out, fn)):
                k, v = line.rstrip("\n").split("\t")
                res[k] = v
    return res


class PidMapper(Mapper):
    """Emits (pid, env var) once per task; prints to stdout (userlogs)."""

    def configure(self, job):
        self.done = False

    def map(self, key, value, output, reporter):
        if not self.done:
            self.done = True
            print("hello from", os.getpid())
            output.collect(Text(str(os.getpid())), Text(os.environ.get("HBMR_TEST_VAR", "-")))


class FirstReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(key, next(iter(values)))


class CrashOnceMapper(Mapper):
    """Kills its own process on the first attempt of partition 0."""

    def configure(self, job):
        self.first = job.get("mapred.task.id").endswith("_m_000000_0")

    def map(self, key, value, output, reporter):
        if self.first:
            os._exit(7)
        output.collect(Text("x"), Text("1"))


class HogMapper(Mapper):
    def map(self, key, value, output, reporter):
        import time
        self.blob = bytearray(400 << 20)
        for i in range(0, len(self.blob), 4096):
            self.blob[i] = 1
        time.sleep(30)


class SleepMapper(Mapper):
    def map(self, key, value, output, reporter):
        import time
        time.sleep(60)


def _pid_job(inp, out, reuse, maps=4):
    job = JobConf()
    job.set_job_name("pids")
    job.set("hbmr.task.child.process", "true")
    job.set_int("mapred.job.reuse.jvm.num.tasks", reuse)
    job.set("mapred.child.env", "HBMR_TEST_VAR=child-env-ok")
    job.set_mapper_class(PidMapper)
    job.set_reducer_class(FirstReducer)
    job.set_output_key_class(Text)
    job.set_output_value_class(Text)
    job.set_num_map_tasks(maps)
    job.set_num_reduce_tasks(1)
    FileInputFormat.setInputPaths(job, str(inp))
    FileOutputFormat.setOutputPath(job, str(out))
    return job


def test_wordcount_in_child_processes(tmp_path):
    inp, cnt = _words(tmp_path)
    with LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) as cl:
        job = wordcount.make_job(str(inp), str(tmp_path / "out"), reduces=2)
        job.set("mapred.task.isolation", "process")
        job.set_num_map_tasks(4)
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
        spawned = sum(t.child_manager.spawned for t in cl.trackers if t.child_manager)
    assert {k: int(v) for k, v in _read(tmp_path / "out").items()} == dict(cnt)
    assert rj.getCounters().get("org.apache.hadoop.mapred.Task$Counter",
                                "MAP_INPUT_RECORDS") == 240
    assert spawned >= 6            # 4+ maps and 2 reduces, a fresh process each (reuse = 1)


def test_process_per_task_and_reuse(tmp_path):
    inp, _ = _words(tmp_path)
    me = str(os.getpid())
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=1) as cl:
        JobClient.runJob(_pid_job(inp, tmp_path / "o1", reuse=1), cluster=cl, verbose=False)
        fresh = _read(tmp_path / "o1")
        JobClient.runJob(_pid_job(inp, tmp_path / "o2", reuse=-1), cluster=cl, verbose=False)
        reused = _read(tmp_path / "o2")
        logs = os.path.join(cl.trackers[0].local_dir, "userlogs")
        outs = [open(os.path.join(logs, a, "stdout")).read() for a in os.listdir(logs)
                if "_m_" in a]
    assert me not in fresh and me not in reused
    assert len(fresh) == 4                     # one process per map attempt
    assert len(reused) == 1                    # one slot, unlimited reuse: one process
    assert set(fresh.values()) == {"child-env-ok"}
    assert any("hello from" in o for o in outs)


def test_child_crash_fails_attempt_then_retry_succeeds(tmp_path):
    inp, _ = _words(tmp_path, files=2)
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        job = _pid_job(inp, tmp_path / "out", reuse=1, maps=2)
        job.set_mapper_class(CrashOnceMapper)
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
    assert rj.isSuccessful()
    assert rj.getCounters().get(JIP, "NUM_FAILED_MAPS") == 1


def test_memory_limit_kills_task(tmp_path):
    inp, _ = _words(tmp_path, files=1)
    conf = JobConf()
    conf.set_int("mapred.tasktracker.taskmemorymanager.monitoring-interval", 200)
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        job = _pid_job(inp, tmp_path / "out", reuse=1, maps=1)
        job.set_mapper_class(HogMapper)
        job.set_int("mapred.job.map.memory.mb", 256)
        job.set_int("mapred.map.max.attempts", 1)
        rj = cl.submit_job(job)
        rj.waitForCompletion()
    assert not rj.isSuccessful()
    assert "beyond memory-limits" in (rj.getFailureInfo() or "")


def test_timeout_kills_child(tmp_path):
    inp, _ = _words(tmp_path, files=1)
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=1) as cl:
        job = _pid_job(inp, tmp_path / "out", reuse=1, maps=1)
        job.set_mapper_class(SleepMapper)
        job.set_int("mapred.task.timeout", 1500)
        job.set_int("mapred.map.max.attempts", 1)
        rj = cl.submit_job(job)
        rj.waitForCompletion()
        import time
        deadline = time.time() + 10
        while time.time() < deadline:
            pids = [c.pid for t in cl.trackers if t.child_manager
                    for c in list(t.child_manager._busy)]
            if not pids:
                break
            time.sleep(0.05)
    assert not rj.isSuccessful()
    assert "failed to report status" in (rj.getFailureInfo() or "")
    assert not pids                    # the hung child was SIGKILLed


def test_local_runner_parallel_child_maps(tmp_path):
    inp, cnt = _words(tmp_path)
    conf = JobConf()
    conf.set("mapred.job.tracker", "local")
    conf.set_int("mapred.local.map.tasks.maximum", 3)
    conf.set("mapred.task.isolation", "process")
    job = wordcount.make_job(str(inp), str(tmp_path / "out"), reduces=1, conf=conf)
    rj = JobClient.runJob(job, verbose=False)
    assert {k: int(v) for k, v in _read(tmp_path / "out").items()} == dict(cnt)
    assert rj.getCounters().get("org.apache.hadoop.mapred.Task$Counter",
                                "MAP_INPUT_RECORDS") == 240


def test_local_runner_child_pool_is_warm_across_jobs(tmp_path):
    """Parallel local maps in child processes reuse one warm pool across jobs
    (tasks carry their own conf): the second job starts no interpreter, and
    its output is still right."""
    from hbmr.mapred import local_runner as LR
    inp, cnt = _words(tmp_path)
    conf = JobConf()
    conf.set("mapred.job.tracker", "local")
    conf.set_int("mapred.local.map.tasks.maximum", 3)
    conf.set("mapred.task.isolation", "process")
    conf.set("mapred.child.env", "HBMR_POOL_TEST=1")     # a pool of its own
    spawned = []
    for i in range(2):
        job = wordcount.make_job(str(inp), str(tmp_path / f"out{i}"), reduces=1, conf=conf)
        rj = JobClient.runJob(job, verbose=False)
        assert rj.isSuccessful()
        assert {k: int(v) for k, v in _read(tmp_path / f"out{i}").items()} == dict(cnt)
        mgrs = [m for k, (m, c) in LR._POOLS.items() if c.get("mapred.child.env") ==
                "HBMR_POOL_TEST=1"]
        assert len(mgrs) == 1
        spawned.append(mgrs[0].spawned)
    assert 1 <= spawned[0] <= 3 and spawned[1] == spawned[0]
