"""Out-of-core reduce shuffle/merge, reduce slow-start and the map SpillThread.

The reference: ReduceTask.ReduceCopier shuffleInMemory/shuffleToDisk
(ReduceTask.java:1646, 1775), InMemFSMergeThread (:2692), LocalFSMerger
(:2585), createKVIterator (:2421); reduce slow-start
(JobInProgress.java:879-881) with GetMapEventsThread (:2793); MapOutputBuffer's
SpillThread (MapTask.java:913-915, 1346).  With a tiny shuffle buffer and sort
buffer the job must produce byte-identical output to the in-memory run —
including the order of values within a key, which every merge keeps."""
import os
import random

from hbmr.examples.sleepjob import sleep_job_conf
from hbmr.io.writable import Text
from hbmr.mapred.api import Mapper, Reducer
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.formats import FileInputFormat, FileOutputFormat
from hbmr.mapred.jobconf import JobConf

SHUF = "hbmr.ShuffleCounters"


class WordPosMapper(Mapper):
    """(word, "offset:index") for every word: no combiner, many records."""

    def map(self, key, value, output, reporter):
        for i, w in enumerate(value.toString().split()):
            output.collect(Text(w), Text(f"{key.get()}:{i}"))


class ConcatReducer(Reducer):
    """Writes the values of a key in the order they arrive."""

    def reduce(self, key, values, output, reporter):
        output.collect(key, Text(",".join(v.toString() for v in values)))


def _input(d, files=3, lines=1500, seed=5):
    rng = random.Random(seed)
    words = [f"w{i:03d}" for i in range(300)]
    os.makedirs(d, exist_ok=True)
    for f in range(files):
        with open(os.path.join(d, f"in{f}.txt"), "w") as fh:
            for _ in range(lines):
                fh.write(" ".join(rng.choice(words) for _ in range(8)) + "\n")


def _job(inp, out, conf, reduces=2):
    job = JobConf(conf)
    job.set_job_name("wordpos")
    job.set_output_key_class(Text)
    job.set_output_value_class(Text)
    job.set_map_output_key_class(Text)
    job.set_map_output_value_class(Text)
    job.set_mapper_class(WordPosMapper)
    job.set_reducer_class(ConcatReducer)
    job.set_num_reduce_tasks(reduces)
    FileInputFormat.setInputPaths(job, inp)
    FileOutputFormat.setOutputPath(job, out)
    return job


def _run(tmp, name, **kw):
    conf = JobConf()
    for k, v in kw.items():
        conf.set(k, str(v))
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        rj = cl.submit_job(_job(str(tmp / "in"), str(tmp / name), conf))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        outs = {}
        for fn in sorted(os.listdir(tmp / name)):
            if fn.startswith("part-"):
                outs[fn] = (tmp / name / fn).read_bytes()
        return outs, rj.getCounters()


def test_tiny_buffers_spill_and_merge_on_disk_with_identical_output(tmp_path):
    _input(tmp_path / "in")
    # values reach a reducer in map-output arrival order; with every map done
    # before the copy starts that order is the maps' index order, deterministic
    det = {"mapred.map.tasks": 16, "mapred.reduce.slowstart.completed.maps": 1.0}
    ref, cs_ref = _run(tmp_path, "mem", **det)
    assert cs_ref.get(SHUF, "SEGMENTS_SHUFFLED_TO_DISK") == 0
    got, cs = _run(tmp_path, "disk", **{
        "hbmr.reduce.shuffle.memory.bytes": 48 << 10,   # 34 KB buffer, 8 KB max in memory
        "io.sort.factor": 3,                            # multi-pass merges
        "hbmr.io.sort.bytes": 24 << 10,                 # many map spills (SpillThread)
        **det})
    assert cs.get(SHUF, "SEGMENTS_SHUFFLED_TO_DISK") + cs.get(SHUF, "INMEM_MERGES") > 0
    assert cs.get(SHUF, "ONDISK_MERGES") > 0
    assert cs.get("hbmr.MapSpillCounters", "BACKGROUND_SPILLS") > 0
    assert got == ref
    # with slow-start the arrival order follows map completion: same records
    ss, _ = _run(tmp_path, "slowstart", **{"mapred.map.tasks": 16,
                                            "hbmr.reduce.shuffle.memory.bytes": 48 << 10,
                                            "io.sort.factor": 3})

    def norm(outs):
        return sorted((ln.split(b"\t")[0], tuple(sorted(ln.split(b"\t")[1].split(b","))))
                      for v in outs.values() for ln in v.splitlines())
    assert norm(ss) == norm(ref)


def test_synchronous_spill_matches_background_spill(tmp_path):
    _input(tmp_path / "in", files=2, lines=800)
    det = {"hbmr.io.sort.bytes": 16 << 10, "mapred.reduce.slowstart.completed.maps": 1.0}
    a, _ = _run(tmp_path, "async", **det)
    b, _ = _run(tmp_path, "sync", **det, **{"hbmr.map.spill.async": "false"})
    assert a == b


def test_reduce_slow_start_overlaps_the_map_phase():
    conf = JobConf()
    conf.set_float("mapred.reduce.slowstart.completed.maps", 0.1)
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(sleep_job_conf(maps=10, reduces=1, map_ms=60, reduce_ms=1,
                                          base=conf))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        jip = rj._impl.jip
        red = next(iter(jip.reduces[0].attempts.values()))
        # the reduce started while maps were still running and copied the rest
        # through completion events
        assert red.start < jip.t_maps_done - 0.05
        assert len(jip.completion_events) == 10


def test_reduce_waits_for_all_maps_without_slow_start():
    conf = JobConf()
    conf.set_float("mapred.reduce.slowstart.completed.maps", 1.0)
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(sleep_job_conf(maps=4, reduces=1, map_ms=30, reduce_ms=1, base=conf))
        rj.waitForCompletion(60)
        assert rj.isSuccessful()
        jip = rj._impl.jip
        red = next(iter(jip.reduces[0].attempts.values()))
        assert red.start >= jip.t_maps_done - 1e-3
