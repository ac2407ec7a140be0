"""Map and reduce task execution (the CPU data path).

MapTask (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/MapTask.java):
  record reader -> MapRunnable -> MapOutputBuffer (collect; sort by
  (partition, key) when the buffer passes ``io.sort.mb × io.sort.spill.percent``;
  combiner per spill; spills merged with ``io.sort.factor`` fan-in into
  ``file.out`` + ``file.out.index``, MapTask.java:869-1621), or straight to the
  OutputFormat when there are no reducers (DirectMapOutputCollector, :805).

ReduceTask (ReduceTask.java:348): fetch each map's segment of this partition
(on one node the map outputs are local files — the reference's HTTP fetch,
ReduceTask.java:1231-1775, becomes a read), k-way merge (Merger.java:236-365),
group by the grouping comparator and call the Reducer; output goes through the
OutputCommitter's task work dir.

The GPU data path (split-level GPU mappers, RCCL shuffle) lives in
:mod:`hbmr.gpu`; it plugs in at the same MapTask boundary.
"""
from __future__ import annotations

import heapq
import io
import itertools
import logging
import os
import threading
import time

import numpy as np

from ..fs import mkdirs_fast
from ..io.compress import get_codec
from ..io.ifile import IFileWriter, SpillRecord, read_segment
from ..io.serializer import to_bytes
from ..io.writable import payload_serializer, serialize_in_place
from ..utils.reflection import new_instance
from ..utils.trace import TRACE
from . import counters as C
from . import mapoutput, sortbuf
from .api import OutputCollector, Reporter
from .committer import FileOutputCommitter
from .formats import FileSplit

log = logging.getLogger("hbmr.task")


class TaskReporter(Reporter):
    """Collects progress/status/counters of one task attempt (Task.TaskReporter,
    Task.java:554); the TaskTracker reads ``snapshot()`` on each heartbeat."""

    def __init__(self, split=None, listener=None):
        self.counters = C.Counters()
        self.status = ""
        self.progress_value = 0.0
        self.split = split
        self.last_progress = time.time()
        self.listener = listener
        self._lock = threading.Lock()

    def setStatus(self, status):  # noqa: N802
        self.status = status
        self.progress()

    def progress(self):
        self.last_progress = time.time()

    def set_progress(self, p):
        self.progress_value = float(p)
        self.progress()

    def getCounter(self, group, name=None):  # noqa: N802
        if name is None and isinstance(group, tuple):
            group, name = group
        return self.counters.find_counter(group, name)

    def incrCounter(self, group, name, amount=1):  # noqa: N802
        self.counters.incr(group, name, amount)

    def getInputSplit(self):  # noqa: N802
        return self.split

    def getProgress(self):  # noqa: N802
        return self.progress_value


class _Interrupted(Exception):
    pass


class Task:
    """Base of MapTask / ReduceTask: identity, placement and the commit protocol."""

    def __init__(self, job, attempt_id, partition: int):
        self.job = job
        self.attempt_id = attempt_id
        self.partition = partition
        self.reporter = TaskReporter()
        self.run_on_gpu = False        # Task.runOnGPU (Task.java:169-207)
        self.gpu_device_id = -1        # Task.GPUDeviceId
        self.kill_event = threading.Event()
        self.local_dir = None
        self.start_time = 0.0
        self.finish_time = 0.0

    @property
    def is_map(self):
        return self.attempt_id.is_map

    def runOnGPU(self):  # noqa: N802
        return self.run_on_gpu

    def setRunOnGPU(self, b):  # noqa: N802
        self.run_on_gpu = bool(b)

    def setGPUDeviceId(self, d):  # noqa: N802
        self.gpu_device_id = int(d)

    def check_killed(self):
        if self.kill_event.is_set():
            raise _Interrupted(str(self.attempt_id))

    def committer(self):
        cls = self.job.get_output_committer()
        return cls() if isinstance(cls, type) else FileOutputCommitter()

    def _task_conf(self):
        """Per-attempt JobConf with the committer's work dir set."""
        conf = type(self.job)(self.job)
        wp = None
        com = self.committer()
        if hasattr(com, "work_path"):
            wp = com.work_path(self.job, self.attempt_id)
        if wp:
            conf.set("mapred.work.output.dir", wp)
        conf.set("mapred.task.id", str(self.attempt_id))
        conf.set("mapred.task.partition", self.partition)
        conf.set("mapred.task.is.map", self.is_map)
        return conf


# ------------------------------------------------------------------- map side
class _DirectCollector(OutputCollector):
    def __init__(self, writer, reporter):
        self.writer = writer
        self.reporter = reporter
        self.n = 0

    def collect(self, key, value):
        self.writer.write(key, value)
        self.n += 1

    def flush(self):
        self.writer.close(self.reporter)
        self.reporter.incrCounter(C.TASK_GROUP, C.MAP_OUTPUT_RECORDS, self.n)


class _ListCollector(OutputCollector):
    def __init__(self):
        self.out = []

    def collect(self, key, value):
        self.out.append((key, value))


def group_sorted(records, group_key, vcls):
    """records: iterable of (sort_key, kb, vb) sorted; yields (kb, values_iter)."""
    it = iter(records)
    try:
        first = next(it)
    except StopIteration:
        return
    pending = [first]

    while pending:
        head = pending.pop()
        gk = group_key(head[1])
        state = {"next": None}

        def values(head=head, gk=gk, state=state):
            yield vcls.deserialize(head[2])
            for rec in it:
                if group_key(rec[1]) != gk:
                    state["next"] = rec
                    return
                yield vcls.deserialize(rec[2])

        vals = values()
        yield head[1], vals
        # drain unconsumed values of this group
        for _ in vals:
            pass
        if state["next"] is not None:
            pending.append(state["next"])


def run_combiner(combiner_cls, job, kcls, vcls, records, reporter):
    """Apply the combiner to sorted (sk, kb, vb) records of ONE partition.
    Returns a new sorted list of (sk, kb, vb)."""
    comb = new_instance(combiner_cls, job)
    col = _ListCollector()
    sort_key = job.get_output_key_comparator()
    group_key = job.get_output_value_grouping_comparator()
    recs = list(records)
    nin = len(recs)
    for kb, vals in group_sorted(recs, group_key, vcls):
        comb.reduce(kcls.deserialize(kb), vals, col, reporter)
    comb.close()
    reporter.incrCounter(C.TASK_GROUP, C.COMBINE_INPUT_RECORDS, nin)
    reporter.incrCounter(C.TASK_GROUP, C.COMBINE_OUTPUT_RECORDS, len(col.out))
    out = []
    for k, v in col.out:
        kb = to_bytes(k, kcls)
        out.append((sort_key(kb), kb, to_bytes(v, vcls)))
    out.sort(key=lambda r: r[0])
    return out


class MapOutputBuffer(OutputCollector):
    """Collect → partition → sort → (combine) → spill, then merge spills."""

    #: the job-level settings below, per job conf object (a TaskTracker's
    #: JobState conf, shared by the job's attempts, whose task confs differ
    #: only in task keys): ~20 typed conf reads and class resolutions were a
    #: quarter of a small Pipes map's task-thread time (config 2)
    _SETTINGS = ("R", "kcls", "vcls", "sort_key", "pcls", "combiner_cls", "soft_limit", "factor",
                 "min_spills_for_combine", "codec", "mem_max_conf", "mem_total", "kind",
                 "native_hash", "spill_async")

    @staticmethod
    def _settings(job) -> dict:
        sort_bytes = job.get_int("hbmr.io.sort.bytes", job.get_int("io.sort.mb", 100) << 20)
        kind = sortbuf.key_kind(job)
        return {
            "R": job.get_num_reduce_tasks(),
            "kcls": job.get_map_output_key_class(),
            "vcls": job.get_map_output_value_class(),
            "sort_key": job.get_output_key_comparator(),
            "pcls": job.get_partitioner_class(),
            "combiner_cls": job.get_combiner_class(),
            "soft_limit": int(sort_bytes * job.get_float("io.sort.spill.percent", 0.8)),
            "factor": max(2, job.get_int("io.sort.factor", 10)),
            "min_spills_for_combine": job.get_int("min.num.spills.for.combine", 3),
            "codec": get_codec(job.get("mapred.map.output.compression.codec",
                                       "org.apache.hadoop.io.compress.DefaultCodec"))
            if job.get_compress_map_output() else None,
            "mem_max_conf": job.get_long(mapoutput.MAX_KEY, 4 << 20),
            "mem_total": job.get_long(mapoutput.TOTAL_KEY, 256 << 20),
            # native sort path (hbmr/mapred/sortbuf.py): serialised records
            # only, partition + sort + group + IFile encode per spill in C++
            "kind": kind,
            "native_hash": kind is not None and sortbuf.hash_partitioned(job),
            "spill_async": job.get_boolean("hbmr.map.spill.async", True),
        }

    def __init__(self, task: "MapTask", job, reporter, out_dir):
        self.task = task
        self.job = job
        self.reporter = reporter
        base = getattr(task, "job", None)
        st = None
        if base is not None and base is not job:
            cached = base.__dict__.get("_mob_settings")
            # (keyed by the shared conf's props dict and mutation count: a
            # conf changed since, or rebuilt, recomputes them)
            if cached is not None and cached[0] is base._props and cached[1] == base._gen:
                st = cached[2]
        if st is None:
            st = self._settings(job)
            if base is not None and base is not job:
                base._mob_settings = (base._props, base._gen, st)
        self.R, self.kcls, self.vcls = st["R"], st["kcls"], st["vcls"]
        self.sort_key = st["sort_key"]
        self.partitioner = new_instance(st["pcls"], job)
        self.combiner_cls = st["combiner_cls"]
        self.soft_limit, self.factor = st["soft_limit"], st["factor"]
        self.min_spills_for_combine = st["min_spills_for_combine"]
        self.codec = st["codec"]
        self.out_dir = out_dir
        self._dir_made = False
        # a small single-spill output stays in this process's memory when the
        # tracker's reduces read here (hbmr/mapred/mapoutput.py)
        self.mem_max = st["mem_max_conf"] if getattr(task, "memory_outputs", False) else 0
        self.mem_total = st["mem_total"]
        self._to_memory = False
        self.kind = st["kind"]
        self.native_hash = st["native_hash"]
        self.keys: list = []
        self.vals: list = []
        self.parts: list = []
        self.buf: list = []
        if self.native_hash:
            self.collect = self._collect_native
        self.buf_bytes = 0
        self.spills: list[tuple[str, SpillRecord]] = []
        self.n_out = 0
        self.bytes_out = 0
        # SpillThread (MapTask.java:913-915, 1346): a full buffer is sorted and
        # spilled in the background while map() keeps collecting into a fresh
        # one; collect blocks only if that one fills while a spill is running
        self.spill_async = st["spill_async"]
        self._spill_thread = None
        self._spill_error = None
        self._direct_final = False

    def _spill_path(self, idx):
        # a map's only spill is written under the final name (no rename pair)
        return os.path.join(self.out_dir, "file.out" if self._direct_final else f"spill{idx}.out")

    def _ensure_dir(self):
        if not self._dir_made:
            # the attempt's dir, then its output dir: two mkdirs (os.makedirs
            # stats every level first)
            mkdirs_fast(os.path.dirname(self.out_dir))
            mkdirs_fast(self.out_dir)
            self._dir_made = True

    def _open_spill(self, path):
        """A spill's target: its file, or a buffer for an in-memory output."""
        if self._to_memory:
            return io.BytesIO()
        self._ensure_dir()
        return open(path, "wb")

    def _commit_spill(self, path, f, rec, crc_pending=False):
        """Close a spill: its index file next to it, or both held in memory
        (a store over its cap gets the files after all — with their CRCs,
        which an in-memory output skipped: ``crc_pending``)."""
        if self._to_memory:
            # (f: the spill's BytesIO, or its joined bytes already)
            data = f if isinstance(f, bytes) else f.getvalue()
            if mapoutput.STORE.put(path, data, rec, self.mem_total):
                return
            if crc_pending:
                data = sortbuf.fill_crcs(data, rec)
            self._ensure_dir()
            with open(path, "wb") as out:
                out.write(data)
            size = len(data)
        else:
            size = f.tell()
            f.close()
        rec.write(path + ".index")
        _fs_written(path, size)

    def collect(self, key, value):
        if not isinstance(key, self.kcls):
            raise TypeError(f"Type mismatch in key from map: expected {self.kcls.__name__}, "
                            f"received {type(key).__name__}")
        if not isinstance(value, self.vcls):
            raise TypeError(f"Type mismatch in value from map: expected {self.vcls.__name__}, "
                            f"received {type(value).__name__}")
        kb = to_bytes(key, self.kcls)
        vb = to_bytes(value, self.vcls)
        if self.native_hash:
            self.keys.append(kb)
            self.vals.append(vb)
        else:
            part = self.partitioner.getPartition(key, value, self.R)
            if not 0 <= part < self.R:
                raise ValueError(f"Illegal partition for {key!r} ({part})")
            if self.kind is not None:
                self.keys.append(kb)
                self.vals.append(vb)
                self.parts.append(part)
            else:
                self.buf.append((part, self.sort_key(kb), kb, vb))
        sz = len(kb) + len(vb) + 16  # 16 B accounting per record (MapTask.java:890-903)
        self.buf_bytes += sz
        self.n_out += 1
        self.bytes_out += len(kb) + len(vb)
        if self.buf_bytes >= self.soft_limit:
            self._spill_full()

    def _collect_native(self, key, value):
        """collect() when partitioning is batched in C++: serialise and append."""
        kc = self.kcls
        if key.__class__ is not kc and not isinstance(key, kc):
            raise TypeError(f"Type mismatch in key from map: expected {kc.__name__}, "
                            f"received {type(key).__name__}")
        vc = self.vcls
        if value.__class__ is not vc and not isinstance(value, vc):
            raise TypeError(f"Type mismatch in value from map: expected {vc.__name__}, "
                            f"received {type(value).__name__}")
        kb = key.serialize()
        vb = value.serialize()
        self.keys.append(kb)
        self.vals.append(vb)
        n = len(kb) + len(vb)
        self.bytes_out += n
        self.buf_bytes += n + 16   # 16 B accounting per record (MapTask.java:890-903)
        if self.buf_bytes >= self.soft_limit:
            self._spill_full()

    def raw_sink(self):
        """A ``sink(k, v, part)`` taking a Pipes child's OUTPUT frames as they
        came off the wire (``part``: a PARTITIONED_OUTPUT's partition, else
        None) and appending their serialised form without building Writables
        (the uplink's per-record cost) — or None when the key or value class
        is not one whose wire form is its payload (Text, BytesWritable)."""
        kser, vser = payload_serializer(self.kcls), payload_serializer(self.vcls)
        if kser is None or vser is None:
            return None
        R, native_hash, kind = self.R, self.native_hash, self.kind

        def sink(k, v, part):
            kb = kser(k)
            # (a large value off the uplink: serialised in its own buffer;
            # the native path takes any bytes-like value)
            vb = serialize_in_place(vser, v) if kind is not None and \
                v.__class__ is memoryview else vser(v if v.__class__ is not memoryview
                                                   else bytes(v))
            if native_hash:
                self.keys.append(kb)
                self.vals.append(vb)
            else:
                if part is None:
                    part = 0 if R == 1 else self.partitioner.getPartition(
                        self.kcls.deserialize(kb), self.vcls.deserialize(bytes(vb)), R)
                if not 0 <= part < R:
                    raise ValueError(f"Illegal partition for {k!r} ({part})")
                if kind is not None:
                    self.keys.append(kb)
                    self.vals.append(vb)
                    self.parts.append(part)
                else:
                    self.buf.append((part, self.sort_key(kb), kb, vb))
                self.n_out += 1
            n = len(kb) + len(vb)
            self.bytes_out += n
            self.buf_bytes += n + 16
            if self.buf_bytes >= self.soft_limit:
                self._spill_full()
        return sink

    def _spill_full(self):
        """The buffer passed io.sort.spill.percent: hand it to the spill thread."""
        if not self.spill_async:
            self.sort_and_spill()
            return
        self._wait_spill()
        taken = (self.keys, self.vals, self.parts, self.buf)
        self.keys, self.vals, self.parts, self.buf = [], [], [], []
        self.buf_bytes = 0

        def run():
            try:
                self._spill(*taken)
            except BaseException as e:  # noqa: BLE001
                self._spill_error = e
        self._spill_thread = threading.Thread(target=run, daemon=True,
                                              name=f"SpillThread-{self.task.attempt_id}")
        self._spill_thread.start()
        self.reporter.incrCounter("hbmr.MapSpillCounters", "BACKGROUND_SPILLS", 1)

    def _wait_spill(self):
        t = self._spill_thread
        if t is not None:
            t.join()
            self._spill_thread = None
        if self._spill_error is not None:
            e, self._spill_error = self._spill_error, None
            raise e

    @staticmethod
    def _sorted_partitions(buf, R):
        buf.sort(key=lambda r: (r[0], r[1]))
        parts = [[] for _ in range(R)]
        for p, sk, kb, vb in buf:
            parts[p].append((sk, kb, vb))
        return parts

    def sort_and_spill(self):
        """Spill the current buffer now (in the caller's thread)."""
        self._wait_spill()
        taken = (self.keys, self.vals, self.parts, self.buf)
        self.keys, self.vals, self.parts, self.buf = [], [], [], []
        self.buf_bytes = 0
        self._spill(*taken)

    def _spill(self, keys, vals, parts_l, buf):
        if self.kind is not None:
            return self._sort_and_spill_native(keys, vals, parts_l)
        if not buf and self.spills:
            return
        self.task.check_killed()
        parts = self._sorted_partitions(buf, self.R)
        idx = len(self.spills)
        path = self._spill_path(idx)
        rec = SpillRecord(self.R)
        spilled = 0
        f = self._open_spill(path)
        try:
            for p in range(self.R):
                recs = parts[p]
                if self.combiner_cls is not None and recs:
                    recs = run_combiner(self.combiner_cls, self.job, self.kcls, self.vcls, recs,
                                        self.reporter)
                w = IFileWriter(f, self.codec)
                for _sk, kb, vb in recs:
                    w.append(kb, vb)
                spilled += len(recs)
                rec.put(p, *w.close())
        except BaseException:
            f.close()
            raise
        self._commit_spill(path, f, rec)
        self.spills.append((path, rec))
        self.reporter.incrCounter(C.TASK_GROUP, C.SPILLED_RECORDS, spilled)

    # -- native path ------------------------------------------------------------------------
    def _combine_native(self, b, perm, lo, hi):
        """Run the combiner over the key groups of perm[lo:hi]; returns the IFile
        body of its (re-sorted) output and the record count."""
        ends = b.group_ends(self.kind, perm, lo, hi)
        comb = new_instance(self.combiner_cls, self.job)
        col = _ListCollector()
        kdes, vdes = self.kcls.deserialize, self.vcls.deserialize
        pl = perm.tolist()
        a = lo
        for e in ends.tolist():
            comb.reduce(kdes(b.key(pl[a])), (vdes(b.value(r)) for r in pl[a:e]), col,
                        self.reporter)
            a = e
        comb.close()
        self.reporter.incrCounter(C.TASK_GROUP, C.COMBINE_INPUT_RECORDS, hi - lo)
        self.reporter.incrCounter(C.TASK_GROUP, C.COMBINE_OUTPUT_RECORDS, len(col.out))
        ob = sortbuf.Batch.from_lists([to_bytes(k, self.kcls) for k, _ in col.out],
                                      [to_bytes(v, self.vcls) for _, v in col.out])
        operm = ob.sort(self.kind, np.zeros(ob.n, np.int32))
        return ob.ifile_body(operm, 0, ob.n), ob.n

    def _sort_and_spill_native(self, keys, vals, parts_l):
        if not keys and self.spills:
            return
        self.task.check_killed()
        b = sortbuf.Batch.from_lists(keys, vals)
        if self.native_hash:
            self.n_out += b.n
        part = b.hash_partition(self.kind, self.R) if self.native_hash else \
            np.asarray(parts_l, dtype=np.int32)
        perm = b.sort(self.kind, part)
        starts = np.zeros(self.R + 1, np.int64)
        np.cumsum(np.bincount(part, minlength=self.R), out=starts[1:])
        idx = len(self.spills)
        path = self._spill_path(idx)
        rec = SpillRecord(self.R)
        spilled = 0
        if self._to_memory and self.codec is None:
            # an in-memory output: the segments are joined once into the bytes
            # the store holds (no file object; each encode buffer is a view);
            # their CRC words stay 0 — never read in this process, filled in
            # if the store turns the output away (_commit_spill)
            pieces, pos = [], 0
            for p in range(self.R):
                lo, hi = int(starts[p]), int(starts[p + 1])
                if self.combiner_cls is not None and hi > lo:
                    body, nrec = self._combine_native(b, perm, lo, hi)
                else:
                    body, nrec = b.ifile_body(perm, lo, hi, view=True), hi - lo
                spilled += nrec
                pieces += (body, b"\0\0\0\0")
                rec.put(p, pos, len(body) + 4, len(body) + 4)
                pos += len(body) + 4
            self._commit_spill(path, b"".join(pieces), rec, crc_pending=True)
            self.spills.append((path, rec))
            self.reporter.incrCounter(C.TASK_GROUP, C.SPILLED_RECORDS, spilled)
            return
        f = self._open_spill(path)
        try:
            for p in range(self.R):
                lo, hi = int(starts[p]), int(starts[p + 1])
                if self.combiner_cls is not None and hi > lo:
                    body, nrec = self._combine_native(b, perm, lo, hi)
                else:
                    body, nrec = b.ifile_body(perm, lo, hi), hi - lo
                spilled += nrec
                rec.put(p, *sortbuf.write_segment(f, body, self.codec,
                                                  crc=not self._to_memory))
        except BaseException:
            f.close()
            raise
        self._commit_spill(path, f, rec, crc_pending=self._to_memory)
        self.spills.append((path, rec))
        self.reporter.incrCounter(C.TASK_GROUP, C.SPILLED_RECORDS, spilled)

    def _merge_parts_native(self, final):
        rec_out = SpillRecord(self.R)
        spilled = 0
        combine = self.combiner_cls is not None and \
            len(self.spills) >= self.min_spills_for_combine
        with open(final, "wb") as f:
            for p in range(self.R):
                bodies = []
                for path, rec in self.spills:
                    start, _raw, plen = rec.get(p)
                    with open(path, "rb") as sf:
                        sf.seek(start)
                        bodies.append(sortbuf.segment_body(sf.read(plen), self.codec))
                b = sortbuf.Batch.from_ifile_bodies(bodies)
                # a stable sort of the concatenated runs == the k-way merge
                # (earlier spills win ties, Merger.MergeQueue)
                perm = b.sort(self.kind, np.zeros(b.n, np.int32))
                if combine and b.n:
                    body, nrec = self._combine_native(b, perm, 0, b.n)
                else:
                    body, nrec = b.ifile_body(perm, 0, b.n), b.n
                spilled += nrec
                rec_out.put(p, *sortbuf.write_segment(f, body, self.codec))
        rec_out.write(final + ".index")
        _fs_written(final)
        for path, _ in self.spills:
            for q in (path, path + ".index"):
                if os.path.exists(q):
                    os.remove(q)
        self.reporter.incrCounter(C.TASK_GROUP, C.SPILLED_RECORDS, spilled)

    def flush(self):
        """Final spill + merge into file.out / file.out.index."""
        self._wait_spill()
        final = os.path.join(self.out_dir, "file.out")
        self._direct_final = not self.spills
        self._to_memory = self._direct_final and 0 < self.mem_max and \
            self.buf_bytes <= self.mem_max
        try:
            self.sort_and_spill()
        finally:
            self._direct_final = self._to_memory = False
        if len(self.spills) == 1:
            path, rec = self.spills[0]
            if path != final:
                os.replace(path, final)
                os.replace(path + ".index", final + ".index")
        elif self.kind is not None:
            self._merge_parts_native(final)
        else:
            self._merge_parts(final)
        self.reporter.incrCounter(C.TASK_GROUP, C.MAP_OUTPUT_RECORDS, self.n_out)
        self.reporter.incrCounter(C.TASK_GROUP, C.MAP_OUTPUT_BYTES, self.bytes_out)
        return final

    def _merge_parts(self, final):
        rec_out = SpillRecord(self.R)
        spilled = 0
        with open(final, "wb") as f:
            for p in range(self.R):
                segs = []
                for path, rec in self.spills:
                    start, _raw, plen = rec.get(p)
                    with open(path, "rb") as sf:
                        sf.seek(start)
                        data = sf.read(plen)
                    segs.append([(self.sort_key(kb), kb, vb)
                                 for kb, vb in read_segment(data, self.codec)])
                merged = merge_segments(segs, self.factor)
                if self.combiner_cls is not None and len(self.spills) >= \
                        self.min_spills_for_combine:
                    merged = run_combiner(self.combiner_cls, self.job, self.kcls, self.vcls,
                                          list(merged), self.reporter)
                w = IFileWriter(f, self.codec)
                n = 0
                for _sk, kb, vb in merged:
                    w.append(kb, vb)
                    n += 1
                spilled += n
                rec_out.put(p, *w.close())
        rec_out.write(final + ".index")
        _fs_written(final)
        for path, _ in self.spills:
            for q in (path, path + ".index"):
                if os.path.exists(q):
                    os.remove(q)
        self.reporter.incrCounter(C.TASK_GROUP, C.SPILLED_RECORDS, spilled)


def _fs_written(path, size=None):
    """Local bytes a task wrote (FILE_BYTES_WRITTEN via FileSystem statistics)."""
    from ..fs import STATS
    try:
        STATS.add("file", written=os.path.getsize(path) if size is None else size)
    except OSError:
        pass


def _fs_counters(rep, before):
    """FileSystemCounters of a task from the thread's FileSystem statistics."""
    from ..fs import STATS
    for scheme, (r, w) in STATS.delta(before, STATS.snapshot()).items():
        if r:
            rep.incrCounter(C.FS_GROUP, f"{scheme.upper()}_BYTES_READ", r)
        if w:
            rep.incrCounter(C.FS_GROUP, f"{scheme.upper()}_BYTES_WRITTEN", w)


def merge_segments(segments, factor: int = 10):
    """k-way merge of sorted (sk, kb, vb) runs, at most ``factor`` runs per pass
    (Merger.MergeQueue). Stable: earlier segments win ties."""
    segs = [s for s in segments if s]
    while len(segs) > factor:
        nxt = []
        for i in range(0, len(segs), factor):
            grp = segs[i:i + factor]
            nxt.append(list(_heap_merge(grp)))
        segs = nxt
    return _heap_merge(segs)


def _decorate(si, seg):
    for ri, r in enumerate(seg):
        yield (r[0], si, ri, r)


def _heap_merge(segs):
    for _sk, _si, _ri, r in heapq.merge(*[_decorate(si, s) for si, s in enumerate(segs)]):
        yield r


class MapTask(Task):
    def __init__(self, job, attempt_id, partition, split):
        super().__init__(job, attempt_id, partition)
        self.split = split
        self.reporter.split = split
        self.output_file = None  # (path to file.out) when R > 0

    def run(self, local_dir: str):
        from ..fs import STATS
        fs0 = STATS.snapshot()
        try:
            return self._run(local_dir)
        finally:
            _fs_counters(self.reporter, fs0)

    def _run(self, local_dir: str):
        self.start_time = time.time()
        job = self._task_conf()
        self.local_dir = local_dir
        rep = self.reporter
        R = job.get_num_reduce_tasks()
        committer = self.committer()
        committer.setup_task(job, self.attempt_id)
        if isinstance(self.split, FileSplit):  # MapTask.updateJobWithSplit
            job.set("map.input.file", self.split.path)
            job.set_long("map.input.start", self.split.start)
            job.set_long("map.input.length", self.split.length)
        informat = new_instance(job.get_input_format(), job)
        reader = informat.getRecordReader(self.split, job, rep)
        if isinstance(self.split, FileSplit):
            rep.incrCounter(C.TASK_GROUP, C.MAP_INPUT_BYTES, self.split.length)
        if R == 0:
            outfmt = new_instance(job.get_output_format(), job)
            name = f"part-{self.partition:05d}"
            collector = _DirectCollector(outfmt.getRecordWriter(None, job, name, rep), rep)
        else:
            collector = MapOutputBuffer(self, job, rep, os.path.join(local_dir, "output"))
        # the fork's GPU branch (MapTask.java:432-438): a GPU attempt runs the
        # job's GPU map runner, told its device
        if self.run_on_gpu:
            job.set_int("hbmr.task.gpu.device", self.gpu_device_id)
            runner_cls = job.get_gpu_map_runner_class()
        else:
            runner_cls = job.get_map_runner_class()
        runner = new_instance(runner_cls, job)
        try:
            runner.run(_ProgressReader(reader, rep, self), collector, rep)
        finally:
            reader.close()
        if R == 0:
            collector.flush()
        else:
            self.output_file = collector.flush()
        # side files (MultipleOutputs, lazily created outputs) of a map with
        # reduces are committed the same way as a map-only task's part file
        # (Task.done: commit whenever needsTaskCommit)
        if committer.needs_task_commit(job, self.attempt_id):
            committer.commit_task(job, self.attempt_id)
        rep.set_progress(1.0)
        self.finish_time = time.time()
        return self.output_file


class _ProgressReader:
    def __init__(self, reader, reporter, task):
        self.r = reader
        self.rep = reporter
        self.task = task
        self.n = 0

    def next(self):
        kv = self.r.next()
        self.n += 1
        if (self.n & 4095) == 0:
            self.task.check_killed()
            try:
                self.rep.progress_value = self.r.getProgress()
            except Exception:
                pass
        return kv

    def __iter__(self):
        while True:
            kv = self.next()
            if kv is None:
                return
            yield kv

    def getProgress(self):  # noqa: N802
        return self.r.getProgress()

    def close(self):
        self.r.close()


# ------------------------------------------------------------------- reduce side
class MapOutputLocation:
    """Where to fetch one map's output (the reference's task-completion event +
    TaskTracker /mapOutput URL, ReduceTask.java:1476)."""

    def __init__(self, map_attempt, path, fetch=None):
        self.map_attempt = map_attempt
        self.path = path
        self.fetch = fetch  # optional callable(partition) -> bytes (remote shuffle)

    def read_partition(self, part):
        if self.fetch is not None:
            return self.fetch(part)
        held = mapoutput.STORE.get(self.path) if self.path else None
        if held is not None:            # an in-memory map output of this process
            data, idx = held
            start, _raw, plen = idx.get(part)
            # a view, not a copy (sortbuf.in_process: no CRC to check)
            return memoryview(data)[start:start + plen]
        idx = SpillRecord.read(self.path + ".index")
        start, _raw, plen = idx.get(part)
        with open(self.path, "rb") as f:
            f.seek(start)
            return f.read(plen)


class ReduceTask(Task):
    def __init__(self, job, attempt_id, partition, num_maps):
        super().__init__(job, attempt_id, partition)
        self.num_maps = num_maps
        self.locations: list[MapOutputLocation] = []

    def add_map_output(self, loc: MapOutputLocation):
        self.locations.append(loc)

    #: reduce slow-start: callable(start) -> {"events": [[map tid, attempt, output]],
    #: "num_maps": M, "state": job state} polled for map completions that happen
    #: after the reduce started (GetMapEventsThread, ReduceTask.java:2793)
    event_source = None

    def _map_outputs(self):
        """Yield every map's output location once: the ones known at launch, then
        new completion events until all ``num_maps`` maps have been seen."""
        seen = set()
        for loc in self.locations:
            seen.add(loc.map_attempt)
            yield loc
        if self.event_source is None:
            return
        got_maps = set()
        start = 0
        delay = 0.001
        while len(seen) < self.num_maps:
            self.check_killed()
            r = self.event_source(start)
            evs = r.get("events") or []
            start += len(evs)
            if r.get("state") not in (None, "RUNNING", "PREP"):
                raise RuntimeError(f"job ended ({r.get('state')}) while the reduce was copying")
            new = False
            for tid, aid, out in evs:
                if tid in got_maps or aid in seen:
                    continue        # a re-executed map's second event: already fetched
                got_maps.add(tid)
                seen.add(aid)
                new = True
                yield MapOutputLocation(aid, (out or {}).get("path"))
            if not new:
                if not r.get("waited"):
                    # a source that does not long-poll: back off between polls
                    time.sleep(delay)
                    delay = min(0.05, delay * 2)
            else:
                delay = 0.001

    def run(self, local_dir: str):
        from ..fs import STATS
        fs0 = STATS.snapshot()
        try:
            return self._run(local_dir)
        finally:
            _fs_counters(self.reporter, fs0)

    def _run(self, local_dir: str):
        self.start_time = time.time()
        job = self._task_conf()
        self.local_dir = local_dir
        rep = self.reporter
        codec = get_codec(job.get("mapred.map.output.compression.codec",
                                  "org.apache.hadoop.io.compress.DefaultCodec")) \
            if job.get_compress_map_output() else None
        kcls = job.get_map_output_key_class()
        vcls = job.get_map_output_value_class()
        sort_key = job.get_output_key_comparator()
        group_key = job.get_output_value_grouping_comparator()
        from .skipbadrecords import SkipLog, record_skip, skipping_limit
        skip_max = skipping_limit(job, False)
        kind = sortbuf.key_kind(job) if not skip_max else None
        # copy phase: bounded shuffle buffer, big or overflowing segments go to
        # disk as sorted runs (ReduceCopier, hbmr/mapred/shuffle.py)
        from .shuffle import ShuffleMerger
        merger = ShuffleMerger(job, local_dir, codec, sort_key, kind, rep, self.check_killed)
        for loc in self._map_outputs():
            self.check_killed()
            merger.add(loc.read_partition(self.partition))
        rep.incrCounter(C.TASK_GROUP, C.REDUCE_SHUFFLE_BYTES, merger.shuffled)
        if TRACE.on:
            TRACE.instant("reduce.copied", bytes=merger.shuffled)
        rep.set_progress(1 / 3)
        # sort phase (merge)
        if not merger.on_disk:
            if kind is not None:
                # stable sort of the concatenated map outputs == Merger's k-way merge
                b = sortbuf.Batch.for_reduce(merger.memory_bodies())
                perm = b.sort(kind, np.zeros(b.n, np.int32))
                return self._reduce_native(job, b, perm, kind, kcls, vcls)
            merged = merge_segments(merger.memory_records(), job.get_int("io.sort.factor", 10))
        else:
            merged = merger.final_iter()
        rep.set_progress(2 / 3)
        # reduce phase
        committer = self.committer()
        committer.setup_task(job, self.attempt_id)
        outfmt = new_instance(job.get_output_format(), job)
        writer = outfmt.getRecordWriter(None, job, f"part-{self.partition:05d}", rep)
        reducer = new_instance(job.get_reducer_class(), job)
        n_in = itertools.count()
        n_out = [0]
        n_groups = 0

        class _Out(OutputCollector):
            def collect(self_inner, k, v):
                writer.write(k, v)
                n_out[0] += 1

        counted = ((next(n_in), r)[1] for r in merged)
        out = _Out()
        skipped = 0
        skiplog = None
        try:
            for kb, vals in group_sorted(counted, group_key, vcls):
                n_groups += 1
                if (n_groups & 1023) == 0:
                    self.check_killed()
                if not skip_max:
                    reducer.reduce(kcls.deserialize(kb), vals, out, rep)
                    continue
                # skipping mode: a key group whose reduce() fails is skipped
                key = kcls.deserialize(kb)
                seen = []
                tracked = (seen.append(v) or v for v in vals)
                try:
                    reducer.reduce(key, tracked, out, rep)
                except Exception:  # noqa: BLE001
                    skipped += 1
                    if skipped > skip_max:
                        raise
                    rest = list(vals)
                    record_skip(rep, False, len(seen) + len(rest))
                    if skiplog is None:
                        skiplog = SkipLog(job, kcls, vcls)
                    for v in seen + rest:
                        skiplog.add(key, v)
        finally:
            if skiplog is not None:
                skiplog.close()
            reducer.close()
            writer.close(rep)
        merger.cleanup()
        rep.incrCounter(C.TASK_GROUP, C.REDUCE_INPUT_GROUPS, n_groups)
        rep.incrCounter(C.TASK_GROUP, C.REDUCE_INPUT_RECORDS, next(n_in))
        rep.incrCounter(C.TASK_GROUP, C.REDUCE_OUTPUT_RECORDS, n_out[0])
        if committer.needs_task_commit(job, self.attempt_id):
            committer.commit_task(job, self.attempt_id)
        rep.set_progress(1.0)
        self.finish_time = time.time()

    def _reduce_native(self, job, b, perm, kind, kcls, vcls):
        """Reduce phase over a natively merged partition (no skipping mode)."""
        rep = self.reporter
        rep.set_progress(2 / 3)
        committer = self.committer()
        committer.setup_task(job, self.attempt_id)
        outfmt = new_instance(job.get_output_format(), job)
        writer = outfmt.getRecordWriter(None, job, f"part-{self.partition:05d}", rep)
        reducer = new_instance(job.get_reducer_class(), job)
        n_out = [0]

        class _Out(OutputCollector):
            def collect(self_inner, k, v):
                writer.write(k, v)
                n_out[0] += 1

        out = _Out()
        ends = b.group_ends(kind, perm, 0, b.n).tolist()
        pl = perm.tolist()
        kdes, vdes = kcls.deserialize, vcls.deserialize
        # a reducer that takes serialised groups (PipesReducer.raw_reduce)
        # gets them without a Writable built per record
        rr = getattr(reducer, "raw_reduce", None)
        rr = rr(kcls, vcls) if rr is not None else None
        if TRACE.on:
            TRACE.instant("reduce.sorted", groups=len(ends))
        try:
            a = 0
            for g, e in enumerate(ends):
                if (g & 1023) == 1023:
                    self.check_killed()
                if rr is not None:
                    rr(b.key(pl[a]), [b.value_view(r) for r in pl[a:e]], out, rep)
                else:
                    reducer.reduce(kdes(b.key(pl[a])), (vdes(b.value(r)) for r in pl[a:e]), out,
                                   rep)
                a = e
            if TRACE.on:
                TRACE.instant("reduce.fed")
        finally:
            reducer.close()
            writer.close(rep)
        if TRACE.on:
            TRACE.instant("reduce.closed")
        rep.incrCounter(C.TASK_GROUP, C.REDUCE_INPUT_GROUPS, len(ends))
        rep.incrCounter(C.TASK_GROUP, C.REDUCE_INPUT_RECORDS, b.n)
        rep.incrCounter(C.TASK_GROUP, C.REDUCE_OUTPUT_RECORDS, n_out[0])
        if committer.needs_task_commit(job, self.attempt_id):
            committer.commit_task(job, self.attempt_id)
        if TRACE.on:
            TRACE.instant("reduce.committed")
        rep.set_progress(1.0)
        self.finish_time = time.time()


def iter_bytes(data: bytes):
    return io.BytesIO(data)
