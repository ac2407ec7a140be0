"""WordCount — BASELINE config 1 (CPU-only mappers on the LocalJobRunner).

Same job as hadoop-1.0.3/src/examples/org/apache/hadoop/examples/WordCount.java:
map emits (word, 1) per whitespace token, combiner + reducer sum.

By default the mapper combines in memory (``hbmr.wordcount.inmapper.combine``):
it counts the split's tokens in a C-level Counter and emits each distinct word
once, with its count, when the split ends (or when ``hbmr.wordcount.inmapper.
max.words`` distinct words are held).  The reduce output is the same; the map
side does what WordCount's combiner (IntSumReducer) would, without a Python
collect() per token, which bound the per-token job at 4.4 MB/s.  ``false``
restores the reference's per-token emit.

``hbmr.wordcount.native`` (default true) runs the map through
:class:`NativeWordCountRunner`: the same counts from a C++ tokenizer + hash
table over 4 MiB blocks of the split (native/cpu/wordcount.cc).
"""
from __future__ import annotations

from collections import Counter

from ..io.writable import IntWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from ..mapred.maprunner import MapRunner

INMAPPER_KEY = "hbmr.wordcount.inmapper.combine"


class WordCountMapper(Mapper):
    one = IntWritable(1)

    def configure(self, job):
        self.inmapper = job.get_boolean(INMAPPER_KEY, True)
        self.max_words = job.get_int("hbmr.wordcount.inmapper.max.words", 1 << 20)
        self.counts = Counter()
        self.lines = []         # lines held back: counted 4096 at a time in one C call
        self.out = None

    def map(self, key, value, output, reporter):
        if not getattr(self, "inmapper", False):
            for w in value.bytes.split():
                output.collect(Text(w), self.one)
            return
        self.out = output
        lines = self.lines
        lines.append(value.bytes)
        if len(lines) >= 4096:
            self._count()
            if len(self.counts) >= self.max_words:
                self._flush()

    def _count(self):
        if self.lines:
            self.counts.update(b"\n".join(self.lines).split())
            self.lines.clear()

    def _flush(self):
        self._count()
        out = self.out
        for w, c in self.counts.items():
            out.collect(Text(w), IntWritable(c))
        self.counts.clear()

    def close(self):
        if self.out is not None and (self.counts or self.lines):
            self._flush()


class NativeWordCountRunner(MapRunner):
    """Map runner counting a text split's words in C++ (native/cpu/wordcount.cc):
    the split's bytes are read in 4 MiB blocks of whole lines (the lines
    LineRecordReader would return: those starting at or before the split end),
    tokenised on ASCII whitespace and counted in one open-addressing table, and
    each distinct word is emitted once with its count — the in-mapper combine
    of WordCountMapper without a Python call per line or token.  Other inputs
    (compressed files, other record readers) take the per-record path."""

    BLOCK = 4 << 20

    def run(self, reader, output, reporter):
        from ..mapred import counters as C
        from ..mapred.formats import LineRecordReader
        lr = getattr(reader, "r", reader)
        lib = _wc_lib()
        if lib is None or not isinstance(lr, LineRecordReader) or lr.codec is not None or \
                type(self.mapper) is not WordCountMapper or \
                not self.job.get_boolean(INMAPPER_KEY, True):
            return super().run(reader, output, reporter)
        h = lib.hbmr_wc_cpu_new()
        lines = 0
        try:
            max_words = self.job.get_int("hbmr.wordcount.inmapper.max.words", 1 << 20)
            for block in _owned_blocks(lr, self.BLOCK):
                # (the newlines are counted in the tokeniser's pass)
                lines += 0 if block.endswith(b"\n") else 1
                if lib.hbmr_wc_cpu_add(h, block, len(block)) >= max_words:
                    _emit(lib, h, output)
                if reporter is not None:
                    reporter.progress()
            _emit(lib, h, output)
            lines += lib.hbmr_wc_cpu_newlines(h)
        finally:
            lib.hbmr_wc_cpu_free(h)
        reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, lines)


def _owned_blocks(lr, size):
    """Blocks of whole lines of ``lr``'s split, from its current position (the
    first partial line already skipped) through the line that starts at or
    before the split end; each block ends with a newline except possibly the
    file's last."""
    f, pos, end = lr.f, lr.pos, lr.end
    tail = b""
    while pos <= end:
        data = f.read(size)
        if not data:
            if tail:
                yield tail
            return
        buf = tail + data if tail else data
        base = pos - len(tail)          # file offset of buf[0]
        cut = buf.rfind(b"\n")
        if cut < 0:
            tail = buf
            pos = base + len(buf)
            continue
        # lines starting at <= end are ours: stop after the first newline at
        # offset >= end (the line holding `end`, or the one starting there)
        if base + cut >= end:
            stop = buf.find(b"\n", max(0, end - base))
            yield buf[:stop + 1]
            return
        yield buf[:cut + 1]
        tail = buf[cut + 1:]
        pos = base + len(buf)
    if tail:
        yield tail


def _emit(lib, h, output):
    import ctypes
    import numpy as np
    w = lib.hbmr_wc_cpu_words(h)
    if w == 0:
        return
    nbytes = lib.hbmr_wc_cpu_bytes(h)
    words = ctypes.create_string_buffer(max(1, nbytes))
    offs = np.empty(w + 1, dtype=np.int64)
    cnts = np.empty(w, dtype=np.int64)
    lib.hbmr_wc_cpu_export(h, words, offs.ctypes.data, cnts.ctypes.data)
    raw = words.raw[:nbytes]
    o = offs.tolist()
    for i, c in enumerate(cnts.tolist()):
        output.collect(Text(raw[o[i]:o[i + 1]]), IntWritable(c))


_WC_LIB = None


def _wc_lib():
    global _WC_LIB
    if _WC_LIB is None:
        import ctypes
        import os
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                            "libhbmr_cpu.so")
        try:
            L = ctypes.CDLL(path)
            P, I64 = ctypes.c_void_p, ctypes.c_int64
            L.hbmr_wc_cpu_new.restype = P
            L.hbmr_wc_cpu_free.argtypes = [P]
            L.hbmr_wc_cpu_add.argtypes = [P, ctypes.c_char_p, I64]
            L.hbmr_wc_cpu_add.restype = I64
            for f in ("hbmr_wc_cpu_words", "hbmr_wc_cpu_bytes", "hbmr_wc_cpu_tokens",
                      "hbmr_wc_cpu_newlines"):
                getattr(L, f).argtypes = [P]
                getattr(L, f).restype = I64
            L.hbmr_wc_cpu_export.argtypes = [P, P, P, P]
            _WC_LIB = L
        except (OSError, AttributeError):
            _WC_LIB = False
    return _WC_LIB or None


class IntSumReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(key, IntWritable(sum(v.value for v in values)))


def make_job(inputs, output, reduces=1, conf=None) -> JobConf:
    job = JobConf(conf)
    job.set_job_name("wordcount")
    job.set_output_key_class(Text)
    job.set_output_value_class(IntWritable)
    job.set_mapper_class(WordCountMapper)
    if job.get_boolean("hbmr.wordcount.native", True):
        job.set_map_runner_class(NativeWordCountRunner)
    job.set_combiner_class(IntSumReducer)
    job.set_reducer_class(IntSumReducer)
    job.set_num_reduce_tasks(reduces)
    FileInputFormat.setInputPaths(job, *([inputs] if isinstance(inputs, str) else inputs))
    FileOutputFormat.setOutputPath(job, output)
    return job


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr wordcount")
    ap.add_argument("input", nargs="+")
    ap.add_argument("output")
    ap.add_argument("-r", "--reduces", type=int, default=1)
    a = ap.parse_args(argv)
    job = make_job(a.input, a.output, a.reduces)
    rj = JobClient.runJob(job)
    return 0 if rj.isSuccessful() else 1


# --------------------------------------------------------------------------- GPU WordCount
# The same job as a split-level GPU job: a text split
# is read into HBM with LineRecordReader's boundary rule, tokenized and counted
# by native/kernels/text.hip (exact hash aggregation = the fused combiner), the
# per-tracker tables are merged and hash-partitioned like HashPartitioner, the
# shuffle is one all-to-all-v of "word\n" bytes + one of counts (RCCL over
# xGMI), and each tracker writes its partition sorted by Text key order, in
# TextOutputFormat's "word\tcount" lines — the classic job's output, byte for
# byte.
from ..gpu.splitjob import SplitJob, SplitSpec  # noqa: E402


def read_text_split(path, start, length, chunk=1 << 16) -> bytes:
    """Bytes of the lines a LineRecordReader over (path, start, length) returns,
    newlines included: the first partial line is skipped unless start == 0, and
    the line running through the split end is read to its end."""
    from ..fs import strip_scheme
    end = start + length
    with open(strip_scheme(path), "rb") as f:
        f.seek(start)
        begin = start
        if start != 0:
            while True:
                buf = f.read(chunk)
                if not buf:
                    return b""
                i = buf.find(b"\n")
                if i >= 0:
                    begin += i + 1
                    break
                begin += len(buf)
        if begin > end:
            return b""
        f.seek(begin)
        body = f.read(end - begin)
        # finish the line that contains offset `end` (it starts at or before end)
        tail = []
        while True:
            buf = f.read(chunk)
            if not buf:
                break
            i = buf.find(b"\n")
            if i >= 0:
                tail.append(buf[:i + 1])
                break
            tail.append(buf)
        return body + b"".join(tail)


class WordCountSplitJob(SplitJob):
    collective_reduce = True
    needs_reduce = True

    def configure(self, conf):
        self.conf = conf
        self.out = conf.get("mapred.output.dir")

    def get_splits(self, conf, trackers):
        from ..mapred.formats import TextInputFormat
        from ..mapred.jobconf import JobConf
        splits = TextInputFormat().getSplits(JobConf(conf), max(1, conf.get_num_map_tasks()))
        out = []
        for i, s in enumerate(splits):
            loc = [trackers[i * len(trackers) // len(splits)]] if trackers else []
            key = f"wc:{s.path}:{s.start}:{s.length}"
            out.append(SplitSpec(i, key, "file", {"path": s.path, "start": s.start,
                                                  "length": s.length}, loc, s.length))
        return out

    def load_split(self, spec: SplitSpec, device):
        import torch
        p = spec.params
        data = read_text_split(p["path"], p["start"], p["length"])
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else \
            torch.empty(0, dtype=torch.uint8)
        return t if str(device) == "cpu" else t.to(device)

    def _count(self, ctx, data):
        from ..mapred import counters as C
        from ..ops import text
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_BYTES, int(data.numel()))
        return text.count_words(data, getattr(ctx, "stream", None))

    def map_gpu(self, ctx, data):
        return self._count(ctx, data)

    def map_cpu(self, ctx, data):
        return self._count(ctx, data)

    def combine(self, ctx, outputs):
        import torch
        from ..ops import text
        dev = ctx.device if ctx.device is not None else torch.device("cpu")
        blobs = [b.to(dev) for b, _ in outputs]
        counts = [c.to(dev) for _, c in outputs]
        blob = torch.cat(blobs) if blobs else torch.empty(0, dtype=torch.uint8, device=dev)
        cnt = torch.cat(counts) if counts else torch.empty(0, dtype=torch.int64, device=dev)
        return text.merge_tables(blob, cnt, max(1, ctx.world_size))

    def reduce(self, ctx, combined):
        from ..mapred import counters as C
        from ..ops import text
        blob, counts, part_bytes, part_words = combined
        rblob, rcounts = self._shuffle(ctx, blob, counts, part_bytes, part_words)
        mblob, mcounts, _, _ = text.merge_tables(rblob, rcounts, 1)
        items = text.sorted_items(mblob, mcounts)
        total = sum(n for _, n in items)
        ctx.reporter.incrCounter(C.TASK_GROUP, C.REDUCE_INPUT_GROUPS, len(items))
        ctx.reporter.incrCounter(C.TASK_GROUP, C.REDUCE_OUTPUT_RECORDS, len(items))
        if self.out:
            import os
            tmp = os.path.join(self.out, "_temporary")
            os.makedirs(tmp, exist_ok=True)
            name = f"part-{ctx.rank:05d}"
            with open(os.path.join(tmp, name), "wb") as f:
                f.write(b"".join(w + b"\t" + str(n).encode() + b"\n" for w, n in items))
            os.replace(os.path.join(tmp, name), os.path.join(self.out, name))
        return {"distinct": len(items), "words": total}

    @staticmethod
    def _shuffle(ctx, blob, counts, part_bytes, part_words):
        """The word tables' shuffle: two static-shape all-to-alls (bytes, then
        counts) whose slot sizes every rank agrees on through a HOST all-reduce
        of the largest per-destination sizes (the sizes are host values
        already: merge_tables returns them), so no collective here waits for
        the device; the one host read is the compaction after both exchanges
        are enqueued.  An overflowing slot (impossible with exact maxima, kept
        as a guard) sends every rank to all_to_all_v (an all-reduced flag)."""
        import torch

        from ..parallel.collectives import compact_static
        comm = ctx.comm
        W = comm.world_size
        if W <= 1 or not hasattr(comm, "all_to_all_v_static"):
            return comm.all_to_all_v(blob, part_bytes)[0], comm.all_to_all_v(counts, part_words)[0]
        mx = torch.tensor([max(part_bytes or [0]), max(part_words or [0])], dtype=torch.int64)
        mx = comm.all_reduce_max(mx) if hasattr(comm, "all_reduce_max") else mx
        cap_b, cap_w = max(1, int(mx[0])), max(1, int(mx[1]))
        rb, rcb = comm.all_to_all_v_static(blob, part_bytes, cap_b)
        rc, rcw = comm.all_to_all_v_static(counts, part_words, cap_w)
        got_b = compact_static(rb, rcb, cap_b)
        got_w = compact_static(rc, rcw, cap_w)
        # the fallback is a collective: every rank must take it or none (one
        # rank entering all_to_all_v alone would hang the gang), so the
        # overflow flags are all-reduced first
        over = torch.tensor([int(got_b is None or got_w is None)], dtype=torch.int64)
        if hasattr(comm, "all_reduce_max"):
            over = comm.all_reduce_max(over)
        if int(over[0]):
            return comm.all_to_all_v(blob, part_bytes)[0], comm.all_to_all_v(counts, part_words)[0]
        return got_b[0], got_w[0]

    def job_succeeded(self, jip):
        import os
        import shutil
        if self.out:
            shutil.rmtree(os.path.join(self.out, "_temporary"), ignore_errors=True)
            open(os.path.join(self.out, "_SUCCESS"), "wb").close()


def gpu_job(inputs, output, base=None, maps=None) -> JobConf:
    """WordCount as a split-level job (GPU map slots, CPU slots per the hybrid
    cost model)."""
    job = JobConf(base)
    job.set_job_name("wordcount-gpu")
    job.set("hbmr.splitjob.class", "hbmr.models.wordcount:WordCountSplitJob")
    FileInputFormat.setInputPaths(job, *([inputs] if isinstance(inputs, str) else inputs))
    FileOutputFormat.setOutputPath(job, output)
    if maps:
        job.set_num_map_tasks(maps)
    return job
