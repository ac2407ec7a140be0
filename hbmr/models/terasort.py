"""TeraGen / TeraSort / TeraValidate — BASELINE config 5, as a split-level job.

Behaviour of the reference's examples (src/examples/org/apache/hadoop/examples/
terasort): TeraGen writes 100-byte records (10-byte printable key from an LCG,
10-char row id, 78 filler letters, "\\r\\n"; TeraGen.java), TeraSort samples
up to 100,000 keys from ≤10 input splits to pick R-1 split points
(TeraInputFormat.java:101-141, createPartitions :80-99) and range-partitions
into R sorted part files (TeraSort.java:57-211), TeraValidate checks order
within and across parts (TeraValidate.java).

MI355X design:

* map (per split, on its GPU slot): records are generated straight into HBM
  (``teragen:<rows>`` input; the LCG jumps ahead in O(log n), bit-identical to
  TeraGen) or read from TeraGen files; one kernel computes every record's
  key words and range partition (splitters in LDS) and counts the partition
  sizes, a second scatters (key words, record number) into partition order
  (20 B per record; the 100-byte records stay where they are);
* shuffle: one all-to-all-v per tracker over RCCL/xGMI (each GPU owns a
  contiguous range of partitions) — the HTTP shuffle + merge of the
  reference (ReduceTask.java:1231-2514) disappears;
* reduce (collective, one per tracker): per group of consecutive partitions,
  collect the pieces every map produced, radix-sort the keys (8 passes over
  the high 8 key bytes, runs of equal high words ordered by the last 2 bytes),
  gather the 100-byte records once (4 records in flight per lane), verify
  order locally and against the neighbouring ranks' boundary keys
  (TeraValidate), and write ``part-NNNNN`` files if an output directory is set.

CPU slots run the same steps with numpy (hbmr.ops.sort CPU twins).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from ..gpu.splitjob import SplitJob, SplitSpec
from ..mapred import counters as C
from ..ops import sort as S
from ..utils.trace import TRACE

INPUT_KEY = "hbmr.terasort.input"            # "teragen:<rows>" or a directory of TeraGen files
SPLIT_ROWS_KEY = "hbmr.terasort.split.rows"
PARTS_KEY = "hbmr.terasort.partitions"       # R (default: one per tracker)
SAMPLE_KEY = "terasort.partitions.sample"    # the reference's key (default 100000)


def _hex_keys(hi: np.ndarray, lo: np.ndarray) -> list:
    return [f"{int(h):016x}{int(lo_):04x}" for h, lo_ in zip(hi, lo)]


def _parse_keys(hexes: list):
    hi = np.array([int(h[:16], 16) for h in hexes], dtype=np.uint64)
    lo = np.array([int(h[16:], 16) for h in hexes], dtype=np.uint64)
    return torch.from_numpy(hi.view(np.int64)), torch.from_numpy(lo.view(np.int64))


def create_partitions(sample_keys: np.ndarray, nparts: int) -> np.ndarray:
    """TeraInputFormat.createPartitions: sort the sample, take keys at
    Math.round(stepSize * i), i = 1..R-1 (sample_keys: uint8 [m, 10])."""
    m = sample_keys.shape[0]
    if nparts > m:
        raise ValueError(f"Requested more partitions than input keys ({nparts} > {m})")
    order = np.lexsort([sample_keys[:, j] for j in range(9, -1, -1)])
    srt = sample_keys[order]
    step = np.float32(m) / np.float32(nparts)
    idx = [int(math.floor(float(np.float32(step * np.float32(i))) + 0.5)) for i in range(1, nparts)]
    return srt[idx]


def _key_words(keys10: np.ndarray):
    hi = np.zeros(keys10.shape[0], dtype=np.uint64)
    for j in range(8):
        hi = (hi << np.uint64(8)) | keys10[:, j].astype(np.uint64)
    lo = (keys10[:, 8].astype(np.uint64) << np.uint64(8)) | keys10[:, 9].astype(np.uint64)
    return hi, lo


def _s64(x: int) -> int:
    """Wrap to the signed 64-bit range (checksums are sums mod 2^64)."""
    return ((x + (1 << 63)) % (1 << 64)) - (1 << 63)


def _file_records(path):
    n = os.path.getsize(path) // S.RECORD
    return n


_SPLITTER_MEMO: dict = {}


class TeraSortSplitJob(SplitJob):
    collective_reduce = True
    needs_reduce = True

    def configure(self, conf):
        self.conf = conf
        self.input = conf.get(INPUT_KEY, "teragen:1000000")
        self.split_rows = conf.get_long(SPLIT_ROWS_KEY, 10_000_000)
        self.nparts_conf = conf.get_int(PARTS_KEY, 0)
        self.sample = conf.get_long(SAMPLE_KEY, 100000)
        self.out = conf.get("mapred.output.dir")
        # one-rank reduce: consecutive partitions sorted together, up to this many
        # record bytes per sort (bigger sorts run the radix passes at full
        # occupancy; the working set is 1.4x the group)
        self.group_bytes = conf.get_long("hbmr.terasort.reduce.group.bytes", 8 << 30)
        # several ranks: each sender sorts every destination's run before the
        # all-to-all and receivers merge the W sorted runs (K8 merge path,
        # log2 W passes) instead of re-sorting what they received
        self.sorted_runs = conf.get_boolean("hbmr.terasort.shuffle.sorted.runs", False)
        # several ranks: the shuffle runs in this many waves of this rank's map
        # outputs (in launch order), each wave's all-to-all-v issued as soon as
        # its maps are done — with an early reduce (expect mode,
        # hbmr.job.prestage) it overlaps the later maps (map ∥ shuffle)
        # (0, the default: 4 when the job runs on several ranks, else 1)
        self.waves_conf = max(0, conf.get_int("hbmr.terasort.shuffle.waves", 0))
        # the waves' all-to-alls are static-shape: each destination slot is
        # sized from the split sizes and the partition share (x this slack),
        # the counts travel as a tensor and are read on the device, so no wave
        # waits on the host for its maps; one count check after the last wave
        # (an overflowing slot re-runs the shuffle with exact sizes)
        self.static_a2a = conf.get_boolean("hbmr.terasort.shuffle.static", True)
        self.slot_slack = conf.get_float("hbmr.terasort.shuffle.slot.slack", 1.08)
        # one-rank reduce: sort (high key word, packed record id) and gather by
        # the id (v4, default: 0.284 s per 100 GB sort vs 0.341 s for v3 on the
        # same box, profiles/r03_terasort_100gb_v4_1gpu.json); false = the v3
        # path, sort keys then gather through a permutation
        self.gid = conf.get_boolean("hbmr.terasort.reduce.gid", True)
        # out-of-core sort (MapTask.sortAndSpill / mergeParts): with an HBM
        # budget below the input size (or hbmr.terasort.spill=true) each map
        # sorts its split, spills the sorted run to host memory and drops the
        # split; the reduce brings back, per group of partitions sized to the
        # budget, every map's run slice and merges the runs (K8 merge path)
        self.budget = int(conf.get_float("hbmr.terasort.hbm.budget.gb", 0.0) * (1 << 30))
        self.spill = conf.get_boolean("hbmr.terasort.spill", False)
        if not self.spill and self.budget > 0:
            self.spill = sum(r[2] for r in self._ranges()) * S.RECORD > self.budget

    @property
    def cache_inputs(self):
        """Spill mode streams the input: a split is dropped after its map."""
        return not self.spill

    @property
    def max_inflight_maps(self):
        """Spill mode: maps in flight per GPU such that their working sets
        (the split, its sorted copy, keys and permutation: about 3.5x the
        split) stay inside the HBM budget; 0 = no cap."""
        if not self.spill:
            return 0
        split_bytes = max(1, self.split_rows * S.RECORD)
        budget = self.budget if self.budget > 0 else self.group_bytes
        return max(1, int(budget // (4 * split_bytes)))

    # -- splits + sampling (JobTracker side) -----------------------------------------
    def _ranges(self):
        """[(kind, params, rows)] covering the input."""
        if self.input.startswith("teragen:"):
            rows = int(self.input.split(":")[1])
            out = []
            for a in range(0, rows, self.split_rows):
                n = min(self.split_rows, rows - a)
                out.append(("teragen", {"first": a, "rows": n}, n))
            return out
        files = sorted(os.path.join(self.input, f) for f in os.listdir(self.input)
                       if not f.startswith(("_", ".")))
        out = []
        for f in files:
            n = _file_records(f)
            for a in range(0, n, self.split_rows):
                m = min(self.split_rows, n - a)
                out.append(("file", {"path": f, "first": a, "rows": m}, m))
        return out

    def _sample_keys(self, ranges):
        samples = min(10, len(ranges))
        if samples == 0:
            return np.zeros((0, 10), dtype=np.uint8)
        per = max(1, self.sample // samples)
        step = len(ranges) // samples
        keys = []
        for i in range(samples):
            kind, p, rows = ranges[step * i]
            m = min(per, rows)
            if kind == "teragen":
                keys.append(S.teragen_keys_cpu(p["first"], m))
            else:
                recs = np.fromfile(p["path"], dtype=np.uint8, count=m * S.RECORD,
                                   offset=p["first"] * S.RECORD).reshape(m, S.RECORD)
                keys.append(recs[:, :10])
        return np.concatenate(keys)

    def get_splits(self, conf, trackers):
        if self.spill and len(trackers) > 1 and self.needs_reduce:
            # rejected at job setup, before any map runs: the spill reduce
            # merges every map's run on one rank, and the several-rank paths
            # (shuffle waves, all-to-all-v) read device-resident map outputs
            raise ValueError(
                f"out-of-core TeraSort (spill mode: hbmr.terasort.spill, or input above "
                f"hbmr.terasort.hbm.budget.gb) runs its reduce on one rank; this job "
                f"would run on {len(trackers)} trackers")
        ranges = self._ranges()
        # default R: one per tracker, and at least one per ~1.2 GB of input so a
        # single GPU sorts the output a partition at a time, each partition
        # below the packed-key sort's group size (hbmr.ops.sort.PACK_GROUP_MAX)
        total = sum(r[2] for r in ranges) * S.RECORD
        nparts = self.nparts_conf or max(1, len(trackers), -(-total // (1200 << 20)))
        mk = (self.input, self.split_rows, self.sample, nparts)
        splitters = _SPLITTER_MEMO.get(mk) if self.input.startswith("teragen:") else None
        if splitters is None:
            split_keys = create_partitions(self._sample_keys(ranges), nparts) if nparts > 1 \
                else np.zeros((0, 10), dtype=np.uint8)
            hi, lo = _key_words(split_keys)
            splitters = _hex_keys(hi, lo)
            if self.input.startswith("teragen:"):   # generated input: same sample every job
                if len(_SPLITTER_MEMO) > 8:
                    _SPLITTER_MEMO.clear()
                _SPLITTER_MEMO[mk] = splitters
        out = []
        for i, (kind, p, rows) in enumerate(ranges):
            loc = [trackers[i * len(trackers) // len(ranges)]] if trackers else []
            key = f"tera:{kind}:{p.get('path', '')}:{p['first']}:{rows}"
            out.append(SplitSpec(i, key, kind, {**p, "splitters": splitters, "nparts": nparts},
                                 loc, rows * S.RECORD))
        return out

    # -- map ---------------------------------------------------------------------------
    def load_split(self, spec: SplitSpec, device):
        p = spec.params
        if spec.kind == "teragen":
            recs = S.teragen(p["first"], p["rows"], device=device)
        else:
            a = np.fromfile(p["path"], dtype=np.uint8, count=p["rows"] * S.RECORD,
                            offset=p["first"] * S.RECORD).reshape(p["rows"], S.RECORD)
            recs = torch.from_numpy(a).to(device)
        return {"records": recs, "splitters": p["splitters"], "nparts": p["nparts"]}

    def split_nbytes(self, data):
        return int(data["records"].numel())

    def _map(self, ctx, data):
        """Range-partition the split (TeraSort.java's TotalOrderPartitioner):
        key words + partition of every record, then a stable counting sort by
        partition.  The map output is 20 B per record — sorted-by-partition key
        words and row numbers into the (HBM-resident) input split; the 100-byte
        records themselves move once, in the reduce's final gather."""
        recs = data["records"]
        stream = getattr(ctx, "stream", None)
        nparts = data["nparts"]
        shi, slo = _parse_keys(data["splitters"]) if nparts > 1 else (
            torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64))
        n = recs.shape[0]
        # key words + partition + partition sizes, scan, one tile-ranked scatter
        hp, lp, row, offs, kbytes = S.tera_partition(recs, shi, slo, stream=stream,
                                                     kbytes=True)
        # order-independent checksum of the input keys, kept on the device
        # (summed by the partition kernel)
        csum = kbytes[1]
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, n)
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_OUTPUT_RECORDS, n)
        return {"records": recs, "hi": hp, "lo": lp, "row": row, "offsets": offs,
                "checksum": csum, "nparts": nparts, "splitters": data["splitters"],
                "kbytes": kbytes}

    def _map_spill(self, ctx, data):
        """Spill mode: sort the whole split by key (a range partition is a key
        range, so the sorted split is partition-ordered too), cut it at the
        splitters and copy the sorted run to (pinned) host memory on the task's
        stream; the device copies die with the task."""
        recs = data["records"]
        stream = getattr(ctx, "stream", None)
        nparts = data["nparts"]
        shi, slo = _parse_keys(data["splitters"]) if nparts > 1 else (
            torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64))
        n = recs.shape[0]
        srt, hs, ls = S.sort_records(recs, stream=stream)
        cuda = srt.is_cuda
        if cuda:
            shi, slo = shi.to(srt.device), slo.to(srt.device)
        offs = S.split_offsets(hs, ls, shi, slo, stream=stream)
        csum = hs.sum() + ls.sum()
        if cuda:
            host = torch.empty(srt.shape, dtype=torch.uint8, pin_memory=True)
            host.copy_(srt, non_blocking=True)
        else:
            host = srt
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_INPUT_RECORDS, n)
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_OUTPUT_RECORDS, n)
        ctx.reporter.incrCounter(C.TASK_GROUP, "MAP_SPILLED_RECORDS", n)
        return {"spill": host, "offsets": offs, "checksum": csum, "nparts": nparts,
                "splitters": data["splitters"], "rows": n}

    def map_gpu(self, ctx, data):
        return self._map_spill(ctx, data) if self.spill else self._map(ctx, data)

    def map_cpu(self, ctx, data):
        return self._map_spill(ctx, data) if self.spill else self._map(ctx, data)

    def map_gpu_batch(self, ctxs, datas):
        return [self.map_gpu(c, d) for c, d in zip(ctxs, datas)]

    # -- shuffle + reduce -------------------------------------------------------------
    @staticmethod
    def owner_range(rank, world, nparts):
        return rank * nparts // world, (rank + 1) * nparts // world

    def waves_for(self, world):
        """Shuffle waves for a job on ``world`` ranks (the same on every rank:
        the collective sequence must match)."""
        if self.waves_conf:
            return self.waves_conf
        return 4 if world > 1 else 1

    @property
    def orders_own_outputs(self):
        """Wave mode waits on each map output's event itself (combine() waits
        on all of them when one rank runs the job)."""
        return self.waves_conf != 1

    def combine(self, ctx, outputs):
        if self.waves_for(ctx.comm.world_size) > 1 and ctx.comm.world_size > 1:
            marks = getattr(ctx, "output_marks", None) or [None] * len(outputs)
            keep = [(o, m) for o, m in zip(outputs, marks) if o is not None]
            return {"outs": [o for o, _ in keep], "marks": [m for _, m in keep], "waves": True,
                    "nparts": keep[0][0]["nparts"] if keep else None, "offsets": None,
                    "checksum": 0}
        if ctx.device is not None and getattr(ctx, "output_marks", None):
            cur = torch.cuda.current_stream()
            for m in {id(m): m for m in ctx.output_marks if m is not None}.values():
                cur.wait_event(m)
        outs = [o for o in outputs if o is not None]
        if not outs:
            return {"outs": [], "offsets": None, "nparts": None, "checksum": 0}
        # one device->host copy of every map's partition offsets
        offs = torch.stack([o["offsets"] for o in outs]).to("cpu").numpy()
        csum = torch.stack([o["checksum"].reshape(()) for o in outs]).sum()
        return {"outs": outs, "offsets": offs, "nparts": outs[0]["nparts"], "checksum": csum}

    def reduce(self, ctx, combined):
        comm = ctx.comm
        outs = combined["outs"]
        dev = ctx.device if ctx.device is not None else torch.device("cpu")
        nparts = combined["nparts"]
        csum_in = combined["checksum"]
        if self.out:
            self._open_output(ctx)
        try:
            if combined.get("waves"):
                stats, csum_in = self._reduce_shuffle_waves(ctx, outs, combined["marks"], nparts,
                                                            dev)
            elif outs and outs[0].get("spill") is not None:
                if comm.world_size > 1:
                    raise NotImplementedError(
                        "out-of-core TeraSort (spill mode) runs its reduce on one rank")
                stats = self._reduce_spill(ctx, outs, combined["offsets"], nparts or 1, dev)
            elif comm.world_size == 1:
                stats = self._reduce_local(ctx, outs, combined["offsets"], nparts or 1, dev)
            else:
                stats = self._reduce_shuffle(ctx, outs, combined["offsets"], nparts, dev)
        except BaseException:
            # a failed or killed attempt: its partial part files never reach the
            # output directory (FileOutputCommitter.abortTask)
            self._close_output(ctx, commit=False)
            raise
        self._close_output(ctx, commit=True)
        # one device->host copy of this rank's statistics (no per-value syncs)
        n, st = stats
        if not torch.is_tensor(csum_in):
            csum_in = torch.tensor(_s64(int(csum_in)), dtype=torch.int64)
        if st is None:
            st = torch.tensor([0, 0, -1, -1, -1, -1], dtype=torch.int64)
        meta = torch.cat([torch.tensor([n], dtype=torch.int64),
                          csum_in.reshape(1).to("cpu", torch.int64), st.to("cpu")])
        meta = torch.stack([meta[0], meta[1], meta[3], meta[2], meta[4], meta[5], meta[6],
                            meta[7]])
        bad = int(meta[3])
        gathered = comm.all_gather(meta)
        total = sum(int(g[0]) for g in gathered)
        c_in = sum(int(g[1]) for g in gathered)
        c_out = sum(int(g[2]) for g in gathered)
        cross_bad = 0
        prev_last = None
        for g in gathered:
            if int(g[0]) == 0:
                continue
            f = (int(g[4]) & 0xFFFFFFFFFFFFFFFF, int(g[5]))
            if prev_last is not None and f < prev_last:
                cross_bad += 1
            prev_last = (int(g[6]) & 0xFFFFFFFFFFFFFFFF, int(g[7]))
        peak = torch.cuda.max_memory_allocated(dev) if dev.type == "cuda" else 0
        return {"records": n, "total_records": total, "unsorted": bad + cross_bad,
                "checksum_ok": (c_in - c_out) % (1 << 64) == 0, "partitions": nparts or 1,
                "peak_hbm_bytes": int(peak)}

    def _sorted_partition(self, his, los, rows, starts, lens, bases, dev, stream=None,
                          hi_range=None, defer=False, gid=True, alphabet=None, bounds=None):
        """Collect one partition's pieces from every map output, sort its keys,
        gather its records: (records, sorted hi, sorted lo).  The packed-id
        path (v4, hbmr.terasort.reduce.gid) when the map outputs allow it.
        ``defer``: (records, hi, lo, flag) without a host read; a non-zero
        device flag means the group must be redone with ``gid=False``."""
        if gid and self.gid and len(bases) <= S.GID_MAX_SPLITS and \
                max(b.shape[0] for b in bases) < S.GID_MAX_ROWS:
            got = S.sort_gathered(his, rows, starts, lens, bases, stream=stream,
                                  hi_range=hi_range, defer=defer, alphabet=alphabet,
                                  bounds=bounds)
            if got is not None:
                return got
        h, lw, split, row = S.tera_collect(his, los, rows, starts, lens, stream=stream)
        perm, hs, ls = S.sort_keys(h, lw, stream=stream)
        del h, lw
        recs = S.gather_records_multi(bases, split, row, perm, stream=stream)
        if defer:
            return recs, hs, ls, None
        return recs, hs, ls

    def _reduce_local(self, ctx, outs, offs, nparts, dev):
        """One rank owns every partition: no record shuffle.  Consecutive
        partitions are sorted in groups of about ``group_bytes`` (a partition is
        a key range, so a group sorts to its partitions in order and is cut by
        their counts), so peak HBM is the input splits + 20 B/record of map
        output + one group.  In HBM (no output) the groups run without a host
        read; if any group's tie runs were too long for the in-place fix, the
        whole reduce runs again on the full-key path."""
        if not outs:
            return 0, None
        n, st, flags = self._reduce_local_groups(ctx, outs, offs, nparts, dev, True)
        if flags is not None and int(flags.max()):
            n, st, _ = self._reduce_local_groups(ctx, outs, offs, nparts, dev, False)
        return n, st

    def _reduce_local_groups(self, ctx, outs, offs, nparts, dev, use_gid):
        flags = None
        his = [o["hi"] for o in outs]
        los = [o["lo"] for o in outs]
        rows = [o["row"] for o in outs]
        bases = [o["records"] for o in outs]
        # (out of order, checksum) and the stats kernel's scratch
        gstats = torch.zeros(S.GROUP_STATS_LEN, dtype=torch.int64, device=dev)
        prev_last = None
        first = last = None
        n = 0
        sizes = (offs[:, 1:] - offs[:, :-1]).sum(axis=0)     # records per partition
        groups, pa = [], 0
        # a group stays below the packed-key sort's record limit when its
        # partitions allow (one larger partition sorts as pairs)
        lim = min(self.group_bytes // S.RECORD, S.PACK_GROUP_MAX - 1) if self.gid else \
            self.group_bytes // S.RECORD
        while pa < nparts:
            pb, acc = pa, 0
            while pb < nparts and (pb == pa or acc + int(sizes[pb]) <= lim):
                acc += int(sizes[pb])
                pb += 1
            groups.append((pa, pb))
            pa = pb
        spl_hi = [int(h[:16], 16) for h in outs[0].get("splitters") or []] if nparts > 1 else []
        # the key alphabet [0, 2^bits) holding every key byte of the high
        # words (the maps' OR of them): the packed sort's dense window needs
        # it (one host read)
        alphabet = None
        if use_gid and all(o.get("kbytes") is not None for o in outs):
            orb = 0
            for x in torch.stack([o["kbytes"][0].to(dev) for o in outs]).tolist():
                orb |= int(x)
            alphabet = (0, 1 << max(1, orb.bit_length()))
        for pa, pb in groups:
            starts = offs[:, pa]
            lens = offs[:, pb] - offs[:, pa]
            m = int(lens.sum())
            if m == 0:
                continue
            # the group's keys lie between its partitions' splitters (inclusive
            # in hi): the bits above their highest differing bit need no pass
            hr = (spl_hi[pa - 1] if pa > 0 else 0,
                  spl_hi[pb - 1] if pb < nparts else (1 << 64) - 1) \
                if len(spl_hi) == nparts - 1 else None
            # the window's bounds: the group's splitters (None at the ends:
            # sort_gathered takes the group's own smallest / largest key)
            bnd = (spl_hi[pa - 1] if pa > 0 else None, spl_hi[pb - 1] if pb < nparts else None) \
                if len(spl_hi) == nparts - 1 else (None, None)
            if self.out:
                # output: each group's order is final before its part files
                recs, hs, ls = self._sorted_partition(his, los, rows, starts, lens, bases, dev,
                                                      hi_range=hr, gid=use_gid,
                                                      alphabet=alphabet, bounds=bnd)
            else:
                # in HBM: no host read per group; the tie-run flags are read
                # once after the last group (a flagged job is redone below)
                recs, hs, ls, flag = self._sorted_partition(his, los, rows, starts, lens, bases,
                                                            dev, hi_range=hr, defer=True,
                                                            gid=use_gid, alphabet=alphabet,
                                                            bounds=bnd)
                if flag is not None:
                    flags = flag if flags is None else flags + flag
            # order within the group and across the seam to the previous one,
            # and the key checksum, in one pass into gstats (no host read)
            S.tera_group_stats(hs, ls, prev_last, gstats)
            prev_last = (hs[-1:], ls[-1:])
            if first is None:
                first = (hs[:1], ls[:1])
            last = (hs[-1:], ls[-1:])
            n += m
            if self.out:
                at, items = 0, []
                for p in range(pa, pb):
                    items.append((p, recs[at:at + int(sizes[p])]))
                    at += int(sizes[p])
                self._write_parts(ctx, items)
            del recs
        if first is None:
            return 0, None, flags
        return n, torch.cat([gstats[:2], first[0], first[1], last[0], last[1]]), flags

    def _groups(self, sizes, nparts, limit):
        """Consecutive partitions in groups of at most ``limit`` record bytes
        (a single larger partition forms its own group)."""
        groups, pa = [], 0
        while pa < nparts:
            pb, acc = pa, 0
            while pb < nparts and (pb == pa or (acc + int(sizes[pb])) * S.RECORD <= limit):
                acc += int(sizes[pb])
                pb += 1
            groups.append((pa, pb))
            pa = pb
        return groups

    def _reduce_spill(self, ctx, outs, offs, nparts, dev):
        """Out-of-core reduce (ReduceTask's merge of spilled map outputs,
        ReduceTask.java:2421-2514, in-memory limit :1102-1111): per group of
        partitions no larger than a third of the HBM budget, every map's sorted
        run slice comes back from host memory, the runs are merged on their
        keys (merge path, log2 #runs passes) and the records gathered in
        merged order; peak HBM is about 2.3x the group."""
        sizes = (offs[:, 1:] - offs[:, :-1]).sum(axis=0)
        limit = self.budget // 3 if self.budget > 0 else self.group_bytes
        cuda = dev is not None and getattr(dev, "type", "") == "cuda"
        zero = torch.zeros((), dtype=torch.int64, device=dev)
        bad, csum = zero.clone(), zero.clone()
        prev_last = first = last = None
        n = 0
        for pa, pb in self._groups(sizes, nparts, limit):
            lens = offs[:, pb] - offs[:, pa]
            m = int(lens.sum())
            if m == 0:
                continue
            buf = torch.empty((m, S.RECORD), dtype=torch.uint8, device=dev)
            runs, at = [], 0
            for i, o in enumerate(outs):
                a, b = int(offs[i, pa]), int(offs[i, pb])
                if b <= a:
                    continue
                piece = buf[at:at + b - a]
                piece.copy_(o["spill"][a:b], non_blocking=cuda)
                h, lw = S.tera_keys(piece)
                runs.append((h, lw, torch.arange(at, at + b - a, dtype=torch.int32, device=dev)))
                at += b - a
            hs, ls, idx = S.merge_runs(runs)
            del runs
            recs = S.gather_records(buf, idx)
            del buf, idx
            bad = bad + S.count_unsorted_dev(hs, ls)
            if prev_last is not None:
                bad = bad + S.pair_greater(prev_last, (hs[:1], ls[:1]))
            prev_last = (hs[-1:], ls[-1:])
            if first is None:
                first = (hs[:1], ls[:1])
            last = (hs[-1:], ls[-1:])
            csum = csum + hs.sum() + ls.sum()
            n += m
            if self.out:
                at, items = 0, []
                for p in range(pa, pb):
                    items.append((p, recs[at:at + int(sizes[p])]))
                    at += int(sizes[p])
                self._write_parts(ctx, items)
            del recs, hs, ls
        if first is None:
            return 0, None
        return n, torch.cat([bad.reshape(1), csum.reshape(1), first[0], first[1], last[0],
                             last[1]])

    def _agree_parts(self, comm, outs, nparts):
        """R and the splitters, agreed by every rank (a rank may have run no map;
        every rank takes part, so the collective sequence is the same)."""
        nparts = max(int(g[0]) for g in comm.all_gather(
            torch.tensor([nparts or 0], dtype=torch.int64)))
        spl = None
        if nparts > 1:
            k = nparts - 1
            mine = torch.zeros(1 + 2 * k, dtype=torch.int64)
            if outs:
                shi, slo = _parse_keys(self._splitters_of(outs))
                assert shi.numel() == k, (shi.numel(), k)
                mine[0] = 1
                mine[1:1 + k] = shi
                mine[1 + k:] = slo
            for g in comm.all_gather(mine):
                g = g.cpu()
                if int(g[0]):
                    spl = (g[1:1 + k], g[1 + k:])
                    break
        return nparts, spl

    def _send_buffer(self, outs, offs, nparts, W, dev):
        """This rank's records for every destination rank, in destination
        order (one gather), and the per-destination counts."""
        counts = [0] * W
        splits, rowsl, perms = [], [], []
        if not outs:
            return torch.empty(0, S.RECORD, dtype=torch.uint8, device=dev), counts
        his = [o["hi"] for o in outs]
        los = [o["lo"] for o in outs]
        rows = [o["row"] for o in outs]
        bases = [o["records"] for o in outs]
        at = 0
        for d in range(W):
            a, b = self.owner_range(d, W, nparts)
            starts = offs[:, a]
            lens = offs[:, b] - offs[:, a]
            counts[d] = int(lens.sum())
            if counts[d]:
                h, lw, sp, rw = S.tera_collect(his, los, rows, starts, lens,
                                               with_keys=self.sorted_runs)
                if self.sorted_runs:
                    perm, _hs, _ls = S.sort_keys(h, lw)
                    perms.append(perm + at)
                splits.append(sp)
                rowsl.append(rw)
                at += counts[d]
        if not splits:
            return torch.empty(0, S.RECORD, dtype=torch.uint8, device=dev), counts
        return S.gather_records_multi(bases, torch.cat(splits), torch.cat(rowsl),
                                      torch.cat(perms) if perms else None), counts

    def _reduce_shuffle_waves(self, ctx, outs, marks, nparts, dev):
        """The shuffle in ``waves`` all-to-all-v rounds over this rank's map
        outputs in launch order: round g waits (on the device) only for its own
        maps' events, reads their partition offsets, gathers and sends their
        records, while later maps may still be running.  Every rank runs the
        same number of rounds (empty ones send nothing)."""
        comm = ctx.comm
        W, me = comm.world_size, comm.rank
        nparts, spl = self._agree_parts(comm, outs, nparts)
        cuda = dev.type == "cuda"
        cur = torch.cuda.current_stream() if cuda else None
        waves = self.waves_for(W)
        if self.static_a2a and not self.sorted_runs:
            got = self._shuffle_static(comm, outs, marks, nparts, waves, dev)
            if got is not None:
                recv, csum = got
                return self._sort_received(ctx, recv, spl, nparts, W, me, dev), csum
            # a slot overflowed on some rank: every rank re-runs the shuffle
            # with exact sizes (the maps' outputs are still held)
            if TRACE.on:
                TRACE.instant("tera.shuffle.static_overflow")
        n_local = len(outs)
        bounds = [n_local * g // waves for g in range(waves + 1)]
        csum = torch.zeros((), dtype=torch.int64, device=dev)
        recvs, rcs = [], []
        for g in range(waves):
            grp = outs[bounds[g]:bounds[g + 1]]
            if cuda:
                for m in {id(m): m for m in marks[bounds[g]:bounds[g + 1]]
                          if m is not None}.values():
                    cur.wait_event(m)
            offs = torch.stack([o["offsets"] for o in grp]).to("cpu").numpy() if grp else None
            if grp:
                csum = csum + torch.stack([o["checksum"].reshape(()) for o in grp]).sum()
            send, counts = self._send_buffer(grp, offs, nparts, W, dev)
            if TRACE.on:
                TRACE.instant("tera.wave.send", wave=g, records=int(sum(counts)))
            recv, rc = comm.all_to_all_v(send, counts)
            del send
            recvs.append(recv)
            rcs.append(rc)
        if self.sorted_runs:
            # runs arrive per (wave, source): merge them all
            recv = torch.cat(recvs)
            runs_counts = [c for rc in rcs for c in rc]
        else:
            recv = torch.cat(recvs)
        del recvs
        if recv.shape[0] == 0:
            return (0, None), csum
        if self.sorted_runs:
            srt, hs, ls = self._merge_received(recv, runs_counts)
            del recv
            return self._owned_stats(ctx, srt, hs, ls, spl, nparts, W, me, dev), csum
        return self._sort_received(ctx, recv, spl, nparts, W, me, dev), csum

    def _sort_received(self, ctx, recv, spl, nparts, W, me, dev):
        if recv.shape[0] == 0:
            return 0, None
        srt, hs, ls = S.sort_records(recv)
        del recv
        return self._owned_stats(ctx, srt, hs, ls, spl, nparts, W, me, dev)

    def _owned_stats(self, ctx, srt, hs, ls, spl, nparts, W, me, dev):
        n = int(srt.shape[0])
        st = torch.cat([S.count_unsorted_dev(hs, ls).reshape(1),
                        (hs.sum() + ls.sum()).reshape(1), hs[:1], ls[:1], hs[-1:], ls[-1:]])
        if self.out:
            self._write_owned(ctx, srt, hs, ls, spl, nparts, W, me, n, dev)
        return n, st

    def _slot_capacity(self, grp, nparts, W):
        """Records per destination slot of one wave: the wave's records times
        the largest destination's share of the partitions (sampled splitters
        cut near-equal partitions), times the slack, plus a floor.  Host-side
        shapes only — no device value is read."""
        rows = sum(int(o["row"].shape[0]) for o in grp)
        share = max(self.owner_range(d, W, nparts)[1] - self.owner_range(d, W, nparts)[0]
                    for d in range(W)) / max(1, nparts)
        return max(1024, int(rows * share * self.slot_slack) + 1024)

    def _shuffle_static(self, comm, outs, marks, nparts, waves, dev):
        """The shuffle waves as static-shape all-to-alls (see ``static_a2a``).
        Wave g: wait (on the device) for its maps' events; per-destination
        piece starts, lengths and slot prefixes from the maps' device offsets;
        one collect + gather into W slots of ``cap`` records; one all-to-all
        of the slots and one of the counts.  After the last wave ONE host read
        (the received counts and an all-reduced overflow flag) compacts the
        received slots.  Returns (received records, input checksum), or None
        if any rank's slot overflowed (the caller falls back, collectively)."""
        W = comm.world_size
        cuda = dev.type == "cuda"
        cur = torch.cuda.current_stream() if cuda else None
        n_local = len(outs)
        bounds = [n_local * g // waves for g in range(waves + 1)]
        own = [self.owner_range(d, W, nparts) for d in range(W)]
        ia = torch.tensor([a for a, _ in own], dtype=torch.int64, device=dev)
        ib = torch.tensor([b for _, b in own], dtype=torch.int64, device=dev)
        # the capacity must be the same on every rank (equal-split all-to-all):
        # the largest wave of any rank decides it (one small host collective
        # before any map output is read)
        caps = [self._slot_capacity(outs[bounds[g]:bounds[g + 1]], nparts, W) if
                bounds[g + 1] > bounds[g] else 0 for g in range(waves)]
        capt = torch.stack(comm.all_gather(torch.tensor(caps, dtype=torch.int64)))
        caps = [int(c) for c in capt.cpu().max(0).values.tolist()]
        csum = torch.zeros((), dtype=torch.int64, device=dev)
        over = torch.zeros((), dtype=torch.int64, device=dev)
        recvs, rcnts = [], []
        for g in range(waves):
            grp = outs[bounds[g]:bounds[g + 1]]
            cap = caps[g]
            if cap == 0:
                continue          # no rank has maps in this wave: nothing moves
            if cuda:
                for m in {id(m): m for m in marks[bounds[g]:bounds[g + 1]]
                          if m is not None}.values():
                    cur.wait_event(m)
            if grp:
                offs = torch.stack([o["offsets"].to(dev) for o in grp])      # [S, R+1]
                csum = csum + torch.stack([o["checksum"].reshape(()).to(dev)
                                           for o in grp]).sum()
                starts = offs.index_select(1, ia)                              # [S, W]
                lens = offs.index_select(1, ib) - starts
                pre = torch.cat([torch.zeros(W, 1, dtype=torch.int64, device=dev),
                                 lens.t().cumsum(1)], 1)                       # [W, S+1]
                cnt = pre[:, -1]
                over = over + (cnt > cap).sum()
                split, row = S.tera_collect_slots([o["row"] for o in grp], starts, pre, cap)
                send = S.gather_records_multi([o["records"] for o in grp], split, row)
                del split, row
                sent = torch.clamp(cnt, max=cap)
            else:
                send = torch.empty(W * cap, S.RECORD, dtype=torch.uint8, device=dev)
                sent = torch.zeros(W, dtype=torch.int64, device=dev)
            if TRACE.on:
                TRACE.instant("tera.wave.send_static", wave=g, cap=cap)
            recvs.append((comm.all_to_all_fixed(send), cap))
            rcnts.append(comm.all_to_all_fixed(sent))
            del send
        over = comm.all_reduce(over.reshape(1))
        if not recvs:
            return torch.empty(0, S.RECORD, dtype=torch.uint8, device=dev), csum
        # the one host read of the shuffle: received counts + the overflow flag
        host = torch.cat([over.reshape(1).to(dev)] + [r.to(dev) for r in rcnts]).cpu().tolist()
        if host[0]:
            return None
        pieces, at = [], 1
        for recv, cap in recvs:
            for src in range(W):
                c = int(host[at + src])
                if c:
                    pieces.append(recv[src * cap:src * cap + c])
            at += W
        recv = torch.cat(pieces) if pieces else recvs[0][0][:0]
        return recv, csum

    def _write_owned(self, ctx, srt, hs, ls, spl, nparts, W, me, n, dev):
        a, b = self.owner_range(me, W, nparts)
        if b - a > 1:
            if spl is None:
                raise RuntimeError("no rank holds the splitters of this job")
            shi, slo = spl
            cut = S.split_offsets(hs, ls, shi[a:b - 1].to(dev), slo[a:b - 1].to(dev)) \
                .to("cpu").tolist()
            cut = [0] + cut[1:-1] + [n]
        else:
            cut = [0, n]
        self._write_parts(ctx, [(p, srt[cut[i]:cut[i + 1]]) for i, p in enumerate(range(a, b))])

    def _reduce_shuffle(self, ctx, outs, offs, nparts, dev):
        """world > 1: every rank gathers the records of each destination's
        partition range from its splits (one pass), one all-to-all-v over
        RCCL/xGMI, then sorts what it received (its contiguous key range)."""
        comm = ctx.comm
        W, me = comm.world_size, comm.rank
        # a rank that ran no map learns R (and the splitters) from its peers
        nparts = max(int(g[0]) for g in comm.all_gather(
            torch.tensor([nparts or 0], dtype=torch.int64)))
        # ... and the splitters, which a rank owning several partitions needs to
        # cut its output (every rank takes part: the collective sequence must
        # not depend on whether a rank ran maps)
        spl = None
        if nparts > 1:
            k = nparts - 1
            mine = torch.zeros(1 + 2 * k, dtype=torch.int64)
            if outs:
                shi, slo = _parse_keys(self._splitters_of(outs))
                assert shi.numel() == k, (shi.numel(), k)
                mine[0] = 1
                mine[1:1 + k] = shi
                mine[1 + k:] = slo
            for g in comm.all_gather(mine):
                g = g.cpu()
                if int(g[0]):
                    spl = (g[1:1 + k], g[1 + k:])
                    break
        counts = [0] * W
        splits, rowsl, perms = [], [], []
        if outs:
            his = [o["hi"] for o in outs]
            los = [o["lo"] for o in outs]
            rows = [o["row"] for o in outs]
            bases = [o["records"] for o in outs]
            at = 0
            for d in range(W):
                a, b = self.owner_range(d, W, nparts)
                starts = offs[:, a]
                lens = offs[:, b] - offs[:, a]
                counts[d] = int(lens.sum())
                if counts[d]:
                    h, lw, sp, rw = S.tera_collect(his, los, rows, starts, lens,
                                                   with_keys=self.sorted_runs)
                    if self.sorted_runs:
                        perm, _hs, _ls = S.sort_keys(h, lw)
                        perms.append(perm + at)
                        del h, lw, _hs, _ls
                    splits.append(sp)
                    rowsl.append(rw)
                    at += counts[d]
            if splits:
                send = S.gather_records_multi(bases, torch.cat(splits), torch.cat(rowsl),
                                              torch.cat(perms) if perms else None)
            else:
                send = torch.empty(0, S.RECORD, dtype=torch.uint8, device=dev)
            del splits, rowsl, perms
        else:
            send = torch.empty(0, S.RECORD, dtype=torch.uint8, device=dev)
        recv, rcounts = comm.all_to_all_v(send, counts)
        del send
        if recv.shape[0] == 0:
            return 0, None
        if self.sorted_runs:
            srt, hs, ls = self._merge_received(recv, rcounts)
        else:
            srt, hs, ls = S.sort_records(recv)
        del recv
        n = int(srt.shape[0])
        st = torch.cat([S.count_unsorted_dev(hs, ls).reshape(1),
                        (hs.sum() + ls.sum()).reshape(1), hs[:1], ls[:1], hs[-1:], ls[-1:]])
        if self.out:
            a, b = self.owner_range(me, W, nparts)
            if b - a > 1:
                if spl is None:
                    raise RuntimeError("no rank holds the splitters of this job")
                shi, slo = spl
                cut = S.split_offsets(hs, ls, shi[a:b - 1].to(dev), slo[a:b - 1].to(dev)) \
                    .to("cpu").tolist()
                cut = [0] + cut[1:-1] + [n]
            else:
                cut = [0, n]
            self._write_parts(ctx, [(p, srt[cut[i]:cut[i + 1]])
                                    for i, p in enumerate(range(a, b))])
        return n, st

    @staticmethod
    def _merge_received(recv, rcounts):
        """recv holds one sorted run per source rank: merge them (K8)."""
        hi, lo = S.tera_keys(recv)
        runs, at = [], 0
        for c in rcounts:
            if c:
                idx = torch.arange(at, at + c, dtype=torch.int32, device=recv.device)
                runs.append((hi[at:at + c], lo[at:at + c], idx))
            at += c
        hs, ls, perm = S.merge_runs(runs)
        return S.gather_records(recv, perm), hs, ls

    def _splitters_of(self, outs):
        if not outs:
            raise RuntimeError("writing several partitions needs the splitters of a local map")
        return outs[0]["splitters"]

    # -- output (TeraOutputFormat + FileOutputCommitter) ---------------------------------
    def _open_output(self, ctx):
        """Part files go to the attempt's work directory and are committed
        (renamed into the output directory) when the reduce ends
        (FileOutputCommitter); ``terasort.final.sync`` (TeraSort sets it)
        fsyncs every part before it is closed (TeraOutputFormat.java:63-75)."""
        from ..mapred.committer import FileOutputCommitter
        com = FileOutputCommitter()
        attempt = getattr(ctx, "attempt_id", None) or "attempt_local_r_000000_0"
        com.setup_task(self.conf, attempt)
        dev = getattr(ctx, "device", None)
        ctx.tera_out = (com, attempt, com.work_path(self.conf, attempt),
                        _PartWriter(dev, self.conf.get_boolean("terasort.final.sync", True),
                                    self.conf.get_int("hbmr.terasort.output.writers", 16)))

    def _write_part(self, ctx, p, recs):
        self._write_parts(ctx, [(p, recs)])

    def _write_parts(self, ctx, items):
        """Partitions [(p, records)] that are ready together (one sort group)
        are written together: their pieces interleave, so the writers work
        on different files (one file's writes serialise on its inode)."""
        _com, _att, workdir, pw = ctx.tera_out
        pw.write_many([(os.path.join(workdir, f"part-{p:05d}"), recs) for p, recs in items])

    def _close_output(self, ctx, commit=True):
        """Close the part writer; commit the attempt's work directory only on
        success, else abort it (rmtree of the work path)."""
        out = getattr(ctx, "tera_out", None)
        if out is None:
            return
        ctx.tera_out = None
        com, attempt, _wd, pw = out
        try:
            pw.close()
        except BaseException:
            com.abort_task(self.conf, attempt)
            raise
        if not commit:
            com.abort_task(self.conf, attempt)
        elif com.needs_task_commit(self.conf, attempt):
            com.commit_task(self.conf, attempt)

    def job_succeeded(self, jip):
        if self.out:
            from ..mapred.committer import FileOutputCommitter
            FileOutputCommitter().commit_job(jip.conf)


# (nbuf, chunk) -> idle rings of pinned host buffers, reused across jobs: a
# writer takes a ring of its own (two reduces of one process — trackers of a
# LocalCluster — must never share one) and gives it back when it closes
_PINNED: dict = {}
_PINNED_LOCK = __import__("threading").Lock()


class _PartWriter:
    """Streams device record runs to part files (TeraOutputFormat's writes).

    Each run is cut into CHUNK-byte pieces; a piece is copied device -> host
    into a free buffer of a ring of pinned buffers on a copy stream (≈50 GB/s),
    and a pool of writer threads ``pwrite``s it at its offset in the file —
    pieces of one file may land in any order, several files are written at
    once — so D2H and file writes overlap and a fast filesystem sees
    ``hbmr.terasort.output.writers`` concurrent writers.  The piece that
    completes a file flushes it, fsyncs it (``terasort.final.sync``) and
    closes it: at most the files in flight are open.  CPU tensors are written
    by the same pool.  The pinned ring is allocated once per process."""

    CHUNK = 64 << 20

    def __init__(self, device, final_sync, writers=8):
        import concurrent.futures as cf
        import threading
        self.sync = final_sync
        self.writers = max(1, int(writers))
        self.pool = cf.ThreadPoolExecutor(self.writers, thread_name_prefix="tera-out")
        self.cuda = device is not None and getattr(device, "type", "") == "cuda"
        self.lock = threading.Lock()
        self.files = []              # futures of every piece
        self.k = 0
        self.errors = []
        if self.cuda:
            nbuf = 2 * self.writers
            key = (nbuf, self.CHUNK)
            with _PINNED_LOCK:
                idle = _PINNED.setdefault(key, [])
                bufs = idle.pop() if idle else None
            if bufs is None:
                bufs = [torch.empty(self.CHUNK, dtype=torch.uint8, pin_memory=True)
                        for _ in range(nbuf)]
            self.ring_key = key
            self.bufs = bufs
            self.pending = [None] * nbuf
            self.stream = torch.cuda.Stream(device)

    def _piece(self, fd, st, view, off, ev=None):
        try:
            if ev is not None:
                ev.synchronize()
            mv = memoryview(view)
            done = 0
            while done < len(mv):
                done += os.pwrite(fd, mv[done:], off + done)
        finally:
            with self.lock:
                st[0] -= 1
                last = st[0] == 0
            if last:
                if self.sync:
                    os.fsync(fd)
                os.close(fd)

    def write(self, path, recs):
        self.write_many([(path, recs)])

    def write_many(self, items):
        """Several files at once: piece i of every file before piece i + 1 of
        any, so the writers in flight hold different files."""
        files = []
        for path, recs in items:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            flat = recs.reshape(-1)
            n = flat.numel()
            pieces = max(1, -(-n // self.CHUNK))
            st = [pieces]
            if n == 0:
                self.files.append(self.pool.submit(self._piece, fd, st, b"", 0))
                continue
            if not self.cuda or not flat.is_cuda:
                a = flat.numpy()
                for i in range(pieces):
                    o = i * self.CHUNK
                    self.files.append(self.pool.submit(self._piece, fd, st,
                                                       a[o:o + self.CHUNK], o))
                continue
            self.stream.wait_stream(torch.cuda.current_stream(flat.device))
            flat.record_stream(self.stream)
            files.append((fd, st, flat, n, pieces))
        for i in range(max((f[4] for f in files), default=0)):
            for fd, st, flat, n, pieces in files:
                if i >= pieces:
                    continue
                o = i * self.CHUNK
                c = min(self.CHUNK, n - o)
                j = self.k % len(self.bufs)
                self.k += 1
                if self.pending[j] is not None:
                    self.pending[j].result()          # the buffer's previous piece is out
                buf = self.bufs[j]
                with torch.cuda.stream(self.stream):
                    buf[:c].copy_(flat[o:o + c], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                fut = self.pool.submit(self._piece, fd, st, buf[:c].numpy(), o, ev)
                self.pending[j] = fut
                self.files.append(fut)

    def close(self):
        try:
            for fut in self.files:
                fut.result()
        finally:
            self.pool.shutdown()
            self.files = []
            bufs = getattr(self, "bufs", None)
            if bufs is not None:
                # every piece is written (or failed): the ring is free again
                self.bufs = None
                with _PINNED_LOCK:
                    _PINNED.setdefault(self.ring_key, []).append(bufs)


def terasort_conf(base=None, rows=1_000_000, split_rows=None, output=None, inp=None,
                  partitions=0):
    from ..mapred.jobconf import JobConf
    job = JobConf(base)
    job.set_job_name(f"TeraSort {inp or rows}")
    job.set("hbmr.splitjob.class", "hbmr.models.terasort:TeraSortSplitJob")
    job.set(INPUT_KEY, inp or f"teragen:{rows}")
    if split_rows:
        job.set_long(SPLIT_ROWS_KEY, split_rows)
    if partitions:
        job.set_int(PARTS_KEY, partitions)
    if output:
        job.set("mapred.output.dir", output)
    return job


# --------------------------------------------------------------------------- TeraGen job
class TeraGenSplitJob(SplitJob):
    """Map-only TeraGen: each map writes ``part-NNNNN`` with its rows (generated
    on its GPU, or with the CPU twin on CPU slots) — TeraGen.java's output."""

    collective_reduce = True
    needs_reduce = False

    def configure(self, conf):
        self.conf = conf
        self.rows = conf.get_long("terasort.num-rows", 1000)
        self.split_rows = conf.get_long(SPLIT_ROWS_KEY, 10_000_000)
        self.out = conf.get("mapred.output.dir")

    def get_splits(self, conf, trackers):
        out = []
        nsplit = max(1, -(-self.rows // self.split_rows))
        for i in range(nsplit):
            a = i * self.split_rows
            n = min(self.split_rows, self.rows - a)
            loc = [trackers[i * len(trackers) // nsplit]] if trackers else []
            out.append(SplitSpec(i, f"teragen-out:{a}:{n}", "teragen", {"first": a, "rows": n},
                                 loc, n * S.RECORD))
        return out

    def load_split(self, spec, device):
        return spec

    def split_nbytes(self, data):
        return 0

    def _map(self, ctx, spec):
        p = spec.params
        dev = ctx.device if ctx.device is not None else "cpu"
        recs = S.teragen(p["first"], p["rows"], device=dev)
        os.makedirs(self.out, exist_ok=True)
        recs.to("cpu").numpy().tofile(os.path.join(self.out, f"part-{spec.index:05d}"))
        ctx.reporter.incrCounter(C.TASK_GROUP, C.MAP_OUTPUT_RECORDS, p["rows"])
        return p["rows"]

    def map_gpu(self, ctx, data):
        return self._map(ctx, data)

    def map_cpu(self, ctx, data):
        return self._map(ctx, data)

    def map_gpu_batch(self, ctxs, datas):
        return [self._map(c, d) for c, d in zip(ctxs, datas)]


def teragen_conf(base=None, rows=1000, output=None, split_rows=None):
    from ..mapred.jobconf import JobConf
    job = JobConf(base)
    job.set_job_name(f"TeraGen {rows}")
    job.set("hbmr.splitjob.class", "hbmr.models.terasort:TeraGenSplitJob")
    job.set_long("terasort.num-rows", rows)
    if split_rows:
        job.set_long(SPLIT_ROWS_KEY, split_rows)
    job.set("mapred.output.dir", output)
    return job


def teravalidate(path, progress=None) -> dict:
    """TeraValidate over the part files of ``path`` in name order: records out of
    order within a file or across file boundaries, total records and an
    order-independent key checksum (sum of the 10-byte keys mod 2^64).
    ``progress(i, nfiles)`` is called before each file."""
    files = sorted(f for f in os.listdir(path) if f.startswith("part-"))
    bad = 0
    total = 0
    csum = 0
    prev_last = None
    for i, fn in enumerate(files):
        if progress is not None:
            progress(i, len(files))
        recs = np.fromfile(os.path.join(path, fn), dtype=np.uint8)
        if recs.size % S.RECORD:
            raise ValueError(f"{fn}: not a whole number of 100-byte records")
        recs = recs.reshape(-1, S.RECORD)
        if not recs.shape[0]:
            continue
        hi, lo = _key_words(recs[:, :10])
        h = torch.from_numpy(hi.view(np.int64))
        lw = torch.from_numpy(lo.view(np.int64))
        bad += S.count_unsorted(h, lw)
        first = (int(hi[0]), int(lo[0]))
        if prev_last is not None and first < prev_last:
            bad += 1
        prev_last = (int(hi[-1]), int(lo[-1]))
        total += recs.shape[0]
        csum = (csum + int(hi.sum(dtype=np.uint64)) + int(lo.sum(dtype=np.uint64))) % (1 << 64)
    return {"files": len(files), "records": total, "misordered": bad, "checksum": csum}


def _cli_cluster(cluster):
    if cluster is not None:
        return cluster, False
    from ..mapred.cluster import LocalCluster
    from ..mapred.jobconf import JobConf
    gpus = [[0]] if torch.cuda.is_available() else None
    return LocalCluster(JobConf(), num_trackers=1, gpus=gpus), True


def main_teragen(argv=None, cluster=None):
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr teragen")
    ap.add_argument("rows", type=int)
    ap.add_argument("output")
    ap.add_argument("--split-rows", type=int, default=10_000_000)
    a = ap.parse_args(argv)
    cl, own = _cli_cluster(cluster)
    try:
        rj = cl.submit_job(teragen_conf(rows=a.rows, output=a.output, split_rows=a.split_rows))
        rj.waitForCompletion()
        return 0 if rj.isSuccessful() else 1
    finally:
        if own:
            cl.shutdown()


def main_terasort(argv=None, cluster=None):
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr terasort")
    ap.add_argument("input", help="directory of TeraGen files, or teragen:<rows>")
    ap.add_argument("output")
    ap.add_argument("--split-rows", type=int, default=10_000_000)
    a = ap.parse_args(argv)
    cl, own = _cli_cluster(cluster)
    try:
        inp = a.input if a.input.startswith("teragen:") else os.path.abspath(a.input)
        rj = cl.submit_job(terasort_conf(inp=inp, output=a.output, split_rows=a.split_rows))
        rj.waitForCompletion()
        if rj.isSuccessful():
            print(rj._impl.jip.result)
        return 0 if rj.isSuccessful() else 1
    finally:
        if own:
            cl.shutdown()


def main_teravalidate(argv=None, cluster=None):
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr teravalidate")
    ap.add_argument("output")
    a = ap.parse_args(argv)
    r = teravalidate(a.output)
    print(r)
    return 0 if r["misordered"] == 0 else 1
