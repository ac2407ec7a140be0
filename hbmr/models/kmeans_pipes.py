"""K-Means through Pipes task binaries — BASELINE config 2 (and the paper's setup).

The fork's users ran K-Means as a Hadoop Pipes job with two executables: a
CPU binary for CPU map slots and a GPU binary for GPU map slots
(`-cpubin`/`-gpubin`, Submitter.java:419-420, 523-529), one Lloyd iteration
per job with the centroids side-loaded from a file.  This module drives the
same shape against hbmr's binaries (native/apps/kmeans_cpu.cc,
native/apps/kmeans_gpu.hip):

* input: SequenceFile<LongWritable, FloatVectorWritable> points
  (:func:`write_points`), split by FileInputFormat;
* the C++ record reader hands each map its whole split; maps emit exact
  int64 fixed-point (count, sums) partials per cluster;
* reducers (CPU, C++) emit ``cluster \\t c0,c1,...``; :func:`read_centroids`
  folds the part files into the next centroid file (clusters that received
  no point keep their previous centroid).

The in-process split-level job (hbmr.models.kmeans) is the fast path; this is
the compatibility path for Pipes users, and both produce bit-identical
centroids from the same inputs (same fixed-point partials, same update rule).
"""
from __future__ import annotations

import os
import struct

import numpy as np
import torch

from ..io import sequencefile as seqf
from ..io.writable import BytesWritable, FloatVectorWritable, IntWritable, LongWritable, Text
from ..mapred import FileInputFormat, FileOutputFormat, JobConf
from . import kmeans as K

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.path.join(ROOT, "hbmr", "bin")


def write_points(path, n, d, seed=1, centers=8, files=1, bf16_exact=True, chunk=1 << 16,
                 compression="NONE", codec=None):
    """Synthetic Gaussian-mixture points (hbmr.models.kmeans.synthetic_points) as
    ``files`` SequenceFiles under directory ``path``.  ``bf16_exact`` rounds the
    values to bf16 first, so CPU fp32 and GPU bf16 maps see identical data."""
    os.makedirs(path, exist_ok=True)
    per = -(-n // files)
    out = []
    for fi in range(files):
        a, b = fi * per, min(n, (fi + 1) * per)
        fn = os.path.join(path, f"points-{fi:05d}.seq")
        if compression == "NONE" and codec is None:
            # native writer (native/io/seqpoints.cc): same bytes, ~100x faster
            from ..io import nativeio
            x = K.synthetic_points(seed, a, b - a, d, centers, "cpu")
            if bf16_exact:
                x = x.to(torch.bfloat16).to(torch.float32)
            nativeio.write_points(fn, x.numpy(), first_id=a)
            out.append(fn)
            continue
        with seqf.Writer(fn, LongWritable, FloatVectorWritable, compression=compression,
                         codec=codec) as w:
            for c0 in range(a, b, chunk):
                c1 = min(b, c0 + chunk)
                x = K.synthetic_points(seed, c0, c1 - c0, d, centers, "cpu")
                if bf16_exact:
                    x = x.to(torch.bfloat16).to(torch.float32)
                xb = x.numpy().astype(">f4")
                hdr = struct.pack(">i", d)
                for i in range(c1 - c0):
                    w.append_raw(struct.pack(">q", c0 + i), hdr + xb[i].tobytes())
        out.append(fn)
    return out


def write_centroids(path, cen: torch.Tensor):
    cen = cen.detach().to("cpu", torch.float32)
    with seqf.Writer(path, IntWritable, FloatVectorWritable) as w:
        for j in range(cen.shape[0]):
            w.append(IntWritable(j), FloatVectorWritable(cen[j].numpy()))
    return path


def read_centroids(outdir, old: torch.Tensor) -> torch.Tensor:
    """The reducers' ``cluster \t c0,c1,...`` lines folded into the next
    centroids (clusters without a line keep theirs).  One numpy parse of all
    the values (the reducer prints %.9g: every fp32 round-trips exactly).
    Binary output (hbmr.kmeans.pipes.binary.output): SequenceFile parts of
    (Text cluster, BytesWritable d little-endian fp32) — the same floats."""
    new = old.detach().to("cpu", torch.float32).numpy().copy()
    keys, vals = [], []
    parts = [fn for fn in sorted(os.listdir(outdir)) if fn.startswith("part-")]
    if parts and _is_seqfile(os.path.join(outdir, parts[0])):
        rows = []
        for fn in parts:
            with seqf.Reader(os.path.join(outdir, fn)) as r:
                while True:
                    raw = r.next_raw()
                    if raw is None:
                        break
                    kb, vb = raw
                    keys.append(int(Text.deserialize(kb).bytes))
                    rows.append(BytesWritable.deserialize(vb).bytes)
        if keys:
            arr = np.frombuffer(b"".join(rows), dtype="<f4")
            new[np.asarray(keys)] = arr.reshape(len(keys), -1)
        return torch.from_numpy(new)
    for fn in parts:
        with open(os.path.join(outdir, fn)) as f:
            for line in f:
                k, sep, v = line.rstrip("\n").partition("\t")
                if sep:
                    keys.append(int(k))
                    vals.append(v)
    if keys:
        arr = np.array(",".join(vals).split(","), dtype=np.float64).astype(np.float32)
        new[np.asarray(keys)] = arr.reshape(len(keys), -1)
    return torch.from_numpy(new)


def _is_seqfile(path) -> bool:
    with open(path, "rb") as f:
        return f.read(3) == b"SEQ"


def iteration_conf(base, inp, out, cen_file, k, d, cpubin=None, gpubin=None, reduces=1,
                   maps=None, reuse=True, exact=True, block=True, binary=True) -> JobConf:
    from ..pipes import submitter
    job = JobConf(base)
    job.set_job_name(f"kmeans-pipes {os.path.basename(out)}")
    FileInputFormat.setInputPaths(job, inp)
    FileOutputFormat.setOutputPath(job, out)
    job.set("mapred.input.format.class", "hbmr.mapred.formats:SequenceFileInputFormat")
    job.set_boolean("hadoop.pipes.java.recordreader", False)
    job.set_boolean("hadoop.pipes.java.recordwriter", True)
    job.set_int("hbmr.kmeans.k", k)
    job.set_int("hbmr.kmeans.dims", d)
    job.set("hbmr.kmeans.centroids.file", os.path.abspath(cen_file))
    # exact mode (hbmr.kmeans.exact): both binaries give the fp64 arg-min of the
    # fp32 points and the fixed point of the fp32 rows — the same partials
    # whichever slots ran a map, so a hybrid job's centroids do not depend on
    # the placement (the bf16 GPU mode differs from the CPU binary on near-ties)
    job.set_boolean("hbmr.kmeans.exact", exact)
    # block mode (kmeans_pipes.h): one record per map carrying every cluster's
    # partial (in-mapper combining) instead of one record per cluster — the
    # same int64 partials, a k-th of the frames through the parent.  A block
    # has one key, so it would send every partial to one reducer: with several
    # reduces the per-cluster records spread them instead
    if block and reduces > 1:
        block = False
    job.set_boolean("hbmr.kmeans.pipes.block", block)
    # kmeans_gpu reads only job-level keys: the shared GPU child takes the
    # conf once per job (hbmr/pipes/mux.py)
    job.set_boolean("hbmr.pipes.gpu.mux.shared.conf", True)
    # the new centroids as raw fp32 bytes in a SequenceFile (read_centroids),
    # not %.9g text: the same floats without a format and a parse per value
    job.set_boolean("hbmr.kmeans.pipes.binary.output", binary)
    if binary:
        job.set("mapred.output.format.class", "hbmr.mapred.formats:SequenceFileOutputFormat")
        job.set_output_key_class(Text)
        job.set_output_value_class(BytesWritable)
    # every map's partials block stays in the reduce's memory (a 1,024-cluster
    # block is ~1 MB per map)
    job.set_int("hbmr.reduce.shuffle.memory.mb",
                max(512, (4 * k * (d + 1) * 8 * max(maps or 0, 128)) >> 20))
    # keep the task binaries alive across tasks and iteration jobs: the GPU
    # binary keeps its HIP context and the HBM-resident splits
    job.set_boolean("hbmr.pipes.child.reuse", reuse)
    job.set_num_reduce_tasks(reduces)
    if maps:
        job.set_num_map_tasks(maps)
    if cpubin:
        submitter.set_executable(job, cpubin)
    if gpubin:
        submitter.set_gpu_executable(job, gpubin)
    return job


class KMeansPipesDriver:
    """Chains Pipes K-Means iterations (one job each)."""

    def __init__(self, workdir, inp, k, d, init: torch.Tensor, base=None, cluster=None,
                 cpubin=os.path.join(BIN, "kmeans_cpu"), gpubin=os.path.join(BIN, "kmeans_gpu"),
                 reduces=1, maps=None, exact=True, block=True, binary=True):
        self.workdir, self.inp, self.k, self.d = workdir, inp, k, d
        self.block, self.binary = block, binary
        self.base, self.cluster = base, cluster
        self.cpubin, self.gpubin, self.reduces, self.maps = cpubin, gpubin, reduces, maps
        self.exact = exact
        self.centroids = init.detach().to("cpu", torch.float32)
        self.iteration = 0
        self.history = []
        os.makedirs(workdir, exist_ok=True)

    def step(self):
        from ..pipes import submitter
        i = self.iteration
        cen_file = write_centroids(os.path.join(self.workdir, f"centroids-{i:03d}.seq"),
                                   self.centroids)
        out = os.path.join(self.workdir, f"iter-{i:03d}")
        job = iteration_conf(self.base, self.inp, out, cen_file, self.k, self.d, self.cpubin,
                             self.gpubin, self.reduces, self.maps, exact=self.exact,
                             block=self.block, binary=self.binary)
        from ..utils.trace import TRACE
        if TRACE.on:
            TRACE.instant("kmeans_pipes.submit")
        rj = submitter.run_job(job, cluster=self.cluster, verbose=False)
        if TRACE.on:
            TRACE.instant("kmeans_pipes.job_done")
        if not rj.isSuccessful():
            raise RuntimeError(f"K-Means Pipes iteration {i} failed: {rj.getFailureInfo()}")
        new = read_centroids(out, self.centroids)
        if TRACE.on:
            TRACE.instant("kmeans_pipes.centroids_read")
        shift = float((new - self.centroids).norm(dim=1).max())
        self.centroids = new
        self.history.append({"iteration": i, "shift": shift, "counters": rj.getCounters()})
        self.iteration += 1
        return self.history[-1]

    def run(self, iters):
        for _ in range(iters):
            self.step()
        return self.centroids


def main(argv=None, cluster=None):
    """``hbmr examples kmeans-pipes <points-dir> <workdir> --k K --dims D --iters I``."""
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr kmeans-pipes")
    ap.add_argument("input")
    ap.add_argument("workdir")
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--reduces", type=int, default=1)
    ap.add_argument("--exact", action=argparse.BooleanOptionalAction, default=True,
                    help="fp64-exact labels on both binaries (default; --no-exact: bf16 GPU maps)")
    a = ap.parse_args(argv)
    init = K.initial_centroids(a.input, a.k, a.dims, exact=a.exact)
    drv = KMeansPipesDriver(a.workdir, a.input, a.k, a.dims, init, cluster=cluster,
                            reduces=a.reduces, exact=a.exact)
    for _ in range(a.iters):
        r = drv.step()
        print(f"iteration {r['iteration']}: shift {r['shift']:.6f}")
    return 0
