"""PiEstimator: quasi-Monte Carlo estimate of pi
(src/examples/org/apache/hadoop/examples/PiEstimator.java).

Each map takes (offset, size), walks ``size`` points of the 2-D Halton sequence
(bases 2 and 3) from index ``offset``, and counts points inside / outside the
inscribed circle; one reducer sums the counts.  pi ≈ 4 · inside / total.
The map's inner loop is vectorised over numpy (the reference's Java loop).

:class:`PiSplitJob` is the GPU form: each map task is one launch of the fp64
Halton kernel (native/kernels/pi.hip) on its GPU slot's stream — bit-exact with
the numpy map, so CPU and GPU slots can share a job under the hybrid
scheduler — and the reduce is a collective sum."""
from __future__ import annotations

import argparse
import os
import tempfile
from decimal import Decimal

import numpy as np

from ..io import sequencefile as seqf
from ..io.writable import BooleanWritable, LongWritable
from ..mapred import FileInputFormat, FileOutputFormat, JobClient, JobConf, Mapper, Reducer
from ..mapred.formats import SequenceFileInputFormat, SequenceFileOutputFormat


def halton(index: np.ndarray, base: int) -> np.ndarray:
    """Radical inverse of ``index + 1`` in ``base`` (vectorised)."""
    i = index.astype(np.int64) + 1
    f = np.ones(i.shape, dtype=np.float64) / base
    r = np.zeros(i.shape, dtype=np.float64)
    while np.any(i > 0):
        r += f * (i % base)
        i //= base
        f /= base
    return r


class PiMapper(Mapper):
    def map(self, key, value, output, reporter):
        offset, size = key.get(), value.get()
        inside = 0
        chunk = 1 << 20
        for a in range(0, size, chunk):
            idx = np.arange(offset + a, offset + min(size, a + chunk), dtype=np.int64)
            x = halton(idx, 2) - 0.5
            y = halton(idx, 3) - 0.5
            inside += int(np.count_nonzero(x * x + y * y <= 0.25))
            reporter.progress()
        output.collect(BooleanWritable(True), LongWritable(inside))
        output.collect(BooleanWritable(False), LongWritable(size - inside))


class PiReducer(Reducer):
    def reduce(self, key, values, output, reporter):
        output.collect(key, LongWritable(sum(v.get() for v in values)))


def estimate(maps, samples, conf=None, cluster=None, verbose=False):
    tmp = tempfile.mkdtemp(prefix="pi-")
    inp, out = os.path.join(tmp, "in"), os.path.join(tmp, "out")
    os.makedirs(inp)
    for i in range(maps):
        with seqf.Writer(os.path.join(inp, f"part{i}"), LongWritable, LongWritable) as w:
            w.append(LongWritable(i * samples), LongWritable(samples))
    job = JobConf(conf)
    job.set_job_name("PiEstimator")
    job.set_input_format(SequenceFileInputFormat)
    job.set_output_format(SequenceFileOutputFormat)
    job.set_output_key_class(BooleanWritable)
    job.set_output_value_class(LongWritable)
    job.set_mapper_class(PiMapper)
    job.set_reducer_class(PiReducer)
    job.set_num_reduce_tasks(1)
    job.set_speculative_execution(False)
    FileInputFormat.setInputPaths(job, inp)
    FileOutputFormat.setOutputPath(job, out)
    JobClient.runJob(job, cluster=cluster, verbose=verbose)
    counts = {}
    for fn in os.listdir(out):
        if fn.startswith("part-"):
            with seqf.Reader(os.path.join(out, fn)) as r:
                for k, v in r:
                    counts[bool(k.get())] = v.get()
    inside, outside = counts.get(True, 0), counts.get(False, 0)
    return Decimal(4) * Decimal(inside) / Decimal(inside + outside)


from ..gpu.splitjob import SplitJob, SplitSpec  # noqa: E402


class PiSplitJob(SplitJob):
    collective_reduce = True
    needs_reduce = True

    def configure(self, conf):
        self.conf = conf
        self.maps = conf.get_int("hbmr.pi.maps", 1)
        self.samples = conf.get_long("hbmr.pi.samples", 1000)

    def get_splits(self, conf, trackers):
        out = []
        for i in range(self.maps):
            loc = [trackers[i * len(trackers) // self.maps]] if trackers else []
            out.append(SplitSpec(i, f"pi:{i}:{self.samples}", "range",
                                 {"offset": i * self.samples, "size": self.samples}, loc, 0))
        return out

    def load_split(self, spec, device):
        return (spec.params["offset"], spec.params["size"])

    def load_split_sample(self, spec, device, fraction):
        return (spec.params["offset"], max(1, int(spec.params["size"] * fraction)))

    def split_nbytes(self, data):
        return 0

    def map_gpu(self, ctx, data):
        from ..ops import pi as P
        return (P.count_inside_gpu(data[0], data[1], stream=getattr(ctx, "stream", None)),
                data[1])

    def map_cpu(self, ctx, data):
        from ..ops import pi as P
        return (P.count_inside_cpu(data[0], data[1]), data[1])

    def combine(self, ctx, outputs):
        import torch
        inside = sum(int(o[0].item()) if hasattr(o[0], "item") else int(o[0]) for o in outputs)
        return torch.tensor([inside, sum(o[1] for o in outputs)], dtype=torch.int64)

    def reduce(self, ctx, combined):
        t = combined
        if ctx.device is not None and ctx.device.type == "cuda":
            t = t.to(ctx.device)
        ctx.comm.all_reduce(t)
        inside, total = (int(x) for x in t.cpu().tolist())
        return {"inside": inside, "total": total,
                "pi": str(Decimal(4) * Decimal(inside) / Decimal(max(total, 1)))}


def split_job_conf(maps, samples, base=None) -> JobConf:
    job = JobConf(base)
    job.set_job_name("PiEstimator (split job)")
    job.set("hbmr.splitjob.class", "hbmr.examples.pi:PiSplitJob")
    job.set_int("hbmr.pi.maps", maps)
    job.set_long("hbmr.pi.samples", samples)
    return job


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr pi")
    ap.add_argument("maps", type=int)
    ap.add_argument("samples", type=int)
    ap.add_argument("-split", action="store_true",
                    help="run as a split-level job (GPU slots when a GPU is present)")
    a = ap.parse_args(argv)
    print(f"Number of Maps  = {a.maps}\nSamples per Map = {a.samples}")
    if a.split:
        import torch
        from ..mapred.cluster import LocalCluster
        gpus = [[i for i in range(torch.cuda.device_count())]] if torch.cuda.is_available() \
            else None
        own = cluster is None
        cl = cluster or LocalCluster(JobConf(), num_trackers=1, gpus=gpus)
        try:
            rj = cl.submit_job(split_job_conf(a.maps, a.samples))
            rj.waitForCompletion()
            if not rj.isSuccessful():
                print(f"job failed: {rj.getFailureInfo()}")
                return 1
            pi = rj._impl.jip.result[0]["pi"]
        finally:
            if own:
                cl.shutdown()
        print(f"Estimated value of Pi is {pi}")
        return 0
    pi = estimate(a.maps, a.samples, cluster=cluster, verbose=True)
    print(f"Estimated value of Pi is {pi}")
    return 0
