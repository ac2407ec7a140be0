"""Split-level jobs: the GPU-native job model (hbmr extension).

A classic Hadoop job streams one record at a time through map() — for a GPU
task the reference did that over a loopback socket, one Pipes MAP_ITEM per
record.  A :class:`SplitJob` instead hands a whole input split
to the device: the split is materialised once in HBM (and kept there by the
tracker's :class:`~hbmr.gpu.split_cache.SplitCache` across jobs, so iterative
algorithms re-read nothing from the host), the map is a few kernel launches
on the slot's HIP stream, the per-task output is a small device tensor (the
combiner is fused into the map), and the shuffle + reduce is a collective
(RCCL over xGMI) among the trackers, one pinned reduce per tracker.

Subclasses implement:

* ``get_splits(conf, trackers)``   -> list[SplitSpec]  (locations = preferred trackers)
* ``load_split(spec, device)``     -> split data on ``device`` ("cpu" for CPU slots)
* ``map_gpu(ctx, data)``           -> map output (device tensors), kernels on ctx.stream
* ``map_cpu(ctx, data)``           -> map output (host tensors)
* ``load_split_sample(spec, dev, f)`` -> first fraction f of a split (profiling probes)
* ``combine(ctx, outputs)``        -> one combined output on this tracker
* ``reduce(ctx, combined)``        -> result (collectives via ctx.comm)
* ``job_succeeded(jip)``           -> optional hook on the JobTracker
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class SplitSpec:
    index: int
    key: str                      # cache key: identifies the split's bytes
    kind: str = "synthetic"       # "synthetic" | "file" | "range"
    params: dict = field(default_factory=dict)
    locations: list = field(default_factory=list)
    length: int = 0               # bytes (for split-size bookkeeping)

    def to_dict(self):
        # shallow (dataclasses.asdict deep-copies: ~25 µs per split per job)
        return {"index": self.index, "key": self.key, "kind": self.kind, "params": self.params,
                "locations": self.locations, "length": self.length}

    @classmethod
    def from_dict(cls, d):
        return cls(**{k: d[k] for k in ("index", "key", "kind", "params", "locations", "length")
                      if k in d})


class SplitJob:
    #: one reduce per tracker, run as a collective gang
    collective_reduce = True
    needs_reduce = True

    def configure(self, conf):
        self.conf = conf

    def get_splits(self, conf, trackers):
        raise NotImplementedError

    def load_split(self, spec: SplitSpec, device):
        raise NotImplementedError

    def load_split_sample(self, spec: SplitSpec, device, fraction: float):
        """The first ``fraction`` of a split (a sampled CPU profiling probe times
        the map on it and scales up).  Default: load and slice along dim 0."""
        data = self.load_split(spec, device)
        n = max(1, int(data.shape[0] * fraction))
        return data[:n]

    def split_nbytes(self, data) -> int:
        try:
            return int(data.numel() * data.element_size())
        except AttributeError:
            return 0

    def map_gpu(self, ctx, data):
        raise NotImplementedError

    def map_cpu(self, ctx, data):
        raise NotImplementedError

    def combine(self, ctx, outputs):
        raise NotImplementedError

    def reduce(self, ctx, combined):
        raise NotImplementedError

    def job_succeeded(self, jip):
        pass
