"""``hbmr test <program>`` — the AllTestDriver analogue (hadoop-test.jar)."""
from __future__ import annotations

import importlib
import sys

PROGRAMS = {
    "TestDFSIO": ("hbmr.benchmarks.dfsio:main", "Distributed i/o benchmark."),
    "nnbench": ("hbmr.benchmarks.nnbench:main", "A benchmark that stresses the namenode."),
    "mrbench": ("hbmr.benchmarks.mrbench:main", "A map/reduce benchmark that can create many small jobs"),
    "testbigmapoutput": ("hbmr.benchmarks.bigmapoutput:main_bigmapoutput",
                         "A map/reduce program that works on a very big non-splittable file and does identity map/reduce"),
    "threadedmapbench": ("hbmr.benchmarks.bigmapoutput:main_threadedmap",
                         "A map/reduce benchmark that compares the performance of maps with multiple spills over maps with 1 spill"),
    "sortvalidate": ("hbmr.benchmarks.sortvalidator:main",
                     "A map/reduce program that validates the map-reduce framework's sort."),
}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in PROGRAMS:
        print("Valid program names are:\n" + "\n".join(
            f"  {k}: {v[1]}" for k, v in sorted(PROGRAMS.items())), file=sys.stderr)
        return -1
    mod, fn = PROGRAMS[argv[0]][0].split(":")
    return getattr(importlib.import_module(mod), fn)(argv[1:]) or 0
