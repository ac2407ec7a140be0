"""ExampleDriver: ``hbmr examples <program> [args]`` (src/examples/org/apache/
hadoop/examples/ExampleDriver.java:38-63, plus the hbmr GPU workloads)."""
from __future__ import annotations

import importlib
import sys

PROGRAMS = {
    "aggregatewordcount": ("hbmr.examples.aggregatewordcount:main",
                           "An Aggregate based map/reduce program that counts the words in the input files."),
    "aggregatewordhist": ("hbmr.examples.aggregatewordcount:main_histogram",
                          "An Aggregate based map/reduce program that computes the histogram of the words in the input files."),
    "dbcount": ("hbmr.examples.dbcount:main", "An example job that count the pageview counts from a database."),
    "grep": ("hbmr.examples.grep:main", "A map/reduce program that counts the matches of a regex in the input."),
    "join": ("hbmr.examples.join:main", "A job that effects a join over sorted, equally partitioned datasets"),
    "multifilewc": ("hbmr.examples.multifilewc:main", "A job that counts words from several files."),
    "pentomino": ("hbmr.examples.dancing:main_pentomino", "A map/reduce tile laying program to find solutions to pentomino problems."),
    "pi": ("hbmr.examples.pi:main", "A map/reduce program that estimates Pi using monte-carlo method."),
    "randomtextwriter": ("hbmr.examples.randomwriter:main_text", "A map/reduce program that writes 10GB of random textual data per node."),
    "randomwriter": ("hbmr.examples.randomwriter:main", "A map/reduce program that writes 10GB of random data per node."),
    "secondarysort": ("hbmr.examples.secondarysort:main", "An example defining a secondary sort to the reduce."),
    "sleep": ("hbmr.examples.sleepjob:main", "A job that sleeps at each map and reduce task."),
    "sort": ("hbmr.examples.sort:main", "A map/reduce program that sorts the data written by the random writer."),
    "sudoku": ("hbmr.examples.dancing:main_sudoku", "A sudoku solver."),
    "teragen": ("hbmr.models.terasort:main_teragen", "Generate data for the terasort"),
    "terasort": ("hbmr.models.terasort:main_terasort", "Run the terasort"),
    "teravalidate": ("hbmr.models.terasort:main_teravalidate", "Checking results of terasort"),
    "wordcount": ("hbmr.models.wordcount:main", "A map/reduce program that counts the words in the input files."),
    # hbmr GPU workloads
    "kmeans": ("hbmr.models.kmeans:main", "K-Means (split-level GPU/CPU map tasks, RCCL all-reduce)."),
    "kmeans-pipes": ("hbmr.models.kmeans_pipes:main", "K-Means through the Pipes CPU/GPU task binaries."),
    "matmul": ("hbmr.models.matmul:main", "Mars-style dense matmul map tasks on the MFMA matrix cores."),
}


def usage():
    lines = ["An example program must be given as the first argument.", "Valid program names are:"]
    lines += [f"  {k}: {v[1]}" for k, v in sorted(PROGRAMS.items())]
    return "\n".join(lines)


def run(name, args, cluster=None):
    if name not in PROGRAMS:
        print(f"Unknown program '{name}' chosen.\n{usage()}", file=sys.stderr)
        return -1
    mod, fn = PROGRAMS[name][0].split(":")
    return getattr(importlib.import_module(mod), fn)(list(args), cluster=cluster)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(usage(), file=sys.stderr)
        return -1
    return run(argv[0], argv[1:])


if __name__ == "__main__":
    sys.exit(main())
