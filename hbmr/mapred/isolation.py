"""IsolationRunner: re-run one map attempt alone, in this process, from the
files its tracker kept (hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/
IsolationRunner.java:158-235) — for debugging a failing task under pdb or a
profiler without a cluster.

A job sets ``keep.failed.task.files=true`` (or ``keep.task.files.pattern``
to a regex over attempt ids); the tracker then keeps ``job.xml`` (the task's
conf: ``mapred.task.id``, ``.partition``, ``.is.map``) and ``split.dta`` (the
serialised input split) under ``<mapred.local.dir>/<job>/<attempt>/``.
``python -m hbmr.mapred.isolation <dir>/job.xml [user]`` re-runs that map with
a local reporter (the reference's FakeUmbilical) in a fresh work dir.  As in
the reference only map tasks are supported; outputs go to the work dir's
map output file (or, for map-only jobs, the job's output committer)."""
from __future__ import annotations

import json
import os
import sys

from .ids import TaskAttemptID
from .jobconf import JobConf
from .task import MapTask


class IsolationRunner:
    def run(self, args) -> bool:
        if len(args) < 1:
            print("Usage: IsolationRunner <path>/job.xml <optional-user-name>")
            return False
        job_file = args[0]
        if not os.path.isfile(job_file):
            print(f"{job_file} is not a valid job file.")
            return False
        conf = JobConf()
        conf.add_resource(os.path.abspath(job_file))
        if len(args) > 1:
            conf.set_user(args[1])
        tid = conf.get("mapred.task.id")
        if not tid:
            print("mapred.task.id not found in configuration; job.xml is not a task config")
            return False
        if not conf.get_boolean("mapred.task.is.map", True):
            print("Only map tasks are supported.")
            return False
        aid = TaskAttemptID.for_name(tid)
        part = conf.get_int("mapred.task.partition", 0)
        task_dir = os.path.dirname(os.path.abspath(job_file))
        with open(os.path.join(task_dir, "split.dta")) as f:
            from .tasktracker import _split_from_dict
            split = _split_from_dict(json.load(f))
        work = os.path.join(task_dir, "isolation")
        os.makedirs(work, exist_ok=True)
        task = MapTask(conf, aid, part, split)
        self.task = task
        self.output = task.run(work)
        print(f"Task {tid} reporting done.")
        return True


def main(argv=None) -> int:
    return 0 if IsolationRunner().run(list(sys.argv[1:] if argv is None else argv)) else 1


if __name__ == "__main__":
    sys.exit(main())
