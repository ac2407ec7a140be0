"""Per-task profiling (mapred.task.profile).

Reference: JobConf.getProfileEnabled / getProfileTaskRange / getProfileParams
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/JobConf.java:1482-1541): for
attempts whose partition is inside ``mapred.task.profile.maps`` /
``mapred.task.profile.reduces`` (Configuration.IntegerRanges, default "0-2"),
TaskRunner adds an HPROF agent to the child JVM (TaskRunner.java:461-466) and
the client fetches the resulting ``profile.out`` (JobClient.java:1290-1292).

hbmr tasks run in-process, so a selected attempt runs under cProfile; the
sorted text report goes to ``hbmr.task.profile.dir`` (default
``<output>/_logs/profile``) as ``<attempt>.profile`` — a GPU split task's host
side is profiled the same way (device time is in rocprofv3 / the tracer).
``mapred.task.profile.params`` selects the sort key (cumulative by default).
"""
from __future__ import annotations

import cProfile
import io
import os
import pstats


def parse_ranges(spec: str):
    """IntegerRanges: "0-2,5,7-" → predicate."""
    parts = []
    for item in (spec or "").split(","):
        item = item.strip()
        if not item:
            continue
        if "-" in item:
            a, b = item.split("-", 1)
            parts.append((int(a) if a else 0, int(b) if b else 1 << 62))
        else:
            parts.append((int(item), int(item)))
    return lambda n: any(a <= n <= b for a, b in parts)


def profile_selected(conf, is_map: bool, partition: int) -> bool:
    if not conf.get_boolean("mapred.task.profile", False):
        return False
    key = "mapred.task.profile.maps" if is_map else "mapred.task.profile.reduces"
    return parse_ranges(conf.get(key, "0-2"))(partition)


def profile_dir(conf):
    d = conf.get("hbmr.task.profile.dir")
    if d:
        return d
    out = conf.get("mapred.output.dir")
    return os.path.join(out, "_logs", "profile") if out else None


def run_profiled(conf, attempt_id: str, is_map: bool, partition: int, fn, *args, **kw):
    """Run fn(*args) (under cProfile when this attempt is selected)."""
    if not profile_selected(conf, is_map, partition):
        return fn(*args, **kw)
    prof = cProfile.Profile()
    try:
        return prof.runcall(fn, *args, **kw)
    finally:
        d = profile_dir(conf)
        if d:
            os.makedirs(d, exist_ok=True)
            buf = io.StringIO()
            sort = (conf.get("mapred.task.profile.params") or "cumulative").split()[0]
            if sort not in pstats.Stats.sort_arg_dict_default:
                sort = "cumulative"
            pstats.Stats(prof, stream=buf).sort_stats(sort).print_stats(40)
            with open(os.path.join(d, f"{attempt_id}.profile"), "w") as f:
                f.write(buf.getvalue())
