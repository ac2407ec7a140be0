"""Rumen: job traces from job history, runtime CDFs, and a trace-driven job
model for replay.

Follows hadoop-1.0.3/src/tools/org/apache/hadoop/tools/rumen/:

* ``TraceBuilder`` (TraceBuilder.java, JobBuilder.java) — job history →
  a trace of ``LoggedJob`` records (LoggedJob/LoggedTask/LoggedTaskAttempt
  field names kept: jobID, user, jobName, submitTime, launchTime, finishTime,
  outcome, totalMaps, totalReduces, mapTasks, reduceTasks, attempts, ...) and a
  ``LoggedNetworkTopology`` of racks → hosts (TopologyBuilder.java).
* ``LoggedDiscreteCDF`` (LoggedDiscreteCDF.java) — min, max and the
  5 %..95 % rankings of successful attempt runtimes
  (``successfulMapAttemptCDFs``, ``successfulReduceAttemptCDF``,
  ``failedMapAttemptCDFs``).
* ``JobTraceReader`` / ``ZombieJob`` (ZombieJob.java) — a ``JobStory`` over a
  trace: per-task runtimes (the recorded one, or one drawn from the job's
  CDF for tasks beyond the record), used by Gridmix replay.

hbmr additions: attempts carry the CPU/GPU placement and device the fork's
JobHistory never logged, and the trace keeps separate CPU and
GPU map CDFs so replay can reproduce hybrid scheduling decisions.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import random

from ..webui.history import load_history

RANKINGS = [i / 100 for i in range(5, 100, 5)]


def discrete_cdf(values) -> dict:
    """LoggedDiscreteCDF: min/max + value at each 5 % ranking."""
    xs = sorted(int(v) for v in values)
    if not xs:
        return {"minimum": None, "maximum": None, "rankings": [], "numberValues": 0}
    n = len(xs)
    ranks = [{"relativeRanking": r, "datum": xs[min(n - 1, int(r * n))]} for r in RANKINGS]
    return {"minimum": xs[0], "maximum": xs[-1], "rankings": ranks, "numberValues": n}


def sample_cdf(cdf: dict, rng: random.Random) -> int:
    """Piecewise-linear inverse-CDF draw (CDFPiecewiseLinearRandomGenerator)."""
    if not cdf or not cdf.get("numberValues"):
        return 0
    pts = [(0.0, cdf["minimum"])] + [(r["relativeRanking"], r["datum"]) for r in cdf["rankings"]] \
        + [(1.0, cdf["maximum"])]
    u = rng.random()
    for (r0, d0), (r1, d1) in zip(pts, pts[1:]):
        if u <= r1:
            t = 0.0 if r1 == r0 else (u - r0) / (r1 - r0)
            return int(d0 + t * (d1 - d0))
    return int(cdf["maximum"])


def _ms(t):
    return None if t in (None, 0) else int(float(t) * 1000)


def _host_rack(tracker: str):
    host = (tracker or "").replace("tracker_", "").split(":")[0] or "localhost"
    return host, "/default-rack"


def build_job(job: dict, attempts: list) -> dict:
    """One LoggedJob from a history file's JOB record and its attempts."""
    tasks = {}
    for a in attempts:
        t = tasks.setdefault(a["task"], {"taskID": a["task"], "taskType": a["type"],
                                         "startTime": None, "finishTime": None,
                                         "taskStatus": "FAILED", "attempts": []})
        start, finish = _ms(a.get("start")), _ms(a.get("finish"))
        host, rack = _host_rack(a.get("tracker"))
        t["attempts"].append({
            "attemptID": a["attempt"], "result": a.get("state"), "startTime": start,
            "finishTime": finish, "hostName": f"{rack}/{host}",
            "runOnGPU": bool(a.get("gpu")), "device": a.get("device"),
            "speculative": bool(a.get("speculative")),
            "deviceTimeMs": None if a.get("device_time") is None else
            float(a["device_time"]) * 1000})
        if start is not None:
            t["startTime"] = start if t["startTime"] is None else min(t["startTime"], start)
        if a.get("successful"):
            t["taskStatus"] = "SUCCESS"
            t["finishTime"] = finish
    maps = [t for t in tasks.values() if t["taskType"] == "MAP"]
    reduces = [t for t in tasks.values() if t["taskType"] == "REDUCE"]

    def runtimes(ts, ok, gpu=None):
        out = []
        for t in ts:
            for a in t["attempts"]:
                if ((a["result"] == "SUCCEEDED") == ok and a["startTime"] is not None
                        and a["finishTime"] is not None
                        and (gpu is None or a["runOnGPU"] == gpu)):
                    out.append(a["finishTime"] - a["startTime"])
        return out

    return {
        "jobID": job["job"], "user": job.get("user"), "jobName": job.get("name"),
        "submitTime": _ms(job.get("submit")), "launchTime": _ms(job.get("launch")),
        "finishTime": _ms(job.get("finish")),
        "outcome": "SUCCESS" if job.get("state") in ("SUCCEEDED", 2) else str(job.get("state")),
        "totalMaps": job.get("maps"), "totalReduces": job.get("reduces"),
        "finishedCpuMaps": job.get("cpu_maps"), "finishedGpuMaps": job.get("gpu_maps"),
        "mapTasks": sorted(maps, key=lambda t: t["taskID"]),
        "reduceTasks": sorted(reduces, key=lambda t: t["taskID"]),
        # one CDF per locality level in the reference; hbmr keys by placement
        "successfulMapAttemptCDFs": [discrete_cdf(runtimes(maps, True))],
        "successfulCpuMapAttemptCDF": discrete_cdf(runtimes(maps, True, gpu=False)),
        "successfulGpuMapAttemptCDF": discrete_cdf(runtimes(maps, True, gpu=True)),
        "failedMapAttemptCDFs": [discrete_cdf(runtimes(maps, False))],
        "successfulReduceAttemptCDF": discrete_cdf(runtimes(reduces, True)),
        "failedReduceAttemptCDF": discrete_cdf(runtimes(reduces, False)),
        "counters": job.get("counters", {}),
    }


def build_topology(jobs) -> dict:
    racks = {}
    for j in jobs:
        for t in j["mapTasks"] + j["reduceTasks"]:
            for a in t["attempts"]:
                rack, _, host = a["hostName"].rpartition("/")
                racks.setdefault(rack or "/default-rack", set()).add(host)
    return {"name": "<root>", "children": [
        {"name": r, "children": [{"name": h, "children": []} for h in sorted(hs)]}
        for r, hs in sorted(racks.items())]}


def trace_builder(history_paths, trace_out, topology_out=None) -> list:
    """TraceBuilder: history files / dirs → trace (JSON lines, submit order)."""
    files = []
    for p in history_paths:
        files += sorted(glob.glob(os.path.join(p, "*.jsonl"))) if os.path.isdir(p) else [p]
    jobs = []
    for f in files:
        job, attempts = load_history(f)
        if job is not None:
            jobs.append(build_job(job, attempts))
    jobs.sort(key=lambda j: (j["submitTime"] or 0, j["jobID"]))
    with open(trace_out, "w") as f:
        for j in jobs:
            f.write(json.dumps(j) + "\n")
    if topology_out:
        with open(topology_out, "w") as f:
            json.dump(build_topology(jobs), f, indent=1)
    return jobs


class JobTraceReader:
    """Iterates LoggedJobs from a trace file (JobTraceReader.java)."""

    def __init__(self, path):
        self.path = path

    def __iter__(self):
        with open(self.path) as f:
            for line in f:
                if line.strip():
                    yield json.loads(line)


class ZombieJob:
    """JobStory over one LoggedJob (ZombieJob.java): task counts, submit time
    and per-attempt runtimes, recorded where available, otherwise drawn from
    the job's runtime CDF with a per-job seed (so replays are reproducible)."""

    def __init__(self, logged: dict, seed: int = 0):
        self.job = logged
        self.rng = random.Random(hash((logged["jobID"], seed)) & 0xFFFFFFFF)

    def getName(self):  # noqa: N802
        return self.job.get("jobName")

    def getSubmissionTime(self):  # noqa: N802
        return self.job.get("submitTime") or 0

    def getNumberMaps(self):  # noqa: N802
        return self.job.get("totalMaps") or len(self.job["mapTasks"])

    def getNumberReduces(self):  # noqa: N802
        return self.job.get("totalReduces") or len(self.job["reduceTasks"])

    def _recorded(self, tasks, i):
        if i < len(tasks):
            for a in tasks[i]["attempts"]:
                if a["result"] == "SUCCEEDED" and a["startTime"] is not None \
                        and a["finishTime"] is not None:
                    return a["finishTime"] - a["startTime"], a["runOnGPU"]
        return None

    def getTaskAttemptInfo(self, task_type: str, i: int) -> dict:  # noqa: N802
        """{'runtime_ms', 'gpu'} of the i-th map or reduce task."""
        if task_type.upper() == "MAP":
            rec = self._recorded(self.job["mapTasks"], i)
            if rec:
                return {"runtime_ms": rec[0], "gpu": rec[1]}
            return {"runtime_ms": sample_cdf(self.job["successfulMapAttemptCDFs"][0], self.rng),
                    "gpu": False}
        rec = self._recorded(self.job["reduceTasks"], i)
        if rec:
            return {"runtime_ms": rec[0], "gpu": False}
        return {"runtime_ms": sample_cdf(self.job["successfulReduceAttemptCDF"], self.rng),
                "gpu": False}


class ZombieJobProducer:
    def __init__(self, trace_path, seed=0):
        self.reader = iter(JobTraceReader(trace_path))
        self.seed = seed

    def getNextJob(self):  # noqa: N802
        j = next(self.reader, None)
        return None if j is None else ZombieJob(j, self.seed)


def main(argv=None, cluster=None):
    ap = argparse.ArgumentParser(prog="hbmr rumen",
                                 description="TraceBuilder <trace-out> <topology-out> <history>...")
    ap.add_argument("trace")
    ap.add_argument("topology")
    ap.add_argument("history", nargs="+")
    a = ap.parse_args(argv)
    jobs = trace_builder(a.history, a.trace, a.topology)
    print(f"wrote {len(jobs)} jobs to {a.trace}")
    return 0
