"""Job history files, their summary, and rule-based diagnosis.

* :func:`write_job_history` — at job completion the JobTracker writes
  ``<history dir>/<jobid>.jsonl``: a JOB line, then one line per task attempt
  with its placement (CPU/GPU + device — which the fork's JobHistory never
  recorded), times, device time and counters
  (hadoop-1.0.3 JobHistory.java:94, 1485; keys ``hadoop.job.history.location``
  / ``hbmr.history.dir``).
* :func:`summarize_history` — the Rumen-style digest of one file: makespan,
  phase times, CPU vs GPU map counts and mean times, per-tracker load.
* :func:`diagnose` — Vaidya-style rules over the digest (contrib/vaidya):
  CPU stragglers extending the makespan, idle GPU capacity, map-time skew,
  failed attempts, slow reduce tail.
"""
from __future__ import annotations

import json
import os
import statistics


def history_dir(conf):
    return conf.get("hbmr.history.dir") or conf.get("hadoop.job.history.location")


def job_record(jip) -> dict:
    st = jip.status
    return {"type": "JOB", "job": str(jip.job_id), "name": jip.conf.get_job_name(),
            "user": jip.conf.get_user(), "state": st.state, "submit": jip.submit_time,
            "launch": jip.launch_time, "finish": st.finish_time,
            "maps": len(jip.maps), "reduces": len(jip.reduces),
            "cpu_maps": jip.finished_cpu_maps, "gpu_maps": jip.finished_gpu_maps,
            "failure": st.failure_info, "timeline": jip.timeline(),
            "counters": jip.counters.to_dict()}


def attempt_records(jip):
    for tip in list(jip.maps) + list(jip.reduces):
        for a in list(tip.attempts.values()):
            yield {"type": "MAP" if tip.is_map else "REDUCE", "task": str(tip.tid),
                   "attempt": a.aid, "state": a.state, "tracker": a.tracker,
                   "gpu": bool(a.run_on_gpu), "device": a.device, "start": a.start,
                   "finish": a.finish, "device_time": a.device_time,
                   "speculative": bool(a.speculative), "successful": tip.successful is a,
                   "diagnostic": (a.diagnostic or "")[:500],
                   "counters": a.counters if isinstance(a.counters, dict) else {}}


def write_job_history(jip, directory) -> str:
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f"{jip.job_id}.jsonl")
    with open(path, "w") as f:
        f.write(json.dumps(job_record(jip), default=str) + "\n")
        for rec in attempt_records(jip):
            f.write(json.dumps(rec, default=str) + "\n")
    return path


def load_history(path):
    job, attempts = None, []
    with open(path) as f:
        for line in f:
            rec = json.loads(line)
            if rec.get("type") == "JOB":
                job = rec
            else:
                attempts.append(rec)
    return job, attempts


def _stats(xs):
    if not xs:
        return None
    return {"n": len(xs), "mean": statistics.fmean(xs), "min": min(xs), "max": max(xs),
            "p50": statistics.median(xs)}


def summarize_history(path_or_records) -> dict:
    if isinstance(path_or_records, str):
        job, attempts = load_history(path_or_records)
    else:
        job, attempts = path_or_records
    ok = [a for a in attempts if a["successful"]]
    maps = [a for a in ok if a["type"] == "MAP"]

    def dur(a):
        return (a["finish"] or a["start"]) - a["start"]
    cpu = [dur(a) for a in maps if not a["gpu"]]
    gpu = [a["device_time"] or dur(a) for a in maps if a["gpu"]]
    reds = [dur(a) for a in ok if a["type"] == "REDUCE"]
    per_tracker: dict = {}
    for a in ok:
        t = per_tracker.setdefault(a["tracker"], {"maps_cpu": 0, "maps_gpu": 0, "reduces": 0})
        if a["type"] == "REDUCE":
            t["reduces"] += 1
        else:
            t["maps_gpu" if a["gpu"] else "maps_cpu"] += 1
    failed = [a for a in attempts if a["state"] in ("FAILED", "FAILED_UNCLEAN")]
    killed = [a for a in attempts if a["state"] == "KILLED"]
    last_map = max((a["finish"] for a in maps), default=None)
    return {"job": job["job"] if job else None, "name": job and job["name"],
            "state": job and job["state"],
            "makespan": (job["finish"] - job["submit"]) if job and job["finish"] else None,
            "timeline": job and job.get("timeline"),
            "maps": len(maps), "cpu_map_time": _stats(cpu), "gpu_map_time": _stats(gpu),
            "reduce_time": _stats(reds), "failed_attempts": len(failed),
            "killed_attempts": len(killed),
            "speculative_attempts": sum(1 for a in attempts if a["speculative"]),
            "last_map_finish": last_map, "per_tracker": per_tracker,
            "diagnosis": diagnose(job, attempts)}


def diagnose(job, attempts) -> list:
    """Rule-based findings, most important first."""
    out = []
    ok = [a for a in attempts if a["successful"] and a["type"] == "MAP"]
    if not ok:
        return out
    cpu = [a for a in ok if not a["gpu"]]
    gpu = [a for a in ok if a["gpu"]]
    end = max(a["finish"] for a in ok)
    if cpu and gpu:
        t_cpu = statistics.fmean(a["finish"] - a["start"] for a in cpu)
        t_gpu = statistics.fmean((a["device_time"] or (a["finish"] - a["start"])) for a in gpu)
        accel = t_cpu / max(t_gpu, 1e-9)
        gpu_end = max(a["finish"] for a in gpu)
        if max(a["finish"] for a in cpu) > gpu_end and accel > 1.5:
            tail = max(a["finish"] for a in cpu) - gpu_end
            out.append({"rule": "cpu-straggler", "severity": "high",
                        "text": f"CPU map tasks ran {accel:.1f}x slower than GPU tasks and "
                                f"finished {tail:.3f}s after the last GPU task; with the "
                                f"hybrid policy the min-makespan split would leave them on GPU"})
        out.append({"rule": "acceleration", "severity": "info",
                    "text": f"GPU acceleration factor {accel:.1f}x "
                            f"({len(gpu)} GPU / {len(cpu)} CPU map tasks)"})
    durs = [a["finish"] - a["start"] for a in ok]
    if len(durs) >= 8:
        med = statistics.median(durs)
        slow = [d for d in durs if d > 3 * med and d - med > 0.05]
        if slow:
            out.append({"rule": "map-skew", "severity": "medium",
                        "text": f"{len(slow)} map tasks took >3x the median "
                                f"({med:.3f}s): check input split sizes"})
    fails = [a for a in attempts if a["state"] in ("FAILED", "FAILED_UNCLEAN")]
    if fails:
        out.append({"rule": "failures", "severity": "high",
                    "text": f"{len(fails)} failed attempts, e.g. {fails[0]['diagnostic'][:160]}"})
    out += vaidya_rules(job, attempts)
    reds = [a for a in attempts if a["successful"] and a["type"] == "REDUCE"]
    if job and job.get("finish") and reds:
        tail = job["finish"] - end
        span = job["finish"] - job["submit"]
        if span > 0 and tail / span > 0.5:
            out.append({"rule": "reduce-tail", "severity": "medium",
                        "text": f"reduce phase is {100 * tail / span:.0f}% of the makespan"})
    return out


# ---------------------------------------------------------------------------- Vaidya
_TASK = "org.apache.hadoop.mapred.Task$Counter"
_JIP = "org.apache.hadoop.mapred.JobInProgress$Counter"
_FS = "FileSystemCounters"


def _ctr(counters, group, name):
    return int(((counters or {}).get(group) or {}).get(name, 0) or 0)


def _severity(impact, threshold):
    return "high" if impact >= max(threshold, 0.5) else ("medium" if impact >= threshold
                                                         else "info")


def vaidya_rules(job, attempts, thresholds=None) -> list:
    """The reference's post-execution diagnosis tests (contrib/vaidya/.../
    postexdiagnosis/tests/*.java), same inputs and impact formulas:

    * MapSideDiskSpill: (local bytes written by maps − map output bytes) /
      map output bytes, normalised by 3.0 (a map-only job: all of it);
    * BalancedReducePartitioning: 1 − (reducers holding 90 % of the reduce
      input records) / reducers;
    * MapsReExecutionImpact / ReducesReExecutionImpact: (launched − total) /
      total tasks;
    * ReadingHDFSFilesAsSideEffect: HDFS bytes read / map input bytes,
      normalised by 2.0.

    Each finding carries the rule name, its impact in [0, 1] and the
    reference's prescription; impacts over the threshold (0.2 by default,
    ``thresholds[rule]``) are medium/high."""
    th = {"MapSideDiskSpill": 0.3, "BalancedReducePartitioning": 0.4,
          "MapsReExecutionImpact": 0.4, "ReducesReExecutionImpact": 0.4,
          "ReadingHDFSFilesAsSideEffect": 0.3}
    th.update(thresholds or {})
    if not job:
        return []
    jc = job.get("counters") or {}
    out = []
    maps = [a for a in attempts if a["type"] == "MAP"]
    reds_ok = [a for a in attempts if a["type"] == "REDUCE" and a["successful"]]
    total_maps = job.get("maps", 0)
    total_reds = job.get("reduces", 0)

    def add(rule, impact, text, prescription):
        out.append({"rule": rule, "impact": round(float(impact), 4),
                    "severity": _severity(impact, th[rule]), "text": text,
                    "prescription": prescription})

    # MapSideDiskSpill
    written = sum(_ctr(a.get("counters"), _FS, "FILE_BYTES_WRITTEN") for a in maps
                  if a["successful"])
    mob = _ctr(jc, _TASK, "MAP_OUTPUT_BYTES")
    if mob > 0:
        imp = (written - mob) / mob if total_reds > 0 else written / mob
        imp = 1.0 if imp > 3.0 else max(0.0, imp) / 3.0
        add("MapSideDiskSpill", imp,
            f"maps wrote {written} local bytes for {mob} map-output bytes",
            "Use a combiner or compress map output; raise io.sort.mb / "
            "io.sort.record.percent so maps spill once")
    # BalancedReducePartitioning
    if total_reds > 0 and reds_ok:
        recs = sorted((_ctr(a.get("counters"), _TASK, "REDUCE_INPUT_RECORDS") for a in reds_ok),
                      reverse=True)
        tot = sum(recs)
        if tot > 0:
            want = 0.90 * tot
            acc, busy = 0, 0
            for r in recs:
                acc += r
                busy += 1
                if acc >= want:
                    break
            imp = 1 - busy / total_reds
            add("BalancedReducePartitioning", imp,
                f"{busy} of {total_reds} reducers process 90% of the reduce input records",
                "Use a better partitioner (or sample keys, TotalOrderPartitioner) so "
                "reduce input is spread evenly")
    # Maps / Reduces re-execution
    launched_m = _ctr(jc, _JIP, "TOTAL_LAUNCHED_MAPS")
    if total_maps > 0 and launched_m:
        imp = max(0.0, (launched_m - total_maps) / total_maps)
        add("MapsReExecutionImpact", min(1.0, imp),
            f"{launched_m} map attempts launched for {total_maps} maps",
            "Find why maps are re-executed: unstable nodes or application failures")
    launched_r = _ctr(jc, _JIP, "TOTAL_LAUNCHED_REDUCES")
    if total_reds > 0 and launched_r:
        imp = max(0.0, (launched_r - total_reds) / total_reds)
        add("ReducesReExecutionImpact", min(1.0, imp),
            f"{launched_r} reduce attempts launched for {total_reds} reduces",
            "Find why reduces are re-executed: unstable nodes or application failures")
    # ReadingHDFSFilesAsSideEffect
    hdfs_read = _ctr(jc, _FS, "HDFS_BYTES_READ")
    mib = _ctr(jc, _TASK, "MAP_INPUT_BYTES")
    if hdfs_read:
        if mib == 0:
            imp = 1.0
        else:
            imp = hdfs_read / mib
            imp = 1.0 if imp >= 2.0 else imp / 2.0
        add("ReadingHDFSFilesAsSideEffect", imp,
            f"tasks read {hdfs_read} HDFS bytes for {mib} map-input bytes",
            "Tasks read HDFS data beyond their input splits (side files): ship it with the "
            "DistributedCache instead")
    return out
