"""hbmr headline benchmark: K-Means job makespan + map-tasks/s on 1..8 MI355X.

Metric/config from BASELINE.json: "K-Means job makespan + map-tasks/sec (whole
node)", config 3 = K-Means 100M points × 128-d, k=1024, hybrid CPU+GPU
scheduling.  One *step* is one complete K-Means iteration **job** through the
framework: JobTracker scheduling (hybrid cost model, CPU slots enabled), map
tasks on the TaskTrackers' GPU slots (MFMA assign + fixed-point combiner on
HBM-resident splits), the collective reduce (exact int64 all-reduce over
RCCL/xGMI) and the centroid update.  The total problem (100M points) is fixed
as N grows (strong scaling); splits are 781,250 points → 128 map tasks per job.
Precision (default, ``--exact``): the points stay fp32 and every label is the
exact arg-min over the fp32 data — f16 MFMA top candidates, certified against
an error bound, the uncertain points re-scored in fp64 — and the centroid sums
are exact int64 fixed point of the fp32 rows (dtype "fp32"); ``--no-exact``
runs the bf16-input variant.  Data: synthetic Gaussian mixture generated in HBM by the
framework's own split loader; centroids initialised from the first k points.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1, one rank per GPU)

With ``--gpus N > 1`` and no torchrun environment, bench.py launches the N rank
processes itself (same env contract as torchrun: RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT) before anything touches the
GPU, forwards rank 0's JSON line and exits non-zero if any rank fails.

``--simulate-ms T`` rehearses the same job on CPU: GPU slots are simulated
(``hbmr.gpu.simulate``, T ms of device time per split, no split data) and the
collectives run over gloo, so the control plane + reduce can be timed at
world 1/2/4/8 without GPUs (profiles/scale_sim_cpu.json).

Timing: W untimed iterations (the first one materialises the splits in HBM and
profiles the CPU slot), then a barrier job (every tracker: RCCL barrier + device
synchronize), K timed iteration jobs, another barrier job.  Rank 0 hosts the
JobTracker and client and observes the completion of every job, which
requires every rank's reduce to have finished, so its wall time is the max over
ranks.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--points", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--split-points", type=int, default=781_250)
    ap.add_argument("--policy", default="hybrid", choices=["hybrid", "optional", "stock"])
    ap.add_argument("--cpu-slots", type=int, default=2)
    ap.add_argument("--gpu-slots", type=int, default=2, help="HIP streams (GPU map slots) per GPU")
    ap.add_argument("--queue-depth", type=int, default=64)
    ap.add_argument("--simulate-ms", type=float, default=None,
                    help="CPU rehearsal: simulated GPU slots with this device time per split")
    ap.add_argument("--in-process", action="store_true",
                    help="run the GPU slots inside the tracker process (no worker process)")
    ap.add_argument("--prefetch", type=int, default=3, metavar="N",
                    help="keep N iteration jobs submitted ahead, each held by the JobTracker "
                         "until its predecessor succeeds (hbmr.job.depends.on), as a "
                         "JobControl driver would; 0 submits each after the previous finished. "
                         "3: a new job is staged behind a staged one, so its plan rides on "
                         "the trackers' reports (no long-poll ring per tracker per job: "
                         "profiles/r05_control_plane_rehearsal.json)")
    ap.add_argument("--prestage", action=argparse.BooleanOptionalAction, default=True,
                    help="let the JobTracker stage held iteration jobs: their GPU maps wait "
                         "on the device behind the predecessor's reduce (hbmr.job.prestage)")
    ap.add_argument("--exact", action=argparse.BooleanOptionalAction, default=True,
                    help="fp32-faithful assignment (default; hbmr.kmeans.exact: the points stay "
                         "fp32, f16 MFMA candidates certified against the fp32 data, fp64 "
                         "re-score of the uncertain points, fp32 rows summed in exact fixed "
                         "point): dtype fp32.  --no-exact: the bf16-input variant (points "
                         "stored and summed in bf16)")
    ap.add_argument("--input", default=None, metavar="DIR",
                    help="SequenceFile input (tools/write_kmeans_input.py writes the synthetic "
                         "set as files) instead of points generated in HBM")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("-D", dest="defines", action="append", default=[], metavar="KEY=VALUE",
                    help="extra configuration (e.g. -D hbmr.gpu.first.chunk=8)")
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO if a.verbose else logging.WARNING,
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(a.gpus)

    from hbmr.utils.sampler import dump_profiles, maybe_arm_stackdump, maybe_profile_threads, \
        maybe_start
    cprof = maybe_profile_threads()   # HBMR_CPROFILE=path: cProfile of every thread
    maybe_arm_stackdump()       # HBMR_STACKDUMP_S=s: thread stacks to stderr every s
    sampler = maybe_start()     # HBMR_SAMPLE_PROF=prefix: control-plane stack sampling

    import torch
    if a.simulate_ms is not None and world > 1:
        # N rank processes share this host's cores: no intra-op thread pools
        # spinning against each other (on a GPU node the ranks do no torch CPU work)
        torch.set_num_threads(1)

    from hbmr.gpu.syncjob import sync_conf
    from hbmr.mapred.jobconf import JobConf
    from hbmr.mapred.node import Node
    from hbmr.models import kmeans as K

    conf = JobConf()
    conf.set("hbmr.scheduler.policy", a.policy)
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", a.cpu_slots)
    conf.set_int("mapred.tasktracker.map.gpu.tasks.maximum", a.gpu_slots)
    conf.set_int("hbmr.gpu.queue.depth", a.queue_depth)
    conf.set_int("hbmr.heartbeat.interval.ms", 200)
    conf.set_int("mapred.task.timeout", 0)
    # splits are placed on their designated tracker and stay HBM-resident there;
    # only a tracker that is seconds late (not one still warming up) loses its
    # splits to another GPU's queue, which would skew every later iteration
    conf.set_int("hbmr.locality.wait.ms", 5000)
    conf.set_boolean("hbmr.job.prestage", a.prestage)
    conf.set_int("hbmr.job.prestage.depth", max(1, a.prefetch))
    # device_count() does not initialise HIP in this process: with the default
    # per-rank GPU worker process (hbmr.gpu.worker.process) the device work and
    # its synchronisation happen in the workers (the barrier job synchronises
    # every worker's device), and this process never holds a HIP context
    has_gpu = torch.cuda.device_count() > 0 and a.simulate_ms is None
    in_process = a.in_process and has_gpu
    # (a simulated run may also keep its simulated slots in the tracker process)
    conf.set_boolean("hbmr.gpu.worker.process", not (in_process or a.in_process))
    if a.simulate_ms is not None:
        if world > 1:
            conf.set_int("hbmr.worker.torch.threads", 1)
        conf.set("hbmr.gpu.simulate", "true")
        conf.set("hbmr.gpu.simulate.nodata", "true")
        conf.set("hbmr.gpu.simulate.task.ms", str(a.simulate_ms))
    if a.exact:
        conf.set_boolean("hbmr.kmeans.exact", True)
    for kv in a.defines:
        k, _, v = kv.partition("=")
        conf.set(k.strip(), v.strip())
    node = Node(conf, use_gpu=has_gpu)
    if node.is_master and not getattr(node, "jt_process", False):
        from hbmr.utils.sampler import maybe_watch_jobtracker
        maybe_watch_jobtracker(node.jt)
    if not node.is_master:
        node.serve_until_shutdown()
        node.shutdown()
        return 0

    inp = a.input or f"synthetic:{a.points}:7"
    if a.input:
        # one split per input file (the writer's files hold --split-points each)
        conf.set_int("mapred.map.tasks", -(-a.points // a.split_points))
    drv = K.KMeansDriver(node.submit_job, node.job_result, conf=conf, k=a.k, d=a.dims, inp=inp,
                         split_points=a.split_points)

    def barrier():
        rj = node.submit_job(sync_conf(conf))
        rj.waitForCompletion()
        if not rj.isSuccessful():
            raise RuntimeError(f"sync job failed: {rj.getFailureInfo()}")

    try:
        t_setup = time.time()
        pre = max(0, a.prefetch)
        for w in range(a.warmup):
            # (no job submitted ahead crosses into the timed window)
            drv.step(prefetch=min(pre, a.warmup - 1 - w))
            # progress on stderr: a cold first iteration (file input) can take a while
            J = "org.apache.hadoop.mapred.JobInProgress$Counter"
            c = drv.history[-1]["counters"] if drv.history else None
            print(f"bench: warmup {w + 1}/{a.warmup} done at {time.time() - t_setup:.2f} s" +
                  (f" (last job: cpu maps {c.get(J, 'CPU_MAP_TASKS')}, gpu maps "
                   f"{c.get(J, 'GPU_MAP_TASKS')})" if c is not None else ""),
                  file=sys.stderr, flush=True)
        t_warm = time.time() - t_setup
        barrier()
        if in_process:
            torch.cuda.synchronize()
        cpu0 = time.process_time()
        jt_proc = getattr(node, "jt_process", False)
        jt_cpu0 = node.jt.cpu_seconds() if jt_proc else 0.0
        jt_thr0 = node.jt.thread_cpu() if jt_proc else {}
        if sampler is not None:
            sampler.mark()
        t0 = time.perf_counter()
        # every timed job is submitted inside the timed window (the first by this
        # loop, each next one while its predecessor runs); none crosses a barrier
        for s in range(a.steps):
            drv.step(prefetch=min(pre, a.steps - 1 - s))
        barrier()
        if in_process:
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        cpu_rank0 = time.process_time() - cpu0
        jt_cpu = node.jt.cpu_seconds() - jt_cpu0 if jt_proc else None
        jt_thr = {k: round((v - jt_thr0.get(k, 0.0)) / a.steps * 1e3, 3)
                  for k, v in node.jt.thread_cpu().items()} if jt_proc else None
        hist = drv.history[a.warmup:]
        if a.verbose:
            J = "org.apache.hadoop.mapred.JobInProgress$Counter"
            for i, h in enumerate(drv.history):
                c = h["counters"]
                print(f"job {i}: maps/tracker {sorted((h.get('maps_per_tracker') or {}).values())}"
                      f" hbm-local {c.get(J, 'HBM_LOCAL_MAPS')} data-local "
                      f"{c.get(J, 'DATA_LOCAL_MAPS')} cpu {c.get(J, 'CPU_MAP_TASKS')}",
                      file=sys.stderr, flush=True)
        n_maps = sum(h["counters"].get("org.apache.hadoop.mapred.JobInProgress$Counter",
                                       "TOTAL_LAUNCHED_MAPS") for h in hist)
        gpu_maps = sum(h["counters"].get("org.apache.hadoop.mapred.JobInProgress$Counter",
                                         "GPU_MAP_TASKS") for h in hist)
        cpu_maps = sum(h["counters"].get("org.apache.hadoop.mapred.JobInProgress$Counter",
                                         "CPU_MAP_TASKS") for h in hist)
        ms = dt / a.steps * 1e3
        tls = [h.get("timeline") for h in hist if h.get("timeline")]

        def _avg(key):
            v = [t[key] for t in tls if t.get(key) is not None]
            return round(1e3 * sum(v) / len(v), 3) if v else None
        # phases from the job's release (its predecessor's finish, when the
        # JobTracker lets a dependent job complete; its submission otherwise).
        # Pre-staged maps and early collective reduces are launched BEFORE the
        # release: reported as how far ahead they went, never as a negative time
        lead = lambda v: None if v is None else round(max(0.0, -v), 3)  # noqa: E731
        phases_ms = {"release_to_maps_done": _avg("maps_done"),
                     "release_to_finish": _avg("finish"),
                     "maps_launched_ahead_of_release": lead(_avg("first_map")),
                     "reduce_launched_ahead_of_release": lead(_avg("first_reduce"))}
        gk = [h["counters"].get("hbmr.GpuCounters", "GPU_KERNEL_US") for h in hist]
        # device time of the map kernels per job, de-overlapped across the
        # slot streams (hbmr.gpu.runtime._busy_ms), summed over the GPUs
        map_device_ms = round(sum(gk) / len(gk) / 1e3, 3) if gk else None
        splits = -(-a.points // a.split_points)
        value = splits * a.steps / dt
        cm = node.jt.cost_model.snapshot()
        out = {
            "metric": "K-Means job makespan + map-tasks/sec (whole node) at 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "map-tasks/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32" if conf.get_boolean("hbmr.kmeans.exact", False) else "bf16",
            "precision": ("exact: labels = the fp64 arg-min over the fp32 points and centroids "
                          "(f16 MFMA top candidates, certified by an error bound, uncertain "
                          "points re-scored in fp64); centroid sums of the fp32 rows in int64 "
                          "fixed point") if conf.get_boolean("hbmr.kmeans.exact", False) else
                         "bf16 points (storage and sums), bf16 MFMA assign",
            "data": (f"sequencefile input {a.input} (the synthetic set written to disk)"
                     if a.input else "synthetic") if a.simulate_ms is None else
                    f"simulated GPU slots ({a.simulate_ms} ms/split), CPU only",
            "config": {"model": "K-Means 100M pts x 128-d, k=1024 (hybrid CPU+GPU scheduling)"
                       if (a.points, a.dims, a.k) == (100_000_000, 128, 1024) else
                       f"K-Means {a.points} pts x {a.dims}-d, k={a.k}",
                       "global_batch": a.points, "seq_len": a.dims,
                       "parallelism": f"dp{world}", "k": a.k, "split_points": a.split_points,
                       "map_tasks_per_job": splits, "policy": a.policy,
                       "cpu_slots_per_tracker": a.cpu_slots, "gpu_slots_per_gpu": a.gpu_slots,
                       "gpu_worker_process": not (in_process or a.in_process),
                       "iteration_jobs_ahead": a.prefetch, "prestage": a.prestage,
                       "combiner": conf.get("hbmr.kmeans.combiner") or "delta"},
            "job_makespan_ms": round(ms, 3),
            "phases_ms": phases_ms,
            # each timed job's finish after its predecessor's (the first: after
            # its submission, which follows the opening barrier job)
            "release_to_finish_ms_per_job": [round(1e3 * t["finish"], 2) for t in tls
                                             if t.get("finish") is not None],
            "map_device_ms_per_job": map_device_ms,
            "points_per_sec": round(a.points * a.steps / dt, 1),
            "maps_launched": n_maps, "gpu_maps": gpu_maps, "cpu_maps": cpu_maps,
            "warmup_seconds": round(t_warm, 2),
            # CPU time of this (rank-0) process per timed job: its TaskTracker,
            # the driver (and the JobTracker with its RPC handlers, when it
            # runs here: one rank, or hbmr.jobtracker.process=false)
            "rank0_cpu_ms_per_step": round(cpu_rank0 / a.steps * 1e3, 3),
            # with several ranks the JobTracker is a process of its own
            # (hbmr.jobtracker.process): its CPU per timed job, not in rank 0's
            "jobtracker_process": bool(jt_proc),
            "jobtracker_cpu_ms_per_step": None if jt_cpu is None else
            round(jt_cpu / a.steps * 1e3, 3),
            # the JobTracker process's CPU per timed job by thread group
            "jobtracker_thread_cpu_ms_per_step": jt_thr,
            "final_shift": hist[-1].get("shift") if hist else None,
            "maps_per_tracker_last_job": hist[-1].get("maps_per_tracker") if hist else None,
            # per job signature: completed-task mean seconds on each slot type (over
            # every job, warm-up included), the live estimate the scheduler uses
            # (EWMA of the device time each batch adds, hbmr/gpu/busy.py) and the
            # number of tasks behind it (the CPU probe may still be running)
            "cost_model": {k: {s: {"mean_s": round(v["mean"], 6),
                                   "estimate_s": round(v["ewma"], 6), "n": v["n"],
                                   "running": v["running"]} for s, v in d.items()}
                           for k, d in cm.items()},
            "baseline_note": "BASELINE.md publishes only a ratio (hybrid 1.93x faster than stock "
                             "Hadoop scheduling on 2010 hardware); no absolute number to divide by",
        }
        print(json.dumps(out), flush=True)
    finally:
        if sampler is not None:
            sampler.dump()
        if cprof:
            dump_profiles(cprof)
        node.shutdown()
    return 0


def spawn_ranks(n):
    """torchrun-equivalent launcher: N rank processes of this script on one node.
    The parent never initialises HIP (it only spawns and waits)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
                       "HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, start_new_session=True))
    rc = 0

    def _term(signum, _frame):
        # the ranks run in sessions of their own: a SIGTERM to this launcher
        # (timeout, the driver) must not leave them behind
        for q in procs:
            try:
                os.killpg(q.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        raise SystemExit(128 + signum)
    signal.signal(signal.SIGTERM, _term)
    signal.signal(signal.SIGHUP, _term)
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench: rank {procs.index(p)} exited with {code}; stopping the others",
                          file=sys.stderr)
                    for q in live:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs:
            try:
                os.killpg(q.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        raise
    return rc


if __name__ == "__main__":
    rc = main()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # a rank leaves after its exit handlers (trace / profile dumps) without
        # interpreter finalization: daemon threads still inside torch / gloo /
        # RCCL C++ frames when the interpreter tears them down could abort the
        # process ("terminate called without an active exception", seen on
        # the box at 8 ranks with the stack sampler on) after the result line
        # was printed, failing the run
        import atexit
        atexit._run_exitfuncs()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(rc or 0)
    sys.exit(rc)
