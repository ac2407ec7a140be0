"""Matmul benchmarks (BASELINE config 4): the MFMA GEMM kernel alone (TFLOP/s,
vs torch.matmul = hipBLASLt for reference) and matmul map tasks through the
framework (panel of A per map task, Bᵀ resident).

  python tools/bench_matmul.py [--size 8192] [--m 65536 --k 8192 --n 8192 --split-rows 8192]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--split-rows", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--gemm", default="hbmr", choices=["hbmr", "hipblaslt"],
                    help="map-task GEMM (hbmr.matmul.gemm)")
    a = ap.parse_args()
    import torch

    from hbmr.ops import gemm as G
    s = a.size
    x = torch.rand(s, s, device="cuda", dtype=torch.bfloat16) * 2 - 1
    yt = torch.rand(s, s, device="cuda", dtype=torch.bfloat16) * 2 - 1
    flops = 2.0 * s ** 3
    t_k = _time(lambda: G.matmul_tn(x, yt), a.reps)
    t_bf = _time(lambda: G.matmul_tn(x, yt, out_dtype=torch.bfloat16), a.reps)
    t_t = _time(lambda: torch.matmul(x, yt.t()), a.reps)
    res = {"gemm_size": s, "hbmr_tflops_f32out": round(flops / t_k / 1e12, 1),
           "hbmr_tflops_bf16out": round(flops / t_bf / 1e12, 1),
           "torch_hipblaslt_tflops_bf16out": round(flops / t_t / 1e12, 1)}
    del x, yt

    from hbmr.gpu.syncjob import sync_conf
    from hbmr.mapred.cluster import LocalCluster
    from hbmr.mapred.jobconf import JobConf
    from hbmr.models import matmul as MM
    conf = JobConf()
    conf.set_int("hbmr.gpu.queue.depth", 16)
    conf.set_int("mapred.task.timeout", 0)
    conf.set("hbmr.matmul.gemm", a.gemm)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        job = MM.matmul_conf(conf, m=a.m, k=a.k, n=a.n, split_rows=a.split_rows,
                             out_dtype="bfloat16")
        cl.submit_job(job).waitForCompletion()
        cl.submit_job(sync_conf(conf)).waitForCompletion()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            rj = cl.submit_job(MM.matmul_conf(conf, m=a.m, k=a.k, n=a.n, split_rows=a.split_rows,
                                              out_dtype="bfloat16"))
            rj.waitForCompletion()
            assert rj.isSuccessful(), rj.getFailureInfo()
        cl.submit_job(sync_conf(conf)).waitForCompletion()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
    res.update(gemm=a.gemm, job_m=a.m, job_k=a.k, job_n=a.n, split_rows=a.split_rows,
               job_seconds=round(dt, 4), job_tflops=round(2.0 * a.m * a.k * a.n / dt / 1e12, 1),
               map_tasks_per_s=round(-(-a.m // a.split_rows) / dt, 1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
