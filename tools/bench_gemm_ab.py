"""A/B of the GEMM kernels (hbmr_gemm_set_kernel: 1 = v1, 8 = the 8-phase
kernel) against hipBLASLt (torch.matmul) at 8192^3 bf16, interleaved rounds on
one device; uniform [-1, 1) operands (zero-filled operands read high).  One
JSON line per size: best and median TF/s per arm over the rounds."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from hbmr.ops import gemm as G
    sizes = [int(x) for x in (sys.argv[1:] or ["8192", "4096"])]
    vers = os.environ.get("VERS", "1 8").split()
    lib = G._lib.load()
    for s in sizes:
        x = torch.rand(s, s, device="cuda", dtype=torch.bfloat16) * 2 - 1
        yt = torch.rand(s, s, device="cuda", dtype=torch.bfloat16) * 2 - 1
        ref = torch.matmul(x, yt.t())
        flops = 2.0 * s ** 3
        best = {}

        def run(v, reps=20):
            if v == "blas":
                fn = lambda: torch.matmul(x, yt.t())  # noqa: E731
            else:
                lib.hbmr_gemm_set_kernel(int(v))
                fn = lambda: G.matmul_tn(x, yt, out_dtype=torch.bfloat16)  # noqa: E731
            fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            b.synchronize()
            return a.elapsed_time(b) / reps / 1e3

        err = {}
        for v in vers:
            lib.hbmr_gemm_set_kernel(int(v))
            c = G.matmul_tn(x, yt, out_dtype=torch.bfloat16)
            err[v] = float((c.float() - ref.float()).abs().max())
        allt = {}
        for _ in range(int(os.environ.get("ROUNDS", "5"))):
            for v in ["blas"] + vers:
                t = run(v)
                best[v] = min(best.get(v, 1e9), t)
                allt.setdefault(v, []).append(t)
        lib.hbmr_gemm_set_kernel(-1)
        med = {v: sorted(ts)[len(ts) // 2] for v, ts in allt.items()}
        out = {"size": s, "tflops": {v: round(flops / t / 1e12, 1) for v, t in best.items()},
               "tflops_median": {v: round(flops / t / 1e12, 1) for v, t in med.items()},
               "vs_hipblaslt_median": {v: round(med["blas"] / t, 3) for v, t in med.items()},
               "max_abs_diff_vs_hipblaslt": err}
        print(json.dumps(out), flush=True)
        del x, yt, ref


if __name__ == "__main__":
    main()
