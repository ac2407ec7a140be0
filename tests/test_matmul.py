"""Mars-style matmul map tasks (BASELINE config 4) and the bf16 MFMA GEMM kernel."""
import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import matmul as MM
from hbmr.ops import gemm as G


def _ref(m, k, n, seed=1):
    a = MM.synthetic_matrix(seed, 0, m, k, "cpu").float()
    b = MM.synthetic_matrix(seed + 1, 0, k, n, "cpu").float()
    return a @ b


def test_synthetic_matrix_panels_are_consistent():
    full = MM.synthetic_matrix(3, 0, 50, 17, "cpu")
    assert torch.equal(full[20:35], MM.synthetic_matrix(3, 20, 15, 17, "cpu"))
    assert full.float().abs().max() <= 1.0 and full.float().std() > 0.4


@pytest.mark.parametrize("trackers", [1, 2])
def test_matmul_job_cpu_checksum(trackers):
    m, k, n = 1000, 96, 80
    with LocalCluster(JobConf(), num_trackers=trackers, cpu_slots=2) as cl:
        rj = cl.submit_job(MM.matmul_conf(m=m, k=k, n=n, split_rows=256))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result
    ref = _ref(m, k, n).double().sum().item()
    for r in res.values():
        assert abs(r["checksum"] - ref) < 1e-6 * max(1.0, abs(ref)) + 1e-3
    assert sum(r["rows"] for r in res.values()) == m


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n", [(256, 64, 256), (512, 192, 768), (1000, 300, 100),
                                   (2048, 1024, 1536),
                                   # ragged: edge tiles zero-filled in-kernel (K % 8 == 0
                                   # runs without any host padding)
                                   (300, 136, 520), (1, 8, 1), (257, 72, 255),
                                   (4097, 200, 33), (640, 1000, 384)])
def test_gemm_kernel_matches_fp32_reference(m, k, n):
    g = torch.Generator().manual_seed(m + k + n)
    a = torch.randn(m, k, generator=g).to(torch.bfloat16)
    bt = torch.randn(n, k, generator=g).to(torch.bfloat16)
    ref = a.float() @ bt.float().t()
    c = G.matmul_tn(a.cuda(), bt.cuda()).cpu()
    assert torch.allclose(c, ref, atol=2e-3 * k ** 0.5, rtol=1e-3), (c - ref).abs().max()
    cb = G.matmul_tn(a.cuda(), bt.cuda(), out_dtype=torch.bfloat16).cpu().float()
    assert torch.allclose(cb, ref, atol=0.05 * k ** 0.5, rtol=2e-2)
    # the epilogue checksum is the fp64 sum of C as stored (padding adds zeros)
    for dt in (torch.float32, torch.bfloat16):
        c2, cs = G.matmul_tn(a.cuda(), bt.cuda(), out_dtype=dt, with_sum=True)
        want = c2.double().sum().item()
        assert abs(cs.item() - want) <= 1e-9 * max(1.0, c2.double().abs().sum().item())


@pytest.mark.gpu
def test_gemm_layout_identity_with_asymmetric_b():
    # A = I catches a transposed C write that a symmetric B would hide
    n = 256
    a = torch.eye(n, dtype=torch.bfloat16)
    b = (torch.arange(n * n).reshape(n, n) % 97).to(torch.bfloat16)   # asymmetric
    c = G.matmul(a.cuda(), b.cuda()).cpu()
    assert torch.equal(c, b.float())


@pytest.mark.gpu
@pytest.mark.parametrize("gemm", ["hipblaslt", "hbmr"])
def test_matmul_job_gpu(gemm):
    m, k, n = 4096, 512, 1024
    conf = JobConf()
    conf.set(MM.GEMM_KEY, gemm)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        rj = cl.submit_job(MM.matmul_conf(conf, m=m, k=k, n=n, split_rows=1024))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result[0]
    ref = _ref(m, k, n).double().sum().item()
    assert abs(res["checksum"] - ref) < 1e-4 * (abs(ref) + m * n ** 0.5)
    cs = rj.getCounters()
    assert cs.get("org.apache.hadoop.mapred.JobInProgress$Counter", "GPU_MAP_TASKS") == 4


@pytest.mark.gpu
@pytest.mark.parametrize("kern", [1, 8])
@pytest.mark.parametrize("m,k,n", [(256, 128, 256), (512, 384, 768), (768, 4096, 512),
                                   (2048, 1024, 1536)])
def test_gemm_kernels_match_fp32_reference(kern, m, k, n):
    """The tile-multiple kernels (hbmr_gemm_set_kernel: 1 = v1, 8 = the 8-phase
    kernel, the default) against the fp32 reference, K from one 8-phase
    iteration (two K-tiles) to 64 of them, plus the fused checksum."""
    lib = G._lib.load()
    old = lib.hbmr_gemm_set_kernel(kern)
    try:
        g = torch.Generator().manual_seed(m * 7 + k + n)
        a = (torch.rand(m, k, generator=g) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(n, k, generator=g) * 2 - 1).to(torch.bfloat16)
        ref = a.float() @ bt.float().t()
        c, cs = G.matmul_tn(a.cuda(), bt.cuda(), with_sum=True)
        c = c.cpu()
        assert torch.allclose(c, ref, atol=2e-3 * k ** 0.5, rtol=1e-3), (c - ref).abs().max()
        assert abs(cs.item() - c.double().sum().item()) <= \
            1e-9 * max(1.0, c.double().abs().sum().item())
        cb = G.matmul_tn(a.cuda(), bt.cuda(), out_dtype=torch.bfloat16).cpu().float()
        assert torch.allclose(cb, ref, atol=0.05 * k ** 0.5, rtol=2e-2)
        # A = I with an asymmetric B: a transposed or misplaced C write shows
        eye = torch.eye(m, k, dtype=torch.bfloat16)
        ci = G.matmul_tn(eye.cuda(), bt.cuda()).cpu()
        assert torch.equal(ci, (eye.float() @ bt.float().t()))
    finally:
        lib.hbmr_gemm_set_kernel(old)
