"""Numerics of the K-Means HIP kernels vs a plain PyTorch fp32 reference."""
import pytest
import torch

from hbmr.ops import kmeans as km


def _ref_scores(x32, c32):
    # score_j = x·c_j - ||c_j||²/2  (argmax == argmin distance)
    return x32 @ c32.T - 0.5 * (c32 * c32).sum(1)[None, :]


def _check_assign(n, d, k, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    dev = torch.device("cuda")
    x = torch.randn(n, d, generator=g).to(dev)
    c = torch.randn(k, d, generator=g).to(dev) * 1.5
    dp = km.padded_dim(d)
    xb = torch.zeros(n, dp, dtype=torch.bfloat16, device=dev)
    xb[:, :d] = x.to(torch.bfloat16)
    img = km.CentroidImage(c, dev)
    scores = torch.empty(n, dtype=torch.float32, device=dev)
    lab = km.assign(xb, img, scores=scores)
    torch.cuda.synchronize()
    assert lab.min().item() >= 0 and lab.max().item() < k
    # reference on the same bf16-rounded operands, fp32 math
    xr = xb[:, :d].float()
    cr = img.cbf[:k, :d].float()
    s = _ref_scores(xr, cr)
    best = s.max(1).values
    got = s.gather(1, lab.long()[:, None])[:, 0]
    scale = (xr.norm(dim=1) * cr.norm(dim=1).max() + 1.0)
    gap = (best - got) / scale
    assert gap.max().item() < 2e-4, f"assign off: max rel gap {gap.max().item()}"
    # exact agreement on the vast majority of points
    agree = (s.argmax(1) == lab.long()).float().mean().item()
    assert agree > 0.995, agree
    # kernel score ≈ best score
    assert torch.allclose(scores, best, rtol=1e-3, atol=1e-2 * scale.mean().item())
    return xb, lab, img


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,k", [(1000, 128, 64), (4099, 128, 1024), (777, 64, 100),
                                   (513, 256, 192), (300, 100, 7)])
def test_assign_matches_fp32_reference(n, d, k):
    _check_assign(n, d, k)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [km.ACCUM_AUTO, km.ACCUM_LDS, km.ACCUM_SORTED])
@pytest.mark.parametrize("n,d,k", [(20000, 128, 64), (30011, 128, 1024), (5000, 64, 3000),
                                   (7001, 256, 40)])
def test_accumulate_matches_index_add(n, d, k, mode):
    xb, lab, img = _check_assign(n, d, k, seed=1)
    dev = xb.device
    dp = xb.shape[1]
    sums, counts = km.new_partials(k, dp, dev)
    km.accumulate(xb, lab, k, sums, counts, mode=mode)
    torch.cuda.synchronize()
    # exact: fixed-point of bf16 inputs, integer sums
    fx = torch.round(xb.double() * (1 << km.FX_SHIFT)).long()
    ref_s = torch.zeros(k, dp, dtype=torch.int64, device=dev).index_add_(0, lab.long(), fx)
    ref_c = torch.bincount(lab.long(), minlength=k)
    assert torch.equal(counts, ref_c)
    assert torch.equal(sums, ref_s)
    # and order independence: a second run over a permutation gives identical bits
    perm = torch.randperm(n, device=dev)
    s2, c2 = km.new_partials(k, dp, dev)
    km.accumulate(xb[perm].contiguous(), lab[perm].contiguous(), k, s2, c2, mode=mode)
    assert torch.equal(s2, sums) and torch.equal(c2, counts)


@pytest.mark.gpu
def test_update_and_iteration_converges():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    k, d, n = 16, 128, 50000
    true_c = torch.randn(k, d, device=dev) * 8
    lab_true = torch.randint(0, k, (n,), device=dev)
    x = true_c[lab_true] + torch.randn(n, d, device=dev)
    xb = x.to(torch.bfloat16).contiguous()
    init = x[torch.randperm(n, device=dev)[:k]]
    img = km.CentroidImage(init, dev)
    for _ in range(15):
        sums, counts = km.new_partials(k, d, dev)
        km.map_split_gpu(xb, img, sums, counts)
        img.refresh(sums, counts)
    torch.cuda.synchronize()
    # reference Lloyd step from the final centroids is a fixed point (within bf16)
    c = img.cen
    lab = ((x[:, None, :] - c[None]) ** 2).sum(-1).argmin(1) if n * k * d < 2e8 else None
    ref = torch.zeros(k, d, device=dev).index_add_(0, lab, x)
    cnt = torch.bincount(lab, minlength=k).clamp(min=1).float()[:, None]
    assert (ref / cnt - c).abs().max().item() < 0.05


def test_cpu_map_matches_reference():
    torch.manual_seed(0)
    n, d, k = 2000, 24, 9
    x = torch.randn(n, d)
    c = torch.randn(k, d)
    sums, counts = km.new_partials(k, d, "cpu")
    labels = torch.empty(n, dtype=torch.int32)
    cost = km.map_split_cpu(x, c, sums, counts, nthreads=3, labels=labels)
    dist = ((x[:, None, :] - c[None]) ** 2).sum(-1)
    ref = dist.argmin(1)
    assert (labels.long() == ref).float().mean().item() > 0.999
    fx = torch.round(x.double() * (1 << km.FX_SHIFT)).long()
    ref_s = torch.zeros(k, d, dtype=torch.int64).index_add_(0, labels.long(), fx)
    assert (sums - ref_s).abs().max().item() <= 2
    assert torch.equal(counts, torch.bincount(labels.long(), minlength=k))
    assert abs(cost - dist.min(1).values.sum().item()) / dist.min(1).values.sum().item() < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("k,dp,sizes", [(1024, 128, [5000, 1, 70000, 4096, 12345]),
                                        (64, 128, [3000, 9000]),
                                        (300, 64, [777, 20000, 5])])
def test_map_batch_matches_per_split(k, dp, sizes):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(3)
    splits = [torch.randn(n, dp, generator=g).to(dev, torch.bfloat16) for n in sizes]
    img = km.CentroidImage(torch.randn(k, dp, generator=g).to(dev), dev)
    B = len(splits)
    sums = torch.full((B, k, dp), 7, dtype=torch.int64, device=dev)   # poisoned: must be zeroed
    counts = torch.full((B, k), 7, dtype=torch.int64, device=dev)
    nlab, nws = km.batch_scratch_sizes(sizes, k)
    labels = torch.empty(nlab, dtype=torch.int32, device=dev)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev)
    km.map_batch_gpu(splits, img, sums, counts, labels, ws)
    torch.cuda.synchronize()
    for t, x in enumerate(splits):
        lab = km.assign(x, img)
        fx = torch.round(x.double() * (1 << km.FX_SHIFT)).long()
        ref_s = torch.zeros(k, dp, dtype=torch.int64, device=dev).index_add_(0, lab.long(), fx)
        ref_c = torch.bincount(lab.long(), minlength=k)
        assert torch.equal(counts[t], ref_c), t
        assert torch.equal(sums[t], ref_s), t
