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
    off = 0
    for t, x in enumerate(splits):
        lab = km.assign(x, img)
        # every task's labels at its offset (the delta combiner keeps them)
        assert torch.equal(labels[off:off + x.shape[0]], lab), t
        off += x.shape[0]
        fx = torch.round(x.double() * (1 << km.FX_SHIFT)).long()
        ref_s = torch.zeros(k, dp, dtype=torch.int64, device=dev).index_add_(0, lab.long(), fx)
        ref_c = torch.bincount(lab.long(), minlength=k)
        assert torch.equal(counts[t], ref_c), t
        assert torch.equal(sums[t], ref_s), t


# ---------------------------------------------------------------- delta combiner
def _fx_ref(x, lab, k):
    fx = torch.round(x.double() * (1 << km.FX_SHIFT)).long()
    s = torch.zeros(k, x.shape[1], dtype=torch.int64, device=x.device).index_add_(0, lab.long(), fx)
    return s, torch.bincount(lab.long(), minlength=k)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("k,dp,sizes,churn", [(1024, 128, [5000, 1, 70000, 4096], 0.05),
                                              (64, 128, [3000, 9000], 1.0),
                                              (300, 64, [777, 20000, 5], 0.3),
                                              (8192, 256, [30000], 0.01),
                                              (1024, 128, [4000, 4000], 0.0)])
def test_delta_combiner_is_bit_identical_to_direct(dtype, k, dp, sizes, churn):
    """sums/counts from a reference partition + movers equal the direct
    combiner's for the new labels, bit for bit; the baseline advances."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(11)
    xs = [(torch.randn(n, dp, generator=g) * 3).to(dev, dtype) for n in sizes]
    B = len(xs)
    bases, new_labs = [], []
    for x in xs:
        n = x.shape[0]
        l0 = torch.randint(0, k, (n,), generator=g).to(dev, torch.int32)
        s0, c0 = _fx_ref(x, l0, k)
        bases.append(km.Baseline(l0.clone(), s0, c0, x.data_ptr(), n))
        move = torch.rand(n, generator=g) < churn
        l1 = torch.where(move, torch.randint(0, k, (n,), generator=g), l0.cpu().long())
        new_labs.append(l1.to(dev, torch.int32))
    labcat = torch.cat(new_labs)
    sums = torch.full((B, k, dp), 7, dtype=torch.int64, device=dev)
    counts = torch.full((B, k), 7, dtype=torch.int64, device=dev)
    ws = torch.empty(km.delta_workspace_bytes(labcat.numel(), B, k), dtype=torch.uint8,
                     device=dev)
    km.delta_combine(xs, labcat, k, sums, counts, ws, bases)
    torch.cuda.synchronize()
    for t, (x, l1) in enumerate(zip(xs, new_labs)):
        rs, rc = _fx_ref(x, l1, k)
        assert torch.equal(counts[t], rc), t
        assert torch.equal(sums[t], rs), t
        assert torch.equal(bases[t].g, l1), t       # g advanced in place


@pytest.mark.gpu
def test_map_batch_delta_tracks_lloyd_iterations_exactly():
    """Several Lloyd iterations: the delta map batch (assign + movers) gives the
    same partials as the direct map batch at every step."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(5)
    k, dp = 256, 128
    centers = torch.randn(64, dp, generator=g) * 6
    sizes = [20000, 777, 50000]
    xs = []
    for n in sizes:
        lab = torch.randint(0, 64, (n,), generator=g)
        xs.append((centers[lab] + torch.randn(n, dp, generator=g)).to(dev, torch.bfloat16))
    img = km.CentroidImage(xs[0][:k].float(), dev)
    B, tot = len(xs), sum(sizes)
    nlab, nws = km.batch_scratch_sizes(sizes, k)
    labels = torch.empty(nlab, dtype=torch.int32, device=dev)
    ws = torch.empty(max(nws, km.delta_workspace_bytes(tot, B, k)), dtype=torch.uint8, device=dev)
    bases = None
    for it in range(5):
        ref_s = torch.empty(B, k, dp, dtype=torch.int64, device=dev)
        ref_c = torch.empty(B, k, dtype=torch.int64, device=dev)
        km.map_batch_gpu(xs, img, ref_s, ref_c, labels, ws)
        if bases is None:
            bases = []
            off = 0
            for t, x in enumerate(xs):
                n = x.shape[0]
                bases.append(km.Baseline(labels[off:off + n].clone(), ref_s[t].clone(),
                                         ref_c[t].clone(), x.data_ptr(), n))
                off += n
        else:
            s = torch.empty_like(ref_s)
            c = torch.empty_like(ref_c)
            km.map_batch_delta(xs, img, s, c, labels, ws, bases)
            torch.cuda.synchronize()
            assert torch.equal(s, ref_s), it
            assert torch.equal(c, ref_c), it
            for t, b in enumerate(bases):
                b.S0, b.N0 = s[t], c[t]
        img.refresh(ref_s.sum(0), ref_c.sum(0))
