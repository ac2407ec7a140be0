"""Exact K-Means mode (hbmr.kmeans.exact): top-3 MFMA assign on fp16 (default)
or bf16 operands, certification of the arg-max against the fp32 data with
fp64 re-scoring of uncertain points, and the fp32-input fixed-point combiner.  GPU numerics are checked
against fp64 (the "exact" assignment of the fp32 data) and a plain fp32
PyTorch reference; the CPU test runs an exact-mode job on CPU slots."""
import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import kmeans as K


def truth_labels(x32, c32, chunk=1 << 18):
    """argmin_j |x - c_j|^2 in fp64 (ties to the lower index)."""
    c = c32.double()
    cn = (c * c).sum(1)
    out = []
    for a in range(0, x32.shape[0], chunk):
        x = x32[a:a + chunk].double()
        out.append((cn[None, :] - 2.0 * x @ c.T).argmin(1))
    return torch.cat(out).to(torch.int32)


def lloyd64(x32, c0, iters):
    """Lloyd's algorithm with fp64 assignments and the framework's storage
    rules: fixed-point (2^-24) partial sums and fp32 centroids."""
    c = c0.double().clone()
    q = torch.round(x32.double() * (1 << 24)).long()
    for _ in range(iters):
        lab = truth_labels(x32, c).long()
        s = torch.zeros(c.shape, dtype=torch.int64, device=c.device).index_add_(0, lab, q)
        n = torch.bincount(lab, minlength=c.shape[0]).double()[:, None]
        c = torch.where(n > 0, (s.double() / (1 << 24)) / n.clamp(min=1), c).float().double()
    return c


def test_exact_mode_job_on_cpu_slots_matches_fp64_lloyd():
    """Exact mode keeps the fp32 data on CPU slots (no bf16 storage rounding)."""
    n, k, d = 20000, 12, 16
    inp = f"synthetic:{n}:9"
    conf = JobConf()
    conf.set_boolean(K.EXACT_KEY, True)
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=k,
                             d=d, inp=inp, split_points=5000)
        for _ in range(3):
            drv.step()
        got = drv.centroids()
    x = K.synthetic_points(9, 0, n, d, k, "cpu")
    ref = lloyd64(x, K.initial_centroids(inp, k, d, exact=True), 3)
    err = (got.double() - ref).abs().max().item()
    assert err < 1e-4, err


# ------------------------------------------------------------------------------ GPU
def _blobs(n, d, k, seed, dup=2):
    """Points of the bench distribution with k/dup true centers, so about
    every cluster shares its blob with another centroid: many near-ties."""
    x = K.synthetic_points(seed, 0, n, d, max(1, k // dup), "cuda")
    g = torch.Generator(device="cuda").manual_seed(seed)
    c = x[torch.randperm(n, device="cuda", generator=g)[:k]].clone()
    return x, c


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_top3_assign_matches_fp32_reference(dtype):
    from hbmr.ops import kmeans as km
    dt = torch.float16 if dtype == "f16" else torch.bfloat16
    n, d, k = 40000, 128, 256
    x, c = _blobs(n, d, k, 3)
    img = km.CentroidImage(c, "cuda")
    sp = km.ExactSplit(x, km.padded_dim(d), dt)
    assert sp.xb.dtype == dt
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    cand = torch.empty(2 * n, dtype=torch.int32, device="cuda")
    sc, mg = torch.empty(n, device="cuda"), torch.empty(2 * n, device="cuda")
    km.assign_top3(sp.xb, img, lab, cand, sc, mg)
    # reference: fp32 scores of the 16-bit operands (what the MFMA computes)
    c16, ch = img.image16(dt)[:2]
    xb = sp.xb[:, :d].float()
    cb = c16[:k, :d].float()
    s = xb @ cb.T + ch[:k][None, :]
    top = s.topk(3, dim=1)
    got = torch.stack([lab.long(), cand[:n].long(), cand[n:].long()], 1)
    # scores of the kernel's picks must equal the reference top-3 scores up to
    # the accumulation-order / packing tolerance (ties may swap indices)
    picked = s.gather(1, got)
    tol = 1e-3 * top.values[:, :1].abs().clamp(min=1)
    # the default epilogue keeps the top two of 8 tracks (cluster bits 0-2):
    # when the best and the second share a track the third is not known and
    # the kernel reports t = b with a zero margin (certification step 2 then
    # defers the point to the neighbour scan)
    same = got[:, 2] == got[:, 0]
    assert ((got[same, 0] ^ got[same, 1]) & 7 == 0).all()   # 4 tracks (default)
    assert (mg[n:][same] == 0).all()
    assert same.float().mean().item() < 0.15
    cols = torch.ones_like(got, dtype=torch.bool)
    cols[same, 2] = False
    ok = ((picked - top.values).abs() <= tol) | ~cols
    assert ok.all(1).float().mean().item() > 0.9999
    # (the packed arg-max truncates 4 + log2(k/32) mantissa bits: near-equal
    # scores may swap, which the score check above already bounds)
    assert ((got == top.indices) | ~cols).all(1).float().mean().item() > 0.995
    ref_m = top.values[:, :1] - top.values[:, 1:]
    got_m = torch.stack([mg[:n], mg[n:]], 1)
    okm = ((got_m - ref_m).abs() <= tol + 1e-2) | ~cols[:, 1:]
    assert okm.all(1).float().mean().item() > 0.999
    if dt == torch.bfloat16:
        assert torch.equal(lab, km.assign(sp.xb, img))   # same winner as the plain kernel


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_exact_prep_and_image16_match_fp64(dtype):
    """The native staging kernels: the 16-bit copies are round-to-nearest of the
    fp32 data (fp16 saturated at ±65504), and |x|, |x~|², |x - x~|, |c|,
    |c - c~| match fp64 (the errors as upper bounds)."""
    from hbmr.ops import kmeans as km
    dt = torch.float16 if dtype == "f16" else torch.bfloat16
    n, d, k = 5000, 120, 70
    x = torch.randn(n, d, device="cuda") * 20
    x[0, 0] = 1e6          # saturates in fp16
    x[1, :] = 1e-6         # fp16 subnormals
    sp = km.ExactSplit(x, km.padded_dim(d), dt)
    dp = km.padded_dim(d)
    lim = 65504.0 if dt == torch.float16 else float("inf")
    want = x.clamp(-lim, lim).to(dt)
    assert torch.equal(sp.xb[:, :d], want) and int((sp.xb[:, d:] != 0).sum()) == 0
    x64, w64 = x.double(), want.double()
    assert torch.allclose(sp.xnorm.double(), x64.norm(dim=1), rtol=1e-6)
    assert torch.allclose(sp.xbn2.double(), w64.pow(2).sum(1), rtol=1e-6)
    e = (x64 - w64).norm(dim=1)
    assert (sp.xerr.double() >= e).all() and torch.allclose(sp.xerr.double(), e, rtol=1e-6)
    img = km.CentroidImage(x[:k] * 0.5, "cuda")
    c16, ch, cn, cm, ce, cem = img.image16(dt)
    cw = (x[:k] * 0.5).clamp(-lim, lim).to(dt)
    assert torch.equal(c16[:k, :d], cw) and c16.shape == (img.k_pad, dp)
    c64 = (x[:k] * 0.5).double()
    assert (cn.double() >= c64.norm(dim=1)).all() and torch.allclose(cn.double(), c64.norm(dim=1))
    ee = (c64 - cw.double()).norm(dim=1)
    assert (ce.double() >= ee).all() and torch.allclose(ce.double(), ee, rtol=1e-6)
    assert cm.item() == cn.max().item() and cem.item() == ce.max().item()
    assert torch.allclose(ch[:k].double(), -0.5 * cw.double().pow(2).sum(1), rtol=1e-5)
    assert (ch[k:] < -1e29).all()


@pytest.mark.gpu
@pytest.mark.parametrize("d,dtype", [(64, "f16"), (128, "f16"), (128, "bf16")])
def test_exact_assign_agrees_with_fp64(d, dtype):
    from hbmr.ops import kmeans as km
    dt = torch.float16 if dtype == "f16" else torch.bfloat16
    n, k = 1_000_000, 256
    x, c = _blobs(n, d, k, 11)
    img = km.CentroidImage(c, "cuda")
    sp = km.ExactSplit(x, km.padded_dim(d), dt)
    truth = truth_labels(x, c)
    first = torch.empty(n, dtype=torch.int32, device="cuda")
    cand = torch.empty(2 * n, dtype=torch.int32, device="cuda")
    sc, mg = torch.empty(n, device="cuda"), torch.empty(2 * n, device="cuda")
    km.assign_top3(sp.xb, img, first, cand, sc, mg)
    stats = torch.zeros(3, dtype=torch.int64, device="cuda")
    lab = km.assign_exact(sp, img, stats)
    agree_exact = (lab == truth).float().mean().item()
    agree_first = (first == truth).float().mean().item()
    flagged, relabelled, rescans = stats.tolist()
    print(f"d={d} {dtype}: MFMA arg-max agreement {agree_first:.6f}, exact {agree_exact:.7f}, "
          f"flagged {flagged / n:.4f}, relabelled {relabelled}, neighbour scans {rescans}")
    assert int((lab != truth).sum()) <= 1          # fp64 ties aside: the exact assignment
    assert 0 < flagged < n and relabelled == int((first != lab).sum())


@pytest.mark.gpu
def test_exact_assign_with_saturated_fp16_data():
    """Data beyond fp16 range: the saturated copy is still certified against
    the fp32 rows (its rounding error enters the bound), so the labels stay
    the fp64 truth — more of them re-scored."""
    from hbmr.ops import kmeans as km
    n, d, k = 200_000, 64, 128
    x, c = _blobs(n, d, k, 17)
    x = x * 3000.0           # |x_i| up to ~1.5e5 > 65504
    c = c * 3000.0
    img = km.CentroidImage(c, "cuda")
    sp = km.ExactSplit(x, km.padded_dim(d))
    stats = torch.zeros(3, dtype=torch.int64, device="cuda")
    lab = km.assign_exact(sp, img, stats)
    assert int((lab != truth_labels(x, c)).sum()) <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("grouped,fused", [(True, True), (True, False), (False, False)])
def test_assign_exact_batch_equals_per_split(grouped, fused, monkeypatch):
    """The batched exact assign (labels written back to back, shared scratch;
    grouped: one top-3 launch and one step-1 launch for the batch; fused: step
    1 inside the top-3 epilogue, no candidate arrays) gives each split the
    labels and stats (flagged, relabelled, scanned) the per-split call gives."""
    from hbmr.ops import kmeans as km
    monkeypatch.setattr(km, "GROUPED_EXACT", grouped)
    monkeypatch.setattr(km, "FUSED_Q1", fused)
    d, k = 128, 256
    x, c = _blobs(210_000, d, k, 5)
    img = km.CentroidImage(c, "cuda")
    cuts = [0, 50_000, 130_000, 210_000]           # splits of different sizes
    sps = [km.ExactSplit(x[a:b].contiguous(), km.padded_dim(d)) for a, b in zip(cuts, cuts[1:])]
    s1 = torch.zeros(5, dtype=torch.int64, device="cuda")
    want = torch.cat([km.assign_exact(sp, img, s1).clone() for sp in sps])
    s2 = torch.zeros(5, dtype=torch.int64, device="cuda")
    got = torch.full((cuts[-1] + 7,), -1, dtype=torch.int32, device="cuda")
    km.assign_exact_batch(sps, img, s2, got, {})
    assert torch.equal(got[:cuts[-1]], want) and int((got[cuts[-1]:] != -1).sum()) == 0
    assert s1.tolist() == s2.tolist()


@pytest.mark.gpu
def test_accum_f32_is_fixed_point_of_fp32_data():
    from hbmr.ops import kmeans as km
    n, d, k = 300000, 128, 1024
    x = torch.randn(n, d, device="cuda") * 30
    lab = torch.randint(0, k, (n,), device="cuda", dtype=torch.int32)
    sums = torch.zeros(k, d, dtype=torch.int64, device="cuda")
    counts = torch.zeros(k, dtype=torch.int64, device="cuda")
    km.accumulate(x.contiguous(), lab, k, sums, counts)
    q = torch.round(x.double() * (1 << km.FX_SHIFT)).long()     # round-half-even
    ref = torch.zeros(k, d, dtype=torch.int64, device="cuda").index_add_(0, lab.long(), q)
    assert torch.equal(sums, ref)
    assert torch.equal(counts, torch.bincount(lab.long(), minlength=k))


@pytest.mark.gpu
def test_exact_mode_job_matches_fp64_lloyd():
    n, k, d, sp = 400000, 64, 128, 100000
    inp = f"synthetic:{n}:5"
    conf = JobConf()
    conf.set_boolean(K.EXACT_KEY, True)
    conf.set(K.NCENTERS_KEY, str(k // 2))     # duplicated blobs: near-ties
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=k,
                             d=d, inp=inp, split_points=sp)
        for _ in range(3):
            r = drv.step()
        got = drv.centroids()
        flagged = r["counters"].get("KMEANS", "EXACT_FLAGGED_POINTS")
    x = K.synthetic_points(5, 0, n, d, k // 2, "cuda")
    ref = lloyd64(x, K.initial_centroids(inp, k, d, centers=k // 2, exact=True).cuda(), 3)
    # identical assignments: centroids differ only by the 2^-24 fixed-point rounding
    assert (got.cuda().double() - ref).abs().max().item() < 1e-5
    assert flagged > 0


def test_kmeans_driver_resumes_from_checkpoint(tmp_path):
    """A driver that stops after 2 iterations and a new one resumed from its
    checkpoint directory produce the same centroids as 3 uninterrupted
    iterations (fixed-point partials make the iteration exact)."""
    import os
    import time as _t
    n, k, d = 12000, 6, 8
    inp = f"synthetic:{n}:21"
    ck = str(tmp_path / "ck")
    conf = JobConf()
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        res = lambda rj: rj._impl.jip.result[0]   # noqa: E731
        ref = K.KMeansDriver(cl.submit_job, res, conf=conf, k=k, d=d, inp=inp, split_points=3000)
        for _ in range(3):
            ref.step()
        want = ref.centroids().clone()
        a = K.KMeansDriver(cl.submit_job, res, conf=conf, k=k, d=d, inp=inp, split_points=3000,
                           checkpoint_dir=ck)
        a.step()
        a.step()
        f2 = os.path.join(ck, K._centroid_file("", a.key(2)))
        for _ in range(200):             # the reduce writes centroid files asynchronously
            if os.path.exists(f2):
                break
            _t.sleep(0.01)
        K.STORE.host.clear()
        K.STORE.images.clear()
        b = K.KMeansDriver.resume(cl.submit_job, res, ck, conf=conf)
        assert b.iteration == 2 and b.run_id == a.run_id
        b.step()
        got = b.centroids()
    assert torch.equal(got, want)


def test_prefetched_iterations_match_and_wait_for_their_dependency():
    """step(prefetch=True) submits iteration i+1 held on iteration i
    (hbmr.job.depends.on): same centroids as plain steps; a held job starts
    only after its dependency finished; a cancelled one is killed."""
    n, k, d = 12000, 6, 8
    inp = f"synthetic:{n}:23"
    conf = JobConf()
    res = lambda rj: rj._impl.jip.result[0]   # noqa: E731
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        a = K.KMeansDriver(cl.submit_job, res, conf=conf, k=k, d=d, inp=inp, split_points=3000)
        for _ in range(4):
            a.step()
        want = a.centroids().clone()
        b = K.KMeansDriver(cl.submit_job, res, conf=conf, k=k, d=d, inp=inp, split_points=3000)
        b.prefetch_delay = 0.0
        for s in range(4):
            b.step(prefetch=s < 3)
        got = b.centroids()
        jobs = [cl.jt.jobs[h["job"]] for h in b.history]
        for prev, nxt in zip(jobs, jobs[1:]):
            # released by the dependency's finish, or (a loaded host) submitted
            # only after it finished: never started before it
            assert (nxt.release_time or nxt.submit_time) >= prev.status.finish_time > 0
            assert nxt.t_first_map >= nxt.release_time
        c = K.KMeansDriver(cl.submit_job, res, conf=conf, k=k, d=d, inp=inp, split_points=3000)
        c.prefetch_delay = 0.0
        c.step(prefetch=True)
        held = c._ahead[0]
        c.cancel_prefetch()
        assert held.waitForCompletion(10)
        assert held.status().state == "KILLED"   # (released and running by then)
    assert torch.equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_refine_queue_pipeline_equals_single_kernel(dtype, monkeypatch):
    """Refine v3 (step 1 / step 2 / Elkan as compacted queues) gives the same
    labels and the same flagged / relabelled / scan counts as the v2 kernel."""
    from hbmr.ops import kmeans as km
    dt = torch.float16 if dtype == "f16" else torch.bfloat16
    n, d, k = 600_000, 128, 512
    x, c = _blobs(n, d, k, 23)
    img = km.CentroidImage(c, "cuda")
    sp = km.ExactSplit(x, km.padded_dim(d), dt)
    out = {}
    for v in (2, 3):
        monkeypatch.setattr(km, "REFINE_VERSION", v)
        st = torch.zeros(5, dtype=torch.int64, device="cuda")
        lab = km.assign_exact(sp, img, st, {}).clone()
        out[v] = (lab, st.tolist())
    assert torch.equal(out[2][0], out[3][0])
    # v3 flags fewer points (step 1's pair rule) and relabels the same ones;
    # its step 2 decides in fp32 with error bands and defers the (rare) points
    # inside a band to the neighbour scan
    f2, r2, n2 = out[2][1][:3]
    f3, r3, n3 = out[3][1][:3]
    assert 0 < f3 <= f2 and r2 == r3
    assert n3 <= n2 + max(16, f3 // 1000)
    assert int((out[3][0] != truth_labels(x, c)).sum()) <= 1


@pytest.mark.gpu
def test_native_centroid_neighbour_table_bounds():
    """hbmr_kmeans_centroid_nbr: per centroid the L nearest by a lower bound
    rounded down (ascending, ties by index), and the [k, k] upper bounds
    rounded up — checked against fp64 pairwise distances (a duplicated
    centroid gives an off-diagonal zero)."""
    from hbmr.ops import kmeans as km
    g = torch.Generator().manual_seed(3)
    k, d, L = 300, 40, 64
    c = torch.randn(k, d, generator=g) * 3
    c[7] = c[5]
    img = km.CentroidImage(c, "cuda")
    di, f, L2 = img.neighbors(L)
    pd = img.pair_dist()
    torch.cuda.synchronize()
    cd = c.double()
    exact = ((cd[:, None, :] - cd[None, :, :]) ** 2).sum(-1).sqrt()
    di, f, pd = di.cpu().long(), f.cpu().double(), pd.cpu().double()
    assert L2 == L and di.shape == (k, L)
    true = exact[torch.arange(k)[:, None], di]
    assert (f <= true).all() and (f >= true * (1 - 1e-6) - 1e-12).all()
    assert (pd >= exact).all() and (pd <= exact * (1 + 1e-6) + 1e-12).all()
    assert (f[:, 1:] >= f[:, :-1]).all()
    assert di[5, 0].item() == 5 and di[5, 1].item() == 7 and di[7, 0].item() == 5
    own = di[:, 0] == torch.arange(k)
    assert own.sum().item() == k - 1           # every centroid first but 7 (5 ties first)
    kth = exact.sort(dim=1).values[:, L - 1]
    assert (true <= kth[:, None] * (1 + 1e-6) + 1e-9).all()


def test_exact_mode_starts_from_the_fp32_points():
    """Exact mode's first centroids are the fp32 first-k points; the bf16 mode
    keeps their bf16 roundings (what its image holds)."""
    inp = "synthetic:1000:5"
    x = K.synthetic_points(5, 0, 16, 24, 16, "cpu")
    assert torch.equal(K.initial_centroids(inp, 16, 24, exact=True), x)
    assert torch.equal(K.initial_centroids(inp, 16, 24), x.to(torch.bfloat16).float())


def _only_ties(x, c, got, want):
    """Every label that differs from the fp64 arg-min is an exact fp64 tie."""
    bad = (got != want).nonzero().flatten()
    if bad.numel() == 0:
        return 0
    xb = x[bad].double()
    cd = c.double()
    dg = ((xb - cd[got[bad].long()]) ** 2).sum(1)
    dw = ((xb - cd[want[bad].long()]) ** 2).sum(1)
    assert torch.equal(dg, dw), (bad[:8].tolist(), (dg - dw)[:8].tolist())
    return bad.numel()


@pytest.mark.gpu
def test_exact_batch_labels_at_bench_shape():
    """The bench's shape and distribution (k = 1024 centers, d = 128): the
    packed arg-max keeps 9 fewer mantissa bits at k = 1024 (4 + log2(k/32)),
    yet every certified label is the fp64 arg-min of the fp32 data (up to fp64
    ties), for the default fused kernel (v3) and the round-4 one (v2)."""
    from hbmr.ops import kmeans as km
    n, d, k, split = 2_000_000, 128, 1024, 250_000
    x = K.synthetic_points(7, 0, n, d, k, "cuda")
    c = K.initial_centroids(f"synthetic:{n}:7", k, d, exact=True).cuda()
    for _ in range(3):                                   # centroids of a few Lloyd steps
        lab = truth_labels(x, c).long()
        s = torch.zeros(k, d, dtype=torch.float64, device="cuda").index_add_(0, lab, x.double())
        cnt = torch.bincount(lab, minlength=k).double()[:, None]
        c = torch.where(cnt > 0, s / cnt.clamp(min=1), c.double()).float()
    img = km.CentroidImage(c, "cuda")
    sps = [km.ExactSplit(x[a:a + split].contiguous(), km.padded_dim(d))
           for a in range(0, n, split)]
    want = truth_labels(x, c)
    lib = km._lib.load()
    try:
        for kern in (3, 2):                              # v3 (default) and v2
            lib.hbmr_kmeans_set_exact_kernel(kern)
            st = torch.zeros(5, dtype=torch.int64, device="cuda")
            got = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            km.assign_exact_batch(sps, img, st, got, {})
            assert _only_ties(x, c, got, want) <= 4
            assert st[0].item() > 0                      # the certification had work
    finally:
        lib.hbmr_kmeans_set_exact_kernel(-1)


@pytest.mark.gpu
def test_exact_mode_job_at_bench_shape_matches_fp64_lloyd():
    """Three iteration jobs at k = 1024, d = 128 on 2M points of the bench
    distribution, through the JobTracker / GPU slots: the centroids equal
    fp64-assignment Lloyd's with the framework's 2^-24 fixed-point sums."""
    n, k, d, sp = 2_000_000, 1024, 128, 250_000
    inp = f"synthetic:{n}:7"
    conf = JobConf()
    conf.set_boolean(K.EXACT_KEY, True)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        drv = K.KMeansDriver(cl.submit_job, lambda rj: rj._impl.jip.result[0], conf=conf, k=k,
                             d=d, inp=inp, split_points=sp)
        for _ in range(3):
            drv.step()
        got = drv.centroids()
    x = K.synthetic_points(7, 0, n, d, k, "cuda")
    ref = lloyd64(x, K.initial_centroids(inp, k, d, exact=True).cuda(), 3)
    assert (got.cuda().double() - ref).abs().max().item() < 1e-5
