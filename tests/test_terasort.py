"""TeraGen / TeraSort / TeraValidate (BASELINE config 5) — split-level job with
range partitioning and an all-to-all-v shuffle; GPU radix sort kernels are
checked against numpy on the device tests."""
import os

import numpy as np
import pytest
import torch

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf
from hbmr.models import terasort as T
from hbmr.ops import sort as S
from hbmr.parallel.collectives import COLLECTIVE_GROUP


def _ref_sorted(rows):
    recs = S.teragen_cpu(0, rows)
    order = np.lexsort([recs[:, j] for j in range(9, -1, -1)])
    return recs[order]


def test_teragen_matches_reference_generator():
    # the reference's RandomGenerator seed table is the LCG at multiples of 2^27
    seeds = S._lcg_jump_np(np.array([1 << 27, 2 << 27, 31 << 27], dtype=np.uint64))
    assert seeds.tolist() == [4160749568, 4026531840, 134217728]
    r = S.teragen_cpu(0, 2)
    assert bytes(r[0, :10]) == b".t^#\\|v$2\\"
    assert bytes(r[0, 10:20]) == b"         0"
    assert bytes(r[1, 20:30]) == b"IIIIIIIIII" and bytes(r[0, 98:]) == b"\r\n"
    # generating a later range directly equals generating everything
    assert np.array_equal(S.teragen_cpu(5, 7), S.teragen_cpu(0, 12)[5:])


def test_create_partitions_rule():
    keys = np.array([[i] * 10 for i in range(20)], dtype=np.uint8)
    sp = T.create_partitions(keys[::-1].copy(), 4)
    assert sp[:, 0].tolist() == [5, 10, 15]


@pytest.mark.parametrize("trackers,merge,waves,static,slack", [
    (1, False, 1, True, None), (2, False, 1, True, None), (3, False, 1, True, None),
    (3, True, 1, True, None), (3, False, 3, False, None), (2, True, 4, True, None),
    (2, False, 0, True, None), (3, False, 0, True, None), (3, False, 2, True, 0.05)])
def test_terasort_on_cluster_sorts_and_validates(tmp_path, trackers, merge, waves, static, slack):
    """merge: senders sort each destination's run and receivers merge the
    runs (K8 merge path) instead of re-sorting; waves: the shuffle runs in
    rounds over each rank's map outputs (0: the default, 4 waves on several
    ranks) — static-shape all-to-alls with device-side counts unless
    ``static`` is off; a slot slack far too small overflows and the shuffle
    re-runs with exact sizes — the same output bytes every time."""
    rows = 20000
    out = tmp_path / "out"
    with LocalCluster(JobConf(), num_trackers=trackers, cpu_slots=2) as cl:
        conf = T.terasort_conf(rows=rows, split_rows=3000, output=str(out))
        conf.set_boolean("hbmr.terasort.shuffle.sorted.runs", merge)
        conf.set_int("hbmr.terasort.shuffle.waves", waves)
        conf.set_boolean("hbmr.terasort.shuffle.static", static)
        if slack is not None:
            conf.set("hbmr.terasort.shuffle.slot.slack", str(slack))
        rj = cl.submit_job(conf)
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result
        ctr = {c.name: c.getValue() for c in rj.getCounters().group(COLLECTIVE_GROUP)}
    assert all(r["unsorted"] == 0 and r["checksum_ok"] for r in res.values())
    assert sum(r["records"] for r in res.values()) == rows
    if trackers > 1 and waves != 1 and static and not merge:
        # the data moved in static-shape all-to-alls (records + counts per wave)
        assert ctr.get("ALL_TO_ALL_FIXED_CPU", 0) >= 2 * trackers
        # ... unless a slot overflowed: then the exact-size waves ran as well
        assert (ctr.get("ALL_TO_ALL_V_CPU", 0) > 0) == (slack is not None), ctr
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert len(parts) == trackers
    got = np.concatenate([np.fromfile(out / p, dtype=np.uint8).reshape(-1, 100) for p in parts])
    assert np.array_equal(got, _ref_sorted(rows))


@pytest.mark.parametrize("group_bytes,gid", [(1, False), (300_000, False), (8 << 30, False),
                                            (300_000, True), (8 << 30, True)])
def test_terasort_partition_groups_one_rank(tmp_path, group_bytes, gid):
    """The one-rank reduce sorts consecutive partitions together (one per sort,
    a few, or all), through the permutation (v3) or packed record ids (v4);
    output files and order are the same."""
    rows = 12000
    out = tmp_path / "out"
    conf = T.terasort_conf(rows=rows, split_rows=2500, output=str(out), partitions=7)
    conf.set("hbmr.terasort.reduce.group.bytes", str(group_bytes))
    conf.set_boolean("hbmr.terasort.reduce.gid", gid)
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(conf)
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result[0]
    assert res["unsorted"] == 0 and res["checksum_ok"] and res["records"] == rows
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert parts == [f"part-{i:05d}" for i in range(7)]
    got = np.concatenate([np.fromfile(out / p, dtype=np.uint8).reshape(-1, 100) for p in parts])
    assert np.array_equal(got, _ref_sorted(rows))
    assert T.teravalidate(str(out))["misordered"] == 0


def test_terasort_in_hbm_redoes_a_flagged_group_on_the_full_key_path(monkeypatch):
    """In HBM the one-rank reduce reads no flag per group: a group whose tie
    runs were too long (flag set) is noticed after the last group and the
    reduce runs again on the full-key path — same validated result."""
    calls = {"gathered": 0, "full": 0}
    orig_sg, orig_tc = S.sort_gathered, S.tera_collect

    def sg(*a, **k):
        calls["gathered"] += 1
        got = orig_sg(*a, **k)
        if k.get("defer") and calls["gathered"] == 2:
            got = got[:3] + (torch.ones(1, dtype=torch.int32),)
        return got

    def tc(*a, **k):
        calls["full"] += 1
        return orig_tc(*a, **k)
    monkeypatch.setattr(S, "sort_gathered", sg)
    monkeypatch.setattr(S, "tera_collect", tc)
    rows = 12000
    conf = T.terasort_conf(rows=rows, split_rows=2500, partitions=5)
    conf.set("hbmr.terasort.reduce.group.bytes", str(300_000))
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(conf)
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result[0]
    assert res["unsorted"] == 0 and res["checksum_ok"] and res["records"] == rows
    assert calls["gathered"] == 5 and calls["full"] == 5


@pytest.mark.parametrize("trackers", [1, 2, 3])
def test_terasort_more_partitions_than_trackers(tmp_path, trackers):
    """R part files for any R (TeraSort.java writes one per reduce): a rank
    owning several partitions cuts its sorted range by the splitters; one rank
    alone sorts its partitions one at a time."""
    rows = 12000
    out = tmp_path / "out"
    with LocalCluster(JobConf(), num_trackers=trackers, cpu_slots=2) as cl:
        rj = cl.submit_job(T.terasort_conf(rows=rows, split_rows=2500, output=str(out),
                                           partitions=7))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result
    assert all(r["unsorted"] == 0 and r["checksum_ok"] for r in res.values())
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert parts == [f"part-{i:05d}" for i in range(7)]
    got = np.concatenate([np.fromfile(out / p, dtype=np.uint8).reshape(-1, 100) for p in parts])
    assert np.array_equal(got, _ref_sorted(rows))
    assert T.teravalidate(str(out))["misordered"] == 0


def test_terasort_rank_without_maps_writes_its_partitions(tmp_path):
    """2 splits on 3 trackers: at least one rank runs no map, yet owns two of
    the 7 partitions; it learns R and the splitters from its peers (the
    collective sequence is the same on every rank) and writes its part files."""
    rows = 5000
    out = tmp_path / "out"
    with LocalCluster(JobConf(), num_trackers=3, cpu_slots=2) as cl:
        rj = cl.submit_job(T.terasort_conf(rows=rows, split_rows=2500, output=str(out),
                                           partitions=7))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert parts == [f"part-{i:05d}" for i in range(7)]
    got = np.concatenate([np.fromfile(out / p, dtype=np.uint8).reshape(-1, 100) for p in parts])
    assert np.array_equal(got, _ref_sorted(rows))


def test_partition_ops_cpu():
    recs = torch.from_numpy(S.teragen_cpu(0, 5000))
    sp = T.create_partitions(recs.numpy()[::50, :10].copy(), 6)
    shi, slo = (torch.from_numpy(x.view(np.int64)) for x in T._key_words(sp))
    hi, lo, pid = S.tera_keys_part(recs, shi, slo)
    h = hi.numpy().view(np.uint64)
    lw = lo.numpy().view(np.uint64)
    keys = list(zip(h.tolist(), lw.tolist()))
    spl = list(zip(shi.numpy().view(np.uint64).tolist(), slo.numpy().view(np.uint64).tolist()))
    assert pid.tolist() == [sum(1 for s_ in spl if s_ <= k) for k in keys]


def test_terasort_from_teragen_files(tmp_path):
    inp = tmp_path / "in"
    inp.mkdir()
    S.teragen_cpu(0, 3000).tofile(inp / "part-00000")
    S.teragen_cpu(3000, 2000).tofile(inp / "part-00001")
    out = tmp_path / "out"
    with LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) as cl:
        rj = cl.submit_job(T.terasort_conf(inp=str(inp), split_rows=1500, output=str(out)))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
    got = np.concatenate([np.fromfile(out / p, dtype=np.uint8).reshape(-1, 100)
                          for p in sorted(os.listdir(out)) if p.startswith("part-")])
    assert np.array_equal(got, _ref_sorted(5000))


@pytest.mark.gpu
def test_gpu_teragen_bit_exact():
    a = S.teragen(123456789, 5000, device="cuda").cpu().numpy()
    assert np.array_equal(a, S.teragen_cpu(123456789, 5000))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 4096, 100003, 1 << 20])
def test_gpu_radix_sort_pairs_matches_numpy(n):
    g = torch.Generator().manual_seed(n)
    k = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
    k[::7] = k[0]   # duplicates: stability matters
    v = torch.arange(n, dtype=torch.int32)
    kd, vd = k.cuda(), v.cuda()
    S.radix_sort_pairs(kd, vd)
    kc, vc = k.clone(), v.clone()
    S.radix_sort_pairs(kc, vc)     # numpy stable reference
    assert torch.equal(kd.cpu(), kc) and torch.equal(vd.cpu(), vc)


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8, 16])
@pytest.mark.parametrize("n", [2, 1000, 4096, 4097, 16385, 100003, 3 << 20])
@pytest.mark.parametrize("window", [(32, 64), (0, 64), (3, 29), (40, 41)])
def test_gpu_onesweep_radix_sort_keys_matches_numpy(n, window, waves):
    """Keys-only onesweep sort (decoupled look-back): the stable numpy order
    of the window's bits, every tile count and window width (a last digit
    narrower than 8 bits), and the look-back never timed out."""
    g = torch.Generator().manual_seed(n + window[0])
    k = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
    k[::5] = k[1]   # duplicates: stability matters
    kd = k.cuda()
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    from hbmr.ops import _lib
    old = _lib.load().hbmr_radix_set_onesweep_waves(waves)
    try:
        S.radix_sort_keys(kd, *window, err=err)
    finally:
        _lib.load().hbmr_radix_set_onesweep_waves(old)
    kc = k.clone()
    S.radix_sort_keys(kc, *window)     # numpy stable reference
    assert int(err.item()) == 0
    assert torch.equal(kd.cpu(), kc)


@pytest.mark.gpu
def test_gpu_sort_records_and_partition():
    recs = S.teragen(0, 300000, device="cuda")
    srt, hs, ls = S.sort_records(recs)
    assert S.count_unsorted(hs, ls) == 0
    ref = _ref_sorted(300000)
    assert np.array_equal(srt.cpu().numpy(), ref)
    sp = T.create_partitions(ref[::97, :10].copy(), 8)
    hi, lo = T._key_words(sp)
    offs = S.split_offsets(hs, ls, torch.from_numpy(hi.view(np.int64)).cuda(),
                           torch.from_numpy(lo.view(np.int64)).cuda())
    offs_c = S.split_offsets(hs.cpu(), ls.cpu(), torch.from_numpy(hi.view(np.int64)),
                             torch.from_numpy(lo.view(np.int64)))
    assert offs.cpu().tolist() == offs_c.tolist()


@pytest.mark.gpu
def test_gpu_terasort_job(tmp_path):
    rows = 2_000_000
    with LocalCluster(JobConf(), num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        rj = cl.submit_job(T.terasort_conf(rows=rows, split_rows=500_000,
                                           output=str(tmp_path / "out")))
        rj.waitForCompletion(300)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result[0]
    assert res["records"] == rows and res["unsorted"] == 0 and res["checksum_ok"]
    got = np.fromfile(tmp_path / "out" / "part-00000", dtype=np.uint8).reshape(-1, 100)
    assert np.array_equal(got[:1000], _ref_sorted(rows)[:1000])


@pytest.mark.gpu
def test_gpu_partition_collect_and_multi_gather_match_cpu():
    n = 200000
    recs_c = torch.from_numpy(S.teragen_cpu(777, n))
    recs = recs_c.cuda()
    sp = T.create_partitions(recs_c.numpy()[::101, :10].copy(), 37)
    shi, slo = (torch.from_numpy(x.view(np.int64)) for x in T._key_words(sp))
    g = S.tera_keys_part(recs, shi, slo)
    c = S.tera_keys_part(recs_c, shi, slo)
    for a, b in zip(g, c):
        assert torch.equal(a.cpu(), b)
    # collect pieces of three "splits" and gather their records
    parts = [recs[:70000], recs[70000:150000], recs[150000:]]
    his = [S.tera_keys(p)[0] for p in parts]
    los = [S.tera_keys(p)[1] for p in parts]
    rows = [torch.arange(p.shape[0], dtype=torch.int32, device="cuda").flip(0).contiguous()
            for p in parts]
    starts, lens = [5, 0, 1000], [100, 70000, 17]
    h, lw, sp_, rw = S.tera_collect(his, los, rows, starts, lens)
    hc, lc, spc, rwc = S.tera_collect([x.cpu() for x in his], [x.cpu() for x in los],
                                      [x.cpu() for x in rows], starts, lens)
    assert torch.equal(h.cpu(), hc) and torch.equal(lw.cpu(), lc)
    assert torch.equal(sp_.cpu(), spc) and torch.equal(rw.cpu(), rwc)
    perm = torch.randperm(h.numel(), dtype=torch.int32).cuda()
    out = S.gather_records_multi(parts, sp_, rw, perm)
    outc = S.gather_records_multi([p.cpu() for p in parts], spc, rwc, perm.cpu())
    assert torch.equal(out.cpu(), outc)


@pytest.mark.gpu
def test_gpu_terasort_many_partitions_one_gpu(tmp_path):
    rows = 3_000_000
    with LocalCluster(JobConf(), num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        rj = cl.submit_job(T.terasort_conf(rows=rows, split_rows=700_000, partitions=6,
                                           output=str(tmp_path / "out")))
        rj.waitForCompletion(300)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result[0]
    assert res["records"] == rows and res["unsorted"] == 0 and res["checksum_ok"]
    assert res["partitions"] == 6
    v = T.teravalidate(str(tmp_path / "out"))
    assert v["files"] == 6 and v["records"] == rows and v["misordered"] == 0


@pytest.mark.gpu
def test_gpu_tera_partition_matches_cpu():
    """Map v3 (key/partition/count kernel + scan + tile-ranked scatter): the
    same partition boundaries as the CPU twin and, inside every partition,
    the same (hi, lo, row) multiset (order there is unspecified)."""
    n = 250_003
    recs_c = torch.from_numpy(S.teragen_cpu(4242, n))
    sp = T.create_partitions(recs_c.numpy()[::89, :10].copy(), 29)
    shi, slo = (torch.from_numpy(x.view(np.int64)) for x in T._key_words(sp))
    hg, lg, rg, og, kg = S.tera_partition(recs_c.cuda(), shi, slo, kbytes=True)
    hc, lc, rc, oc, kc = S.tera_partition(recs_c, shi, slo, kbytes=True)
    assert kg.cpu().tolist() == kc.tolist()
    assert torch.equal(og.cpu(), oc)
    hg, lg, rg = hg.cpu(), lg.cpu(), rg.cpu()
    for p in range(29):
        a, b = int(oc[p]), int(oc[p + 1])
        g = sorted(zip(hg[a:b].tolist(), lg[a:b].tolist(), rg[a:b].tolist()))
        c = sorted(zip(hc[a:b].tolist(), lc[a:b].tolist(), rc[a:b].tolist()))
        assert g == c, p
    # one partition (no splitters) keeps every record
    h1, _l1, r1, o1 = S.tera_partition(recs_c[:1000].cuda(), shi[:0], slo[:0])
    assert o1.cpu().tolist() == [0, 1000] and sorted(r1.cpu().tolist()) == list(range(1000))


@pytest.mark.gpu
@pytest.mark.parametrize("run", [3, 200])
def test_gpu_sort_keys_orders_ties_on_the_low_word(run):
    """The hi-only sort + tie fix-up: equal high words ordered by the low 16
    bits; a run longer than the fix-up handles takes the full 80-bit sort."""
    n = 100_000
    g = torch.Generator().manual_seed(run)
    hi = torch.randint(0, 1 << 40, (n,), generator=g, dtype=torch.int64)
    hi[: n // 2] = hi[: n // 2] // run * run          # many runs of equal hi
    hi[::997] = hi[0]                                  # one long run
    lo = torch.randint(0, 1 << 16, (n,), generator=g, dtype=torch.int64)
    perm, hs, ls = S.sort_keys(hi.cuda(), lo.cuda())
    pc, hc, lc = S.sort_keys(hi, lo)
    assert torch.equal(hs.cpu(), hc) and torch.equal(ls.cpu(), lc)
    p = perm.cpu().long()
    assert torch.equal(hi[p], hc) and torch.equal(lo[p], lc)
    assert S.count_unsorted(hs, ls) == 0


@pytest.mark.gpu
def test_gpu_terasort_commits_output(tmp_path):
    """TeraSort's output goes through the attempt work dir and the committer:
    parts in the output dir, _SUCCESS, no _temporary left."""
    rows = 1_000_000
    out = tmp_path / "out"
    with LocalCluster(JobConf(), num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        rj = cl.submit_job(T.terasort_conf(rows=rows, split_rows=300_000, partitions=3,
                                           output=str(out)))
        rj.waitForCompletion(300)
        assert rj.isSuccessful(), rj.getFailureInfo()
    assert (out / "_SUCCESS").exists() and not (out / "_temporary").exists()
    v = T.teravalidate(str(out))
    assert v["files"] == 3 and v["records"] == rows and v["misordered"] == 0


def test_merge_runs_cpu_is_stable_and_sorted():
    g = torch.Generator().manual_seed(3)
    runs = []
    for r in range(5):
        h = torch.randint(0, 50, (200 + r,), generator=g, dtype=torch.int64)
        lo = torch.randint(0, 4, (200 + r,), generator=g, dtype=torch.int64)
        o = np.lexsort((lo.numpy(), h.numpy()))
        runs.append((h[o], lo[o], torch.arange(r * 1000, r * 1000 + 200 + r, dtype=torch.int32)))
    hs, ls, vs = S.merge_runs(runs)
    assert S.count_unsorted(hs, ls) == 0 and hs.numel() == sum(r[0].numel() for r in runs)
    # stable: equal keys keep run order (payloads ascend by run)
    key = hs * 8 + ls
    for k in torch.unique(key)[:20]:
        v = vs[key == k]
        assert torch.all(v[1:] // 1000 >= v[:-1] // 1000)


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [(1000, 1), (0, 5000), (33333, 77777, 5, 123456, 9)])
def test_gpu_merge_runs_matches_cpu(sizes):
    g = torch.Generator().manual_seed(sum(sizes))
    runs = []
    base = 0
    for n in sizes:
        h = torch.randint(0, 1 << 20, (n,), generator=g, dtype=torch.int64)
        h[::3] = 7                                          # many equal keys across runs
        lo = torch.randint(0, 1 << 16, (n,), generator=g, dtype=torch.int64)
        lo[::3] = 1
        o = np.lexsort((lo.numpy(), h.numpy())) if n else np.zeros(0, dtype=np.int64)
        runs.append((h[o], lo[o], torch.arange(base, base + n, dtype=torch.int32)))
        base += n
    hc, lc, vc = S.merge_runs(runs)
    hg, lg, vg = S.merge_runs([(a.cuda(), b.cuda(), c.cuda()) for a, b, c in runs])
    assert torch.equal(hg.cpu(), hc) and torch.equal(lg.cpu(), lc) and torch.equal(vg.cpu(), vc)


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("window", [None, "full", "narrow"])
@pytest.mark.parametrize("ties", [0, 5, 100, "prefix"])
def test_gpu_sort_gathered_packed_ids(ties, window, packed):
    """Reduce v4 (hi + packed-id sort, one gather, lo from the gathered records,
    in-place tie fix-up): the records of three map outputs come out in key
    order; ties = equal 8-byte prefixes per run (100: longer than the fix-up
    handles -> None, the caller's full-key path).  window: the group's hi
    bounds given (full range, or every key under one top byte), so the radix
    passes cover only the SORT_BITS below the common prefix and the tie fix-up
    orders the longer equal-prefix runs.  packed: the key alphabet from the
    maps and the group's bounds given, so the packed-key onesweep path runs
    (dense 32-bit window over base-R digits, window ties fixed in place)."""
    parts_c = [torch.from_numpy(S.teragen_cpu(1000 * i, 20_000 + i)) for i in range(3)]
    hi_range = {None: None, "full": (0, (1 << 64) - 1),
                "narrow": (0x5A << 56, (0x5B << 56) - 1)}[window]
    for p in parts_c:
        if window == "narrow":
            p[:, 0] = 0x5A
        if ties == "prefix":
            # runs of 8 keys sharing the sorted 48-bit prefix (bytes 0-5) but
            # not bytes 6-9: the tie fix must order them by the full key
            for k in range(20):
                p[k * 8:(k + 1) * 8, :6] = p[k * 8, :6]
        elif ties == 100:
            p[:100, :8] = p[0, :8]                 # one run longer than the fix-up
        else:
            for k in range(ties):                  # runs of 8 equal high words
                p[k * 8:(k + 1) * 8, :8] = p[k * 8, :8]
    parts = [p.cuda() for p in parts_c]
    outs = [S.tera_partition(p, torch.zeros(0, dtype=torch.int64),
                             torch.zeros(0, dtype=torch.int64), kbytes=True) for p in parts]
    his = [o[0] for o in outs]
    rows = [o[2] for o in outs]
    lens = [p.shape[0] for p in parts]
    kw = {}
    if packed:
        orb = 0
        for o in outs:
            orb |= int(o[4][0])
        assert orb == int(np.bitwise_or.reduce(torch.cat(parts_c)[:, :8].numpy(), axis=None))
        hall = torch.cat(his).cpu().numpy().view(np.uint64)
        bounds = (int(hall.min()), int(hall.max())) if window == "narrow" else (None, None)
        kw = {"alphabet": (0, 1 << orb.bit_length()), "bounds": bounds}
    got = S.sort_gathered(his, rows, [0, 0, 0], lens, parts, hi_range=hi_range, **kw)
    if ties == 100:
        assert got is None
        return
    recs, hs, ls = got
    allr = torch.cat(parts_c).numpy()
    keys = allr[:, :10]
    order = np.lexsort([keys[:, j] for j in range(9, -1, -1)])
    want = allr[order]
    r = recs.cpu().numpy()
    assert np.array_equal(r[:, :10], want[:, :10])
    assert S.count_unsorted(hs, ls) == 0
    # the same multiset of records (equal keys may come in either order)
    assert sorted(map(bytes, r)) == sorted(map(bytes, want))


@pytest.mark.parametrize("budget_rows", [4000, 11000])
def test_terasort_out_of_core_spill_and_merge(tmp_path, budget_rows):
    """Out-of-core TeraSort (MapTask.sortAndSpill / mergeParts): an HBM budget
    below the input size makes every map sort and spill its run to host
    memory (its split not kept) and the reduce merge the runs back in groups
    of partitions sized to the budget; output and order equal the in-memory
    sort's, and TeraValidate passes."""
    rows = 12000
    out = tmp_path / "out"
    conf = T.terasort_conf(rows=rows, split_rows=2500, output=str(out), partitions=10)
    conf.set("hbmr.terasort.hbm.budget.gb", str(budget_rows * 100 / (1 << 30)))
    with LocalCluster(JobConf(), num_trackers=1, cpu_slots=2) as cl:
        rj = cl.submit_job(conf)
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result[0]
        spilled = rj.getCounters().get("org.apache.hadoop.mapred.Task$Counter",
                                       "MAP_SPILLED_RECORDS")
    assert spilled == rows                       # rows * 100 B > budget: spill mode
    assert res["unsorted"] == 0 and res["checksum_ok"] and res["records"] == rows
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert parts == [f"part-{i:05d}" for i in range(10)]
    got = np.concatenate([np.fromfile(out / p, dtype=np.uint8).reshape(-1, 100) for p in parts])
    assert np.array_equal(got, _ref_sorted(rows))
    assert T.teravalidate(str(out))["misordered"] == 0


def test_terasort_spill_mode_on_several_ranks_fails_at_setup(tmp_path):
    """Spill mode merges every map's run on one rank: a job it would put on two
    trackers fails at job setup, before any map runs (it failed
    with a KeyError in the shuffle after every map had run)."""
    conf = T.terasort_conf(rows=12000, split_rows=2500, output=str(tmp_path / "out"),
                           partitions=4)
    conf.set("hbmr.terasort.hbm.budget.gb", str(4000 * 100 / (1 << 30)))
    with LocalCluster(JobConf(), num_trackers=2, cpu_slots=2) as cl:
        rj = cl.submit_job(conf)
        rj.waitForCompletion(60)
        assert not rj.isSuccessful()
        assert "one rank" in (rj.getFailureInfo() or "")
        jip = rj._impl.jip
        assert all(t.successful is None for t in jip.maps)


@pytest.mark.gpu
def test_gpu_terasort_out_of_core(tmp_path):
    """On the GPU: data 3x a deliberately small HBM budget sorts through the
    spill path (pinned host runs, merge-path reduce) and validates."""
    rows = 3_000_000                      # 300 MB of records, budget 100 MB
    out = tmp_path / "out"
    conf = T.terasort_conf(rows=rows, split_rows=400_000, output=str(out), partitions=6)
    conf.set("hbmr.terasort.hbm.budget.gb", str(100e6 / (1 << 30)))
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()      # what earlier tests in this process still hold
    with LocalCluster(JobConf(), num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        rj = cl.submit_job(conf)
        rj.waitForCompletion(300)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result[0]
        cnt = rj.getCounters()
    peak = torch.cuda.max_memory_allocated() - base
    # maps in flight are capped to the budget (one 40 MB split at a time
    # here, its working set ~3.5x), not all 8 allocated at launch (~1.1 GB)
    assert peak == 0 or peak <= 4 * 100e6, peak / 1e6
    assert cnt.get("org.apache.hadoop.mapred.Task$Counter", "MAP_SPILLED_RECORDS") == rows
    assert res["records"] == rows and res["unsorted"] == 0 and res["checksum_ok"]
    v = T.teravalidate(str(out))
    assert v["files"] == 6 and v["records"] == rows and v["misordered"] == 0
    got = np.fromfile(out / "part-00000", dtype=np.uint8).reshape(-1, 100)
    assert np.array_equal(got[:1000], _ref_sorted(rows)[:1000])


@pytest.mark.gpu
@pytest.mark.parametrize("rb", [100, 12, 16, 20, 28, 36, 8, 4])
def test_gpu_record_gather_pieces_match_cpu(rb):
    """The 16-B-piece record gather (7 lanes per 100-B record; other sizes:
    a last piece of 1-3 words) and its key outputs against the CPU gather,
    from several base splits at random rows (record sizes below 12 B take the
    word-per-lane kernel)."""
    g = torch.Generator().manual_seed(rb)
    bases = [torch.randint(0, 256, (n, rb), generator=g, dtype=torch.uint8) for n in (1000, 37, 4099)]
    split = torch.randint(0, 3, (20000,), generator=g)
    row = torch.cat([torch.randint(0, bases[s].shape[0], (1,), generator=g) for s in split.tolist()])
    gid = ((split << 24) | row).to(torch.int32)
    want = S.gather_records_gid(bases, gid)
    keys = None
    if rb >= 12:
        keys = (torch.empty(20000, dtype=torch.int64, device="cuda"),
                torch.empty(20000, dtype=torch.int64, device="cuda"))
    got = S.gather_records_gid([b.cuda() for b in bases], gid.cuda(), keys=keys)
    assert torch.equal(got.cpu(), want)
    if keys is not None:
        h, lo = S.tera_keys(want)
        assert torch.equal(keys[0].cpu(), h) and torch.equal(keys[1].cpu(), lo)
