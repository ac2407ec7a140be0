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


@pytest.mark.parametrize("trackers", [1, 2, 3])
def test_terasort_on_cluster_sorts_and_validates(tmp_path, trackers):
    rows = 20000
    out = tmp_path / "out"
    with LocalCluster(JobConf(), num_trackers=trackers, cpu_slots=2) as cl:
        rj = cl.submit_job(T.terasort_conf(rows=rows, split_rows=3000, output=str(out)))
        rj.waitForCompletion(120)
        assert rj.isSuccessful(), rj.getFailureInfo()
        res = rj._impl.jip.result
    assert all(r["unsorted"] == 0 and r["checksum_ok"] for r in res.values())
    assert sum(r["records"] for r in res.values()) == rows
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert len(parts) == trackers
    got = np.concatenate([np.fromfile(out / p, dtype=np.uint8).reshape(-1, 100) for p in parts])
    assert np.array_equal(got, _ref_sorted(rows))


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
