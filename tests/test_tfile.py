"""TFile container (io/file/tfile; TestTFile*.java): sorted appends, block
index seeks (seekTo / lowerBound / upperBound), range scanners, meta blocks,
compression, unsorted files."""
from __future__ import annotations

import random

import pytest

from hbmr.io import tfile


def _kv(n, seed=0):
    rng = random.Random(seed)
    keys = sorted({rng.randbytes(rng.randrange(1, 12)) for _ in range(n)})
    return [(k, rng.randbytes(rng.randrange(0, 300))) for k in keys]


@pytest.mark.parametrize("comp", ["none", "gz"])
def test_sorted_tfile_roundtrip_and_seeks(tmp_path, comp):
    recs = _kv(5000)
    p = str(tmp_path / "t.tfile")
    with tfile.Writer(p, min_block_size=4096, compression=comp) as w:
        for k, v in recs:
            w.append(k, v)
        w.prepare_meta_block("user.meta", b"hello")
    with tfile.Reader(p) as r:
        assert r.is_sorted() and r.get_entry_count() == len(recs)
        assert len(r.index) > 10
        assert list(r.create_scanner()) == recs
        assert r.get_first_key() == recs[0][0] and r.get_last_key() == recs[-1][0]
        assert r.get_meta_block("user.meta") == b"hello"
        keys = [k for k, _ in recs]
        s = r.create_scanner()
        for i in (0, 1, 777, 2500, len(recs) - 1):
            assert s.seek_to(keys[i]) and s.entry() == recs[i]
            s.upper_bound(keys[i])
            assert (s.entry() == recs[i + 1]) if i + 1 < len(recs) else s.at_end()
        missing = keys[100] + b"\x00"
        assert not s.seek_to(missing)
        s.lower_bound(missing)
        assert s.entry() == recs[101]
        lo, hi = keys[1000], keys[3000]
        assert list(r.create_scanner(lo, hi)) == recs[1000:3000]


def test_sorted_writer_rejects_out_of_order_and_reserved_meta(tmp_path):
    w = tfile.Writer(str(tmp_path / "x"), comparator="memcmp")
    w.append(b"b", b"1")
    with pytest.raises(ValueError):
        w.append(b"a", b"2")
    with pytest.raises(ValueError):
        w.prepare_meta_block("TFile.index", b"")
    w.close()


def test_unsorted_tfile(tmp_path):
    p = str(tmp_path / "u")
    recs = [(b"z", b"1"), (b"a", b"2"), (b"m", b"")]
    with tfile.Writer(p, comparator=None) as w:
        for k, v in recs:
            w.append(k, v)
    with tfile.Reader(p) as r:
        assert not r.is_sorted() and list(r.create_scanner()) == recs
        with pytest.raises(ValueError):
            r.create_scanner(b"a")


def test_not_a_tfile(tmp_path):
    p = tmp_path / "bad"
    p.write_bytes(b"x" * 100)
    with pytest.raises(IOError):
        tfile.Reader(str(p))
