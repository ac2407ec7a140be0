"""GPU WordCount (split-level job, native/kernels/text.hip): split boundary rule,
word-table primitives against collections.Counter, and job output equal to the
classic WordCount's (TextOutputFormat lines, HashPartitioner partitions)."""
import collections
import os
import random

import pytest
import torch

from hbmr.mapred import JobClient, JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.formats import FileSplit, LineRecordReader
from hbmr.models import wordcount
from hbmr.ops import text


def _corpus(tmp_path, files=3, lines=400, seed=5):
    rnd = random.Random(seed)
    vocab = [f"w{i}" for i in range(300)] + ["Straße", "naïve", "x" * 70, "a", "the"]
    d = tmp_path / "in"
    d.mkdir()
    for f in range(files):
        out = []
        for j in range(lines):
            sep = rnd.choice([" ", "  ", "\t", " \x0b "])
            words = [rnd.choice(vocab) for _ in range(rnd.randint(0, 12))]
            out.append(sep.join(words) + ("\r" if j % 7 == 0 else ""))
        (d / f"part-{f}").write_text("\n".join(out) + ("\n" if f != 1 else ""))
    return d


def _outputs(out):
    return {fn: open(os.path.join(out, fn), "rb").read() for fn in sorted(os.listdir(out))
            if fn.startswith("part-")}


def test_read_text_split_matches_line_record_reader(tmp_path):
    d = _corpus(tmp_path, files=1)
    path = str(d / "part-0")
    size = os.path.getsize(path)
    for split in (1, 7, 100, 1000, size):
        got, want = [], []
        for start in range(0, size, split):
            length = min(split, size - start)
            got.append(wordcount.read_text_split(path, start, length))
            rr = LineRecordReader(JobConf(), FileSplit(path, start, length))
            lines = []
            while True:
                kv = rr.next()
                if kv is None:
                    break
                lines.append(kv[1].bytes)
            want.append(lines)
        for g, w in zip(got, want):
            assert [ln.rstrip(b"\r") for ln in g.split(b"\n")[:len(w)]] == w


def test_cpu_word_tables():
    data = b"a b  a\tc\nd a \x0b b\r\n"
    blob, counts = text.count_words_cpu(data)
    assert dict(text.parse_table(bytes(blob.numpy()), counts)) == \
        dict(collections.Counter(data.split()))
    mb, mc, pb, pw = text.merge_tables_cpu(bytes(blob.numpy()) * 2, torch.cat([counts, counts]), 3)
    assert sum(pw) == 4 and sum(pb) == mb.numel()
    assert dict(text.parse_table(bytes(mb.numpy()), mc)) == {b"a": 6, b"b": 4, b"c": 2, b"d": 2}


@pytest.mark.parametrize("trackers", [1, 2])
def test_split_job_output_equals_classic_wordcount(tmp_path, trackers):
    inp = _corpus(tmp_path)
    conf = JobConf()
    with LocalCluster(conf, num_trackers=trackers, cpu_slots=2) as cl:
        classic = wordcount.make_job(str(inp), str(tmp_path / "classic"), reduces=trackers)
        classic.set_num_map_tasks(5)
        JobClient.runJob(classic, cluster=cl, verbose=False)
        job = wordcount.gpu_job(str(inp), str(tmp_path / "split"), maps=5)
        rj = cl.submit_job(job)
        assert rj.waitForCompletion(60) and rj.isSuccessful(), rj.getFailureInfo()
    assert _outputs(tmp_path / "split") == _outputs(tmp_path / "classic")
    assert os.path.exists(tmp_path / "split" / "_SUCCESS")


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_count_words_exact():
    rnd = random.Random(1)
    words = [bytes(rnd.choice(b"abcdefghij") for _ in range(rnd.randint(1, 9)))
             for _ in range(200_000)]
    words += [b"\xc3\xa9t\xc3\xa9", b"z" * 300]
    seps = [b" ", b"\t", b"\n", b"  ", b"\r\n", b"\x0b", b"\x0c"]
    data = b"".join(w + rnd.choice(seps) for w in words)
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    blob, counts = text.count_words(buf)
    got = dict(text.parse_table(bytes(blob.cpu().numpy()), counts.cpu()))
    assert got == dict(collections.Counter(data.split()))
    # merge two copies into 4 partitions: counts double, partitions = HashPartitioner
    mb, mc, pb, pw = text.merge_tables(torch.cat([blob, blob]), torch.cat([counts, counts]), 4)
    items = text.parse_table(bytes(mb.cpu().numpy()), mc.cpu())
    assert dict(items) == {w: 2 * n for w, n in got.items()}
    i = 0
    for p, nw in enumerate(pw):
        assert all(text.partition_of(w, 4) == p for w, _ in items[i:i + nw])
        i += nw
    assert sum(pb) == mb.numel()


@pytest.mark.gpu
def test_gpu_count_words_table_growth(monkeypatch):
    """More distinct words than the first table holds: overflow → retry larger."""
    monkeypatch.setattr(text, "INITIAL_TABLE", 1024)
    words = [b"u%d" % i for i in range(50_000)] * 2
    data = b" ".join(words)
    blob, counts = text.count_words(torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda())
    got = dict(text.parse_table(bytes(blob.cpu().numpy()), counts.cpu()))
    assert len(got) == 50_000 and set(got.values()) == {2}


@pytest.mark.gpu
def test_gpu_count_words_hot_words():
    """Zipf head: a few words are most of the text (LDS pre-aggregation path)."""
    rnd = random.Random(2)
    data = b" ".join(rnd.choice([b"the"] * 90 + [b"of"] * 9 + [b"w%d" % rnd.randint(0, 5000)])
                     for _ in range(300_000)) + b"\n"
    blob, counts = text.count_words(torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda())
    got = dict(text.parse_table(bytes(blob.cpu().numpy()), counts.cpu()))
    assert got == dict(collections.Counter(data.split()))


@pytest.mark.gpu
def test_gpu_count_words_empty_and_unaligned():
    buf = torch.frombuffer(bytearray(b"  x yy x "), dtype=torch.uint8).cuda()
    blob, counts = text.count_words(buf[1:])        # misaligned view
    assert dict(text.parse_table(bytes(blob.cpu().numpy()), counts.cpu())) == {b"x": 2, b"yy": 1}
    blob, counts = text.count_words(torch.empty(0, dtype=torch.uint8, device="cuda"))
    assert blob.numel() == 0 and counts.numel() == 0


@pytest.mark.gpu
def test_gpu_wordcount_job_equals_classic(tmp_path):
    inp = _corpus(tmp_path, files=4, lines=3000)
    conf = JobConf()
    conf.set_int("mapred.tasktracker.map.cpu.tasks.maximum", 0)
    with LocalCluster(conf, num_trackers=1, gpus=[[0]], cpu_slots=0) as cl:
        job = wordcount.gpu_job(str(inp), str(tmp_path / "split"), maps=6)
        rj = cl.submit_job(job)
        assert rj.waitForCompletion(120) and rj.isSuccessful(), rj.getFailureInfo()
        cs = rj.getCounters()
    assert cs.get("org.apache.hadoop.mapred.JobInProgress$Counter", "GPU_MAP_TASKS") >= 6
    classic = wordcount.make_job(str(inp), str(tmp_path / "classic"), reduces=1)
    classic.set("mapred.job.tracker", "local")
    JobClient.runJob(classic, verbose=False)
    assert _outputs(tmp_path / "split") == _outputs(tmp_path / "classic")


def test_native_cpu_tokeniser_matches_bytes_split():
    """The native map runner's tokeniser (native/cpu/wordcount.cc: 64-byte
    AVX2 whitespace masks, masked 16-byte word prefixes, newline count) gives
    Python's bytes.split() counts on random text: every whitespace kind, words
    longer than 16 bytes and across 64-byte chunks, leading/trailing blanks."""
    import collections
    import ctypes
    import random

    import numpy as np

    from hbmr.models.wordcount import _wc_lib
    lib = _wc_lib()
    if lib is None:
        pytest.skip("libhbmr_cpu not built")
    rnd = random.Random(5)
    for trial in range(80):
        toks = [rnd.choice(["a", "bb", "xyz" * rnd.randint(1, 12), "q" * rnd.randint(1, 70),
                            "été"]) for _ in range(rnd.randint(0, 400))]
        seps = [rnd.choice([" ", "\t", "\n", "  ", "\r\n", "\x0b", "\x0c"]) for _ in toks]
        text = "".join(a + b for a, b in zip(toks, seps)).encode()
        if trial % 3 == 0:
            text = text.rstrip()
        if trial % 5 == 0:
            text = b"  " + text
        h = lib.hbmr_wc_cpu_new()
        try:
            lib.hbmr_wc_cpu_add(h, text, len(text))
            assert lib.hbmr_wc_cpu_newlines(h) == text.count(b"\n")
            w, nb = lib.hbmr_wc_cpu_words(h), lib.hbmr_wc_cpu_bytes(h)
            words = ctypes.create_string_buffer(max(1, nb))
            offs = np.empty(w + 1, np.int64)
            cnts = np.empty(w, np.int64)
            lib.hbmr_wc_cpu_export(h, words, offs.ctypes.data, cnts.ctypes.data)
        finally:
            lib.hbmr_wc_cpu_free(h)
        raw = words.raw[:nb]
        got = {raw[offs[j]:offs[j + 1]]: int(cnts[j]) for j in range(w)}
        assert got == dict(collections.Counter(text.split())), trial
