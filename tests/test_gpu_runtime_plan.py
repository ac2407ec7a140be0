"""Launch planning of the GPU runtime (hbmr/gpu/runtime.py) that needs no
device: batch sizes of pre-staged vs unstaged jobs and the tapered chunks of
a job's last batches."""
from types import SimpleNamespace

from hbmr.gpu.runtime import GpuRuntime


def _runs(n, wait=None):
    return [SimpleNamespace(wait=wait) for _ in range(n)]


def test_batch_target_staged_vs_unstaged():
    # maps released behind a gate event: the staged target
    assert GpuRuntime._batch_target(_runs(8, wait=object()), 16, 32) == 16
    # nothing to wait for (the first job of a chain): the larger target
    assert GpuRuntime._batch_target(_runs(8), 16, 32) == 32
    # one gated run makes the batch a staged one
    mixed = _runs(3) + _runs(1, wait=object())
    assert GpuRuntime._batch_target(mixed, 16, 32) == 16


def test_chunks_cover_every_run_once():
    for n in (1, 4, 17, 124, 128):
        for per in (4, 16, 32):
            for taper in (False, True):
                ch = GpuRuntime._chunks(0, n, per, taper)
                covered = [j for s, c in ch for j in range(s, s + c)]
                assert covered == list(range(n)), (n, per, taper)
                assert all(0 < c <= per for _, c in ch)


def test_chunks_taper_halves_the_tail():
    # 124 runs after a first chunk of 4: full batches while more than 2 x per
    # runs remain, then halving batches (the last <= 4 go together)
    sizes = [c for _, c in GpuRuntime._chunks(4, 128, 16, True)]
    assert sizes == [16] * 6 + [14, 7, 4, 3]
    assert [c for _, c in GpuRuntime._chunks(4, 128, 16, False)] == [16] * 7 + [12]
