"""Device busy-time accounting of GPU map batches (hbmr/gpu/busy.py): the
charges of overlapping batches sum to the union of their intervals in any
reporting order, and a staged batch is not charged the time its stream
waited for its gate — the GPU task time the cost model learns (the
reference's map-time estimate, JobInProgress.java:527-565)."""
import itertools
import random

from hbmr.gpu.busy import BusyTimeline, batch_interval


def _union(iv):
    tot, cur_s, cur_e = 0.0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0.0)


def test_two_streams_overlapping_batches_are_charged_once():
    # slot A: [0, 10), [10, 20); slot B: [2, 12), [12, 22) (the device runs
    # both streams at once: busy 0..22, not 40 and not 2 x 20 / 2 floors)
    iv = [(0, 10), (2, 12), (10, 20), (12, 22)]
    for order in itertools.permutations(iv):
        tl = BusyTimeline()
        got = sum(tl.charge(s, e) for s, e in order)
        assert abs(got - 22.0) < 1e-9, order
        assert abs(tl.total - 22.0) < 1e-9


def test_random_intervals_sum_to_the_union():
    rng = random.Random(5)
    for _ in range(200):
        iv = []
        for _ in range(rng.randint(1, 30)):
            s = rng.uniform(0, 100)
            iv.append((s, s + rng.uniform(0, 15)))
        tl = BusyTimeline()
        order = iv[:]
        rng.shuffle(order)
        got = sum(tl.charge(s, e) for s, e in order)
        assert abs(got - _union(iv)) < 1e-6


def test_gate_wait_is_not_charged():
    # a staged batch whose start event fired at t=0 but whose gate (the
    # previous job's reduce result) fired at t=7: its kernels ran 7..10
    start, end = batch_interval(0.0, 10.0, gate_ms=[7.0])
    assert (start, end) == (7.0, 10.0)
    tl = BusyTimeline()
    assert tl.charge(start, end) == 3.0
    # gates that fired before the batch's own start do not move it
    assert batch_interval(5.0, 2.0, gate_ms=[1.0, 3.0]) == (5.0, 7.0)
    # a gate after the batch's end (clock skew): a zero-length charge
    assert batch_interval(0.0, 1.0, gate_ms=[4.0]) == (1.0, 1.0)


def test_old_intervals_are_pruned_but_charges_stay_exact_in_order():
    tl = BusyTimeline(keep=8)
    total = 0.0
    for k in range(1000):
        total += tl.charge(2 * k, 2 * k + 1)
    assert total == 1000.0 and len(tl._starts) <= 8


def test_cost_model_estimate_averages_the_slot_streams_batches():
    """Two slot streams' batches get alternately most and little of the device
    time (the union charges each its uncovered part): the estimate must follow
    the device's throughput per task, not the last batch's share (a per-task
    EWMA stepped once per task of a batch did)."""
    from hbmr.mapred.scheduler.costmodel import CostModel
    cm = CostModel(alpha=0.3)
    for i in range(20):
        big = i % 2 == 0
        ids = [f"b{i}_{j}" for j in range(16)]
        cm.tasks_started("s", ids, True, 0.0)
        cm.tasks_finished("s", ids, True, (0.0076 if big else 0.0004) / 16)
    est, lb = cm.stats("s", True).estimate(0.0)
    assert not lb
    per_task = (0.0076 + 0.0004) / 32
    assert abs(est - per_task) < 0.25 * per_task, (est, per_task)
