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


def _shared_device_batches(jobs, tasks, per_task_ms, batch, streams=2):
    """Batches of ``batch`` tasks alternating over ``streams`` slot streams of
    one device that shares its throughput among the streams with work
    (processor sharing): every batch's [start, end) on the device clock, in
    completion order, tagged with its job."""
    queues = [[] for _ in range(streams)]
    k = 0
    for j in range(jobs):
        for b in range(tasks // batch):
            queues[k % streams].append((f"job{j}", batch * per_task_ms))
            k += 1
    t, heads, out = 0.0, [0] * streams, []
    left = [q[0][1] if q else 0.0 for q in queues]
    start = [0.0] * streams
    while any(h < len(q) for h, q in zip(heads, queues)):
        act = [s for s in range(streams) if heads[s] < len(queues[s])]
        rate = 1.0 / len(act)
        dt = min(left[s] for s in act) / rate
        t += dt
        for s in act:
            left[s] -= dt * rate
        for s in act:
            if left[s] <= 1e-12:
                out.append((queues[s][heads[s]][0], start[s], t))
                heads[s] += 1
                start[s] = t
                if heads[s] < len(queues[s]):
                    left[s] = queues[s][heads[s]][1]
    return out


def test_cost_model_gpu_estimate_matches_device_time_per_split():
    """two overlapping slot streams (the bench's 2 GPU slots),
    128-split jobs at 0.245 ms of device time per split (rocprof busy / split
    of the round-5 bench): the estimate the scheduler reads is within ±10 %
    of the device time per split at every job end and within ±25 % mid-job;
    the per-task-window decay it replaces read the job's cheap tail."""
    from hbmr.mapred.scheduler.costmodel import CostModel
    per = 0.245
    for batch in (16, 8):
        tl, cm, old = BusyTimeline(), CostModel(alpha=0.3), CostModel(alpha=0.3)
        done = 0
        errs_end, errs_old = [], []
        for i, (job, s, e) in enumerate(_shared_device_batches(6, 128, per, batch)):
            ids = [f"{job}_{i}_{t}" for t in range(batch)]
            dt_each = tl.charge(s, e) / 1000.0 / batch
            for m in (cm, old):
                m.tasks_started("km", ids, True, 0.0)
            cm.tasks_finished("km", ids, True, dt_each, job=job)
            old.tasks_finished("km", ids, True, dt_each)
            done += batch
            est = cm.stats("km", True).estimate(0.0)[0] * 1000.0
            if done % 128 == 0:
                errs_end.append(abs(est - per) / per)
                errs_old.append(abs(old.stats("km", True).estimate(0.0)[0] * 1000.0 - per) / per)
            elif done > 128:
                assert abs(est - per) < 0.25 * per, (batch, done, est)
        assert abs(tl.total - 6 * 128 * per) < 1e-6
        assert max(errs_end) < 0.10, (batch, errs_end)
        assert max(errs_end) < max(errs_old), (errs_end, errs_old)


def test_cpu_probe_estimate_stays_censored_while_gpu_batches_finish():
    """A sampled CPU probe (1 % of a split) that is still running bounds the
    CPU time from below by its age / fraction; GPU batches finishing around it
    do not turn that bound into a mean, and a killed probe keeps it."""
    from hbmr.mapred.scheduler.costmodel import CostModel
    cm = CostModel()
    cm.task_started("km", "probe", False, 100.0, fraction=0.01)
    assert cm.is_probe("km", "probe", False)
    for i in range(4):
        ids = [f"g{i}_{t}" for t in range(16)]
        cm.tasks_started("km", ids, True, 100.0)
        cm.tasks_finished("km", ids, True, 0.000245, job="job0")
    est, lb = cm.stats("km", False).estimate(100.5)
    assert lb and abs(est - 50.0) < 1e-9           # 0.5 s on 1 % of a split
    acc, acc_lb = cm.acceleration("km", 100.5)
    assert acc_lb and abs(acc - 50.0 / 0.000245) < 1e-3 * acc
    assert cm.stats("km", False).n == 0 and cm.stats("km", False).mean == 0.0
    cm.task_finished("km", "probe", False, 100.0, 101.0, succeeded=False)
    est, lb = cm.stats("km", False).estimate(200.0)
    assert lb and abs(est - 100.0) < 1e-9           # killed after 1 s → ≥ 100 s per split
