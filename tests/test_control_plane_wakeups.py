"""No lost wake-ups in the staged-job chain: trackers that long-poll (parked
until their bell rings) at random relative speeds must each receive every
staged job's plan without a long-poll timeout.  A tracker that ran its share of
the chain ahead of the others has no report coming; staging a job behind a
staged job rings it — counting only attempts it was actually sent as its work
(the plan's own attempts sit in its running set before delivery: a ring
decided on ``running`` alone never came, and the job waited out the 200 ms
long-poll; 8-rank rehearsal, profiles/r05_control_plane_rehearsal.json).
Since round 6 a job staged behind a RUNNING one rings only such idle
trackers too (ahead=1 stages every job that way); busy ones get the plan
with their next report."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools"))


@pytest.mark.parametrize("ahead", [1, 2, 3])
@pytest.mark.parametrize("seed", [0, 3, 7])
def test_parked_trackers_get_every_staged_plan(ahead, seed):
    import jt_microbench as M
    h = M.Harness(8, ahead=ahead, points=12_800_000, split_points=100_000)
    h.park = True
    h.rng = random.Random(seed)
    h.speed = [h.rng.choice([1.0, 0.5, 0.2]) for _ in range(8)]
    r = h.run(16, warmup=4)        # raises RuntimeError("no progress") on a lost wake-up
    assert r["jobs"] == 16
