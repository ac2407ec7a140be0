"""Balancer: evens out DataNode utilisation by moving block replicas.

Behaviour from hadoop-1.0.3/src/hdfs/org/apache/hadoop/hdfs/server/balancer/
Balancer.java: a DataNode is over-utilised when its utilisation (used /
capacity) exceeds the cluster average by more than ``threshold`` percent
(default 10) and under-utilised when it is below by more; each iteration pairs
over- with under-utilised nodes (same rack first), moves up to the smaller
of the source's excess and the target's room (bounded by
``dfs.balance.bandwidthPerSec`` × iteration time in the reference, by
``max_bytes_per_iteration`` here), never onto a node that already holds the
block, waits for the moves, and stops when the cluster is balanced, no block
can be moved, or after ``max_iterations`` (exit statuses SUCCESS /
NO_MOVE_BLOCK / NO_MOVE_PROGRESS of the reference).

Moves go through the NameNode (``move_block``): the source DataNode copies the
replica on its next heartbeat; once the target reports it, the NameNode drops
the source replica and tells the source to delete it.
"""
from __future__ import annotations

import time

SUCCESS, ALREADY_RUNNING, NO_MOVE_BLOCK, NO_MOVE_PROGRESS = 1, -1, -2, -3


def utilisation(nn):
    """{dn: (used_bytes, capacity, rack)} from the NameNode's block map."""
    rep = {d["id"]: d for d in nn.datanode_report() if d["alive"] and not d["decommission"]}
    used = {dn: 0 for dn in rep}
    for dn in rep:
        used[dn] = sum(b["len"] for b in nn.get_blocks(dn))
    total_used = sum(used.values())
    caps = {dn: (rep[dn]["capacity"] or 0) for dn in rep}
    if any(c <= 0 for c in caps.values()):   # unknown capacity: equal shares of the total
        share = max(total_used, 1) * 2
        caps = {dn: share for dn in rep}
    return {dn: (used[dn], caps[dn], rep[dn]["rack"]) for dn in rep}


class Balancer:
    def __init__(self, namenode, threshold=10.0, max_bytes_per_iteration=10 << 30,
                 max_iterations=5, move_timeout_s=30.0):
        self.nn = namenode
        self.threshold = float(threshold)
        self.max_bytes = max_bytes_per_iteration
        self.max_iterations = max_iterations
        self.move_timeout = move_timeout_s
        self.moved_bytes = 0
        self.moved_blocks = 0

    def plan(self):
        u = utilisation(self.nn)
        if not u:
            return [], u
        avg = 100.0 * sum(x[0] for x in u.values()) / max(1, sum(x[1] for x in u.values()))
        util = {dn: 100.0 * x[0] / x[1] for dn, x in u.items()}
        over = {dn: (util[dn] - avg - 0) * u[dn][1] / 100.0 for dn in u
                if util[dn] > avg + self.threshold}
        under = {dn: (avg - util[dn]) * u[dn][1] / 100.0 for dn in u
                 if util[dn] < avg - self.threshold}
        # above-average but within threshold nodes can also give (ref: "aboveAvg") when
        # a target is far below; and below-average ones can take from over-utilised
        if over and not under:
            under = {dn: (avg - util[dn]) * u[dn][1] / 100.0 for dn in u if util[dn] < avg}
        if under and not over:
            over = {dn: (util[dn] - avg) * u[dn][1] / 100.0 for dn in u if util[dn] > avg}
        pairs = []
        for same_rack in (True, False):
            for s in sorted(over, key=lambda d: -over[d]):
                for t in sorted(under, key=lambda d: -under[d]):
                    if (u[s][2] == u[t][2]) != same_rack:
                        continue
                    amt = min(over[s], under[t])
                    if amt <= 0:
                        continue
                    pairs.append((s, t, amt))
                    over[s] -= amt
                    under[t] -= amt
        return pairs, u

    def iterate(self) -> int:
        """One iteration; returns bytes scheduled (0 = nothing to do / possible)."""
        pairs, _ = self.plan()
        budget = self.max_bytes
        scheduled = 0
        for src, dst, amt in pairs:
            left = min(amt, budget - scheduled)
            for b in self.nn.get_blocks(src):
                if left <= 0:
                    break
                if dst in b["locs"] or b["len"] <= 0 or b["len"] > left + b["len"] / 2:
                    continue
                if self.nn.move_block(b["block"], src, dst):
                    left -= b["len"]
                    scheduled += b["len"]
                    self.moved_blocks += 1
            if scheduled >= budget:
                break
        deadline = time.time() + self.move_timeout
        while scheduled and self.nn.pending_moves() and time.time() < deadline:
            time.sleep(0.05)
        self.moved_bytes += scheduled
        return scheduled

    def run(self) -> int:
        for _ in range(self.max_iterations):
            pairs, _ = self.plan()
            if not pairs:
                return SUCCESS   # "The cluster is balanced."
            if self.iterate() == 0:
                return NO_MOVE_BLOCK
        return SUCCESS if not self.plan()[0] else NO_MOVE_PROGRESS
