"""HBM-resident split cache.

Each tracker keeps the splits its GPU tasks materialised, keyed by
(split key, device), so later jobs over the same input (every K-Means
iteration) find their data already in HBM — "locality" for the scheduler means
*resident in this GPU's HBM* (SURVEY.md §7 "HBM-resident split sizing").
Capacity is bounded by ``hbmr.gpu.hbm.reserve.gb`` below the device's free
memory (or set outright by ``hbmr.gpu.split.cache.bytes``); eviction is LRU,
or with ``hbmr.gpu.split.cache.policy=scan`` a full cache keeps its resident
splits and streams the rest through (iterative jobs over more data than HBM:
LRU would miss on every split of every iteration, scan hits on the resident
fraction).  The tracker reports additions/evictions in its next
heartbeat so the JobTracker's locality view stays current.
"""
from __future__ import annotations

import collections
import threading


class SplitCache:
    def __init__(self, capacity_bytes_per_device: dict | None = None, policy: str = "lru"):
        if policy not in ("lru", "scan"):
            raise ValueError(f"split cache policy must be lru or scan, not {policy!r}")
        self.policy = policy
        self._lock = threading.Lock()
        self._entries: "collections.OrderedDict[tuple, tuple]" = collections.OrderedDict()
        self._bytes = collections.Counter()
        self.capacity = dict(capacity_bytes_per_device or {})
        self.added: list = []
        self.removed: list = []
        self.hits = 0
        self.misses = 0
        self.bypassed = 0       # splits streamed through without being cached (scan policy)
        # eviction listeners fn(key, device): device state derived from a
        # split (e.g. the K-Means delta combiner's reference partitions)
        # goes with it; charge() counts that state against the capacity
        self._listeners: list = []

    def add_listener(self, fn):
        with self._lock:
            if fn not in self._listeners:
                self._listeners.append(fn)

    def charge(self, key, device, nbytes: int) -> bool:
        """Count ``nbytes`` of device memory that belongs to the resident split
        (key, device) against the cache capacity (evicting other splits if
        that overfills it).  False if the split is not resident."""
        evicted = []
        with self._lock:
            k = (key, device)
            e = self._entries.get(k)
            if e is None:
                return False
            self._entries[k] = (e[0], e[1] + int(nbytes))
            self._bytes[device] += int(nbytes)
            cap = self.capacity.get(device)
            if cap is not None:
                while self._bytes[device] > cap:
                    victim = next((kk for kk in self._entries
                                   if kk[1] == device and kk != k), None)
                    if victim is None:
                        break
                    _, vb = self._entries.pop(victim)
                    self._bytes[device] -= vb
                    self.removed.append(list(victim))
                    evicted.append(victim)
            listeners = list(self._listeners)
        for vk, vd in evicted:
            for fn in listeners:
                fn(vk, vd)
        return True

    def get(self, key, device):
        with self._lock:
            k = (key, device)
            e = self._entries.get(k)
            if e is not None:
                self._entries.move_to_end(k)
                self.hits += 1
                return e[0]
            self.misses += 1
            return None

    def put(self, key, device, data, nbytes: int):
        with self._lock:
            k = (key, device)
            if k in self._entries:
                return
            cap = self.capacity.get(device)
            if cap is not None and self.policy == "scan" and \
                    self._bytes[device] + nbytes > cap:
                # scan-resistant: a data set larger than HBM is read in the same
                # split order every iteration, where LRU would evict each split
                # just before its next use (no hits at all); instead the
                # resident set stays and the overflow streams through
                self.bypassed += 1
                return
            evicted = []
            if cap is not None:
                while self._bytes[device] + nbytes > cap:
                    victim = next((kk for kk in self._entries if kk[1] == device), None)
                    if victim is None:
                        break
                    _, vb = self._entries.pop(victim)
                    self._bytes[device] -= vb
                    self.removed.append(list(victim))
                    evicted.append(victim)
            self._entries[k] = (data, nbytes)
            self._bytes[device] += nbytes
            self.added.append([key, device])
            listeners = list(self._listeners) if evicted else ()
        for vk, vd in evicted:
            for fn in listeners:
                fn(vk, vd)

    def get_or_load(self, key, device, loader, nbytes_fn, cache=True):
        """``cache=False``: the split job streams its inputs (e.g. an
        out-of-core TeraSort): a resident copy is used, a loaded one is not
        kept."""
        data = self.get(key, device)
        if data is not None:
            return data, True
        data = loader()
        if cache:
            self.put(key, device, data, nbytes_fn(data))
        else:
            with self._lock:
                self.bypassed += 1
        return data, False

    def drain_changes(self):
        with self._lock:
            a, r = self.added, self.removed
            self.added, self.removed = [], []
            return a, r

    def readvertise(self):
        """After re-registering with a (restarted) JobTracker: report every
        resident split as newly added."""
        with self._lock:
            self.added = [list(k) for k in self._entries]
            self.removed = []

    def resident(self):
        with self._lock:
            return [list(k) for k in self._entries]

    def bytes_on(self, device):
        return self._bytes[device]

    def clear(self, device=None):
        gone = []
        with self._lock:
            for k in list(self._entries):
                if device is None or k[1] == device:
                    _, b = self._entries.pop(k)
                    self._bytes[k[1]] -= b
                    self.removed.append(list(k))
                    gone.append(k)
            listeners = list(self._listeners)
        for vk, vd in gone:
            for fn in listeners:
                fn(vk, vd)


def configure(tracker):
    """Apply the tracker's split-cache keys (capacity override, policy)."""
    conf = tracker.conf
    cache = tracker.split_cache
    cap = conf.get_long("hbmr.gpu.split.cache.bytes", 0)
    if cap > 0:
        for d in list(cache.capacity) or [0]:
            cache.capacity[d] = cap
    policy = conf.get("hbmr.gpu.split.cache.policy", "lru")
    if policy not in ("lru", "scan"):
        raise ValueError(f"hbmr.gpu.split.cache.policy must be lru or scan, not {policy!r}")
    cache.policy = policy
