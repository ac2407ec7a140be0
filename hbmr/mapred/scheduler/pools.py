"""Fair-scheduler allocation file (contrib/fairscheduler PoolManager.java:57-400).

``mapred.fairscheduler.allocation.file`` (else ``fair-scheduler.xml`` on the
configuration path) holds::

    <allocations>
      <pool name="research">
        <minMaps>4</minMaps> <minReduces>2</minReduces> <minGpuMaps>1</minGpuMaps>
        <maxMaps>20</maxMaps> <maxReduces>8</maxReduces> <maxGpuMaps>4</maxGpuMaps>
        <maxRunningJobs>3</maxRunningJobs> <weight>2.0</weight>
        <minSharePreemptionTimeout>60</minSharePreemptionTimeout>
        <schedulingMode>fifo</schedulingMode>
      </pool>
      <user name="bob"><maxRunningJobs>2</maxRunningJobs></user>
      <userMaxJobsDefault>5</userMaxJobsDefault>
      <poolMaxJobsDefault>10</poolMaxJobsDefault>
      <fairSharePreemptionTimeout>600</fairSharePreemptionTimeout>
      <defaultMinSharePreemptionTimeout>60</defaultMinSharePreemptionTimeout>
      <defaultPoolSchedulingMode>fair</defaultPoolSchedulingMode>
    </allocations>

(``minGpuMaps`` / ``maxGpuMaps`` are hbmr's GPU-slot additions; times are
seconds.)  The file is re-read when it changed, checked at most every
``mapred.fairscheduler.allocation.reload.interval`` seconds (10) and only once
the change is ``…reload.wait`` seconds old (5), so a half-written file is not
picked up; a bad file keeps the previous allocations.  Values not in the file
fall back to hbmr's ``hbmr.fair.pool.<pool>.<key>`` configuration keys."""
from __future__ import annotations

import logging
import os
import time
import xml.etree.ElementTree as ET

log = logging.getLogger("hbmr.scheduler.fair")

INF = 1 << 62
_INT_FIELDS = {"minMaps", "minReduces", "minGpuMaps", "maxMaps", "maxReduces", "maxGpuMaps",
               "maxRunningJobs"}


class AllocationConfigurationException(ValueError):
    pass


def _text(el):
    return (el.text or "").strip()


def _mode(s):
    s = s.lower()
    if s not in ("fair", "fifo"):
        raise AllocationConfigurationException(
            f"Unknown scheduling mode : {s}; expected 'fifo' or 'fair'")
    return s


class Allocations:
    """One parsed allocation file."""

    def __init__(self):
        self.pools: dict[str, dict] = {}      # pool -> {field: value}
        self.user_max_jobs: dict[str, int] = {}
        self.user_max_jobs_default = INF
        self.pool_max_jobs_default = INF
        self.fair_share_timeout = None        # seconds, or None (not in the file)
        self.default_min_share_timeout = None
        self.default_mode = "fair"

    @classmethod
    def parse(cls, path) -> "Allocations":
        a = cls()
        root = ET.parse(path).getroot()
        if root.tag != "allocations":
            raise AllocationConfigurationException(
                "Bad fair scheduler config file: top-level element not <allocations>")
        for el in root:
            if not isinstance(el.tag, str):
                continue
            if el.tag == "pool":
                name = el.get("name")
                p = a.pools.setdefault(name, {})
                for f in el:
                    if f.tag in _INT_FIELDS:
                        p[f.tag] = int(_text(f))
                    elif f.tag == "weight":
                        p["weight"] = float(_text(f))
                    elif f.tag == "minSharePreemptionTimeout":
                        p["minSharePreemptionTimeout"] = float(_text(f))
                    elif f.tag == "schedulingMode":
                        p["mode"] = _mode(_text(f))
                    else:
                        log.warning("Bad element in pool %s: %s", name, f.tag)
                for kind in ("Maps", "Reduces", "GpuMaps"):
                    if p.get("max" + kind, INF) < p.get("min" + kind, 0):
                        log.warning("Pool %s has max %s %d less than min %s %d", name, kind,
                                    p["max" + kind], kind, p["min" + kind])
            elif el.tag == "user":
                for f in el:
                    if f.tag == "maxRunningJobs":
                        a.user_max_jobs[el.get("name")] = int(_text(f))
            elif el.tag == "userMaxJobsDefault":
                a.user_max_jobs_default = int(_text(el))
            elif el.tag == "poolMaxJobsDefault":
                a.pool_max_jobs_default = int(_text(el))
            elif el.tag == "fairSharePreemptionTimeout":
                a.fair_share_timeout = float(_text(el))
            elif el.tag == "defaultMinSharePreemptionTimeout":
                a.default_min_share_timeout = float(_text(el))
            elif el.tag == "defaultPoolSchedulingMode":
                a.default_mode = _mode(_text(el))
            else:
                log.warning("Bad element in allocations file: %s", el.tag)
        return a


class PoolManager:
    def __init__(self, conf):
        self.conf = conf
        self.alloc_file = conf.get("mapred.fairscheduler.allocation.file") or \
            _on_conf_path("fair-scheduler.xml")
        self.reload_interval = conf.get_float("mapred.fairscheduler.allocation.reload.interval",
                                              10.0)
        self.reload_wait = conf.get_float("mapred.fairscheduler.allocation.reload.wait", 5.0)
        self.allocs = Allocations()
        self.reloads = 0
        self._last_attempt = self._last_ok = time.time()
        self._failed = False
        if self.alloc_file:
            self.reload()

    def reload(self):
        self.allocs = Allocations.parse(self.alloc_file)
        self.reloads += 1

    def reload_if_necessary(self, now=None):
        """PoolManager.reloadAllocsIfNecessary."""
        now = time.time() if now is None else now
        if not self.alloc_file or now <= self._last_attempt + self.reload_interval:
            return
        self._last_attempt = now
        try:
            mtime = os.path.getmtime(self.alloc_file)
            if mtime > self._last_ok and now > mtime + self.reload_wait:
                self.reload()
                self._last_ok = now
                self._failed = False
        except Exception as e:  # noqa: BLE001 (keep the previous allocations)
            if not self._failed:
                log.error("Failed to reload fair scheduler config file - will use existing "
                          "allocations: %s", e)
            self._failed = True

    # -- lookups (file first, then hbmr.fair.pool.<p>.<key>) ------------------------------
    def pool_value(self, pool, key, default):
        v = self.allocs.pools.get(pool, {}).get(key)
        if v is not None:
            return v
        if key == "mode" and pool in self.allocs.pools:
            return self.allocs.default_mode
        if key == "minSharePreemptionTimeout" and self.allocs.default_min_share_timeout is not None:
            c = self.conf.get(f"hbmr.fair.pool.{pool}.{key}")
            return float(c) if c is not None else self.allocs.default_min_share_timeout
        c = self.conf.get(f"hbmr.fair.pool.{pool}.{key}")
        if c is None:
            return self.allocs.default_mode if key == "mode" else default
        return type(default)(c) if not isinstance(default, str) else c

    def pool_max_jobs(self, pool) -> int:
        return int(self.pool_value(pool, "maxRunningJobs", self.allocs.pool_max_jobs_default))

    def user_max_jobs(self, user) -> int:
        return self.allocs.user_max_jobs.get(user, self.allocs.user_max_jobs_default)

    def fair_share_timeout(self, default):
        t = self.allocs.fair_share_timeout
        return default if t is None else t

    def pool_names(self):
        return sorted(self.allocs.pools)


def _on_conf_path(name):
    from ...conf.configuration import _conf_dir
    d = _conf_dir()
    if d is not None and (d / name).exists():
        return str(d / name)
    return None
