"""Failmon: hardware / log failure monitoring for the node (contrib/failmon).

Behaviour from hadoop-1.0.3/src/contrib/failmon/src/java/org/apache/hadoop/contrib/failmon/:
parsers that turn machine state into ``EventRecord``s (hostname, timestamp,
type, log level, source, properties) — CPUParser (/proc/cpuinfo, load),
NICParser (interface error/drop counters), SensorsParser (temperatures),
SMARTParser (disk health via smartctl), HadoopLogParser / SystemLogParser
(WARN/ERROR/FATAL lines of daemon logs and syslog) — run once (RunOnce) or
periodically (Continuous, ``monitor.interval``), persisted by LocalStore
(here JSON lines) with an Anonymizer that hashes host names and IP
addresses before upload.

MI355X-first: the most failure-relevant component of a GPU node is the GPU,
so a ``GPUParser`` reads the amdgpu sysfs of every card: temperatures (edge,
junction, HBM), power, VRAM use, busy %, and the RAS error counters
(UMC = HBM ECC, GFX, SDMA, XGMI/WAFL link errors); a nonzero uncorrectable
count is logged at ERROR, correctable counts at WARN.  Anything unavailable
on the host (no GPU, no smartctl) is skipped, never an error.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import re
import shutil
import socket
import subprocess
import threading
import time

HOST = socket.gethostname()


def event(type_, level, source, message="", **props) -> dict:
    return {"hostname": HOST, "timestamp": time.time(), "type": type_, "logLevel": level,
            "source": source, "message": message, "properties": props}


def _read(path, default=None):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def _num(v):
    try:
        return int(v)
    except (TypeError, ValueError):
        try:
            return float(v)
        except (TypeError, ValueError):
            return None


# ---------------------------------------------------------------- parsers
class GPUParser:
    """amdgpu sysfs of each card: thermals, power, memory, busy, RAS counters."""

    def __init__(self, drm_root="/sys/class/drm", temp_warn_c=95.0):
        self.root = drm_root
        self.temp_warn = temp_warn_c

    def cards(self):
        return sorted(d for d in glob.glob(os.path.join(self.root, "card*"))
                      if re.fullmatch(r"card\d+", os.path.basename(d))
                      and os.path.exists(os.path.join(d, "device", "vendor")))

    def query(self):
        out = []
        for card in self.cards():
            dev = os.path.join(card, "device")
            if _read(os.path.join(dev, "vendor"), "") != "0x1002":   # AMD only
                continue
            props = {"card": os.path.basename(card),
                     "busy_percent": _num(_read(os.path.join(dev, "gpu_busy_percent"))),
                     "vram_used": _num(_read(os.path.join(dev, "mem_info_vram_used"))),
                     "vram_total": _num(_read(os.path.join(dev, "mem_info_vram_total")))}
            level = "INFO"
            msgs = []
            for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
                for t in glob.glob(os.path.join(hw, "temp*_input")):
                    label = _read(t.replace("_input", "_label"), os.path.basename(t))
                    c = (_num(_read(t)) or 0) / 1000.0
                    props[f"temp_{label}"] = c
                    if c >= self.temp_warn:
                        level = "WARN"
                        msgs.append(f"{label} {c:.0f}C")
                for pw in ("power1_average", "power1_input"):
                    v = _num(_read(os.path.join(hw, pw)))
                    if v is not None:
                        props["power_w"] = v / 1e6
                        break
            for f in glob.glob(os.path.join(dev, "ras", "*_err_count")):
                block = os.path.basename(f)[:-len("_err_count")]
                txt = _read(f, "")
                ue = re.search(r"ue:\s*(\d+)", txt)
                ce = re.search(r"ce:\s*(\d+)", txt)
                ue, ce = int(ue.group(1)) if ue else 0, int(ce.group(1)) if ce else 0
                props[f"ras_{block}_ue"], props[f"ras_{block}_ce"] = ue, ce
                if ue:
                    level = "ERROR"
                    msgs.append(f"{block}: {ue} uncorrectable errors")
                elif ce and level == "INFO":
                    level = "WARN"
                    msgs.append(f"{block}: {ce} correctable errors")
            out.append(event("GPU", level, "amdgpu", "; ".join(msgs), **props))
        return out


class CPUParser:
    def query(self):
        props = {}
        la = _read("/proc/loadavg")
        if la:
            props["load1"], props["load5"], props["load15"] = map(float, la.split()[:3])
        info = _read("/proc/cpuinfo", "")
        props["processors"] = info.count("processor\t:")
        m = re.search(r"model name\s*:\s*(.+)", info)
        if m:
            props["model"] = m.group(1)
        mem = _read("/proc/meminfo", "")
        for k in ("MemTotal", "MemAvailable"):
            m = re.search(rf"{k}:\s*(\d+)", mem)
            if m:
                props[k] = int(m.group(1)) * 1024
        return [event("CPU", "INFO", "/proc", **props)]


class NICParser:
    def query(self):
        out = []
        txt = _read("/proc/net/dev", "")
        for line in txt.splitlines()[2:]:
            name, _, rest = line.partition(":")
            f = [int(x) for x in rest.split()]
            if len(f) < 16:
                continue
            props = {"iface": name.strip(), "rx_bytes": f[0], "rx_errs": f[2], "rx_drop": f[3],
                     "tx_bytes": f[8], "tx_errs": f[10], "tx_drop": f[11]}
            bad = props["rx_errs"] + props["tx_errs"]
            out.append(event("NIC", "WARN" if bad else "INFO", "/proc/net/dev",
                             f"{bad} errors" if bad else "", **props))
        return out


class SensorsParser:
    """Non-GPU hwmon sensors (CPU package, board)."""

    def query(self):
        out = []
        for hw in glob.glob("/sys/class/hwmon/hwmon*"):
            name = _read(os.path.join(hw, "name"), "")
            if name == "amdgpu":
                continue   # reported by GPUParser
            props = {"chip": name}
            for t in glob.glob(os.path.join(hw, "temp*_input")):
                props[os.path.basename(t)[:-6]] = (_num(_read(t)) or 0) / 1000.0
            if len(props) > 1:
                out.append(event("SENSORS", "INFO", "hwmon", **props))
        return out


class SMARTParser:
    def query(self):
        exe = shutil.which("smartctl")
        if not exe:
            return []
        out = []
        for disk in sorted(glob.glob("/dev/nvme[0-9]") + glob.glob("/dev/sd[a-z]")):
            try:
                r = subprocess.run([exe, "-H", disk], capture_output=True, text=True, timeout=10)
            except (OSError, subprocess.TimeoutExpired):
                continue
            ok = "PASSED" in r.stdout or "OK" in r.stdout
            out.append(event("SMART", "INFO" if ok else "ERROR", disk,
                             "" if ok else r.stdout[-200:], healthy=ok))
        return out


_LOG_RE = re.compile(r"\b(FATAL|ERROR|WARN(?:ING)?)\b\s*(.*)")


class LogParser:
    """Hadoop-style daemon logs (HadoopLogParser) or syslog (SystemLogParser):
    WARN/ERROR/FATAL lines since the last read offset of each file."""

    def __init__(self, paths, source="hadoop"):
        self.paths = list(paths)
        self.source = source
        self.offsets: dict[str, int] = {}

    def query(self):
        out = []
        for p in self.paths:
            for f in glob.glob(p):
                try:
                    size = os.path.getsize(f)
                    off = self.offsets.get(f, 0)
                    if size < off:
                        off = 0   # rotated
                    with open(f, errors="replace") as fh:
                        fh.seek(off)
                        for line in fh:
                            m = _LOG_RE.search(line)
                            if m:
                                lvl = "WARN" if m.group(1).startswith("WARN") else m.group(1)
                                out.append(event("LOG", lvl, f, m.group(2).strip()[:500]))
                        self.offsets[f] = fh.tell()
                except OSError:
                    continue
        return out


# ---------------------------------------------------------------- store / anonymize
_IP = re.compile(r"\b\d{1,3}(?:\.\d{1,3}){3}\b")


def anonymize(rec: dict, salt: str = "") -> dict:
    """Anonymizer: hash host names and IPv4 addresses (SHA-1, truncated)."""
    def h(s):
        return hashlib.sha1((salt + s).encode()).hexdigest()[:12]
    r = dict(rec)
    r["hostname"] = h(rec["hostname"])
    r["message"] = _IP.sub(lambda m: h(m.group(0)), rec.get("message", ""))
    r["properties"] = {k: (_IP.sub(lambda m: h(m.group(0)), v) if isinstance(v, str) else v)
                       for k, v in rec.get("properties", {}).items()}
    return r


class LocalStore:
    def __init__(self, path, anonymize_records=False):
        self.path = path
        self.anon = anonymize_records
        self.lock = threading.Lock()
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)

    def insert(self, records):
        with self.lock, open(self.path, "a") as f:
            for r in records:
                f.write(json.dumps(anonymize(r) if self.anon else r, default=str) + "\n")

    def read(self):
        if not os.path.exists(self.path):
            return []
        with open(self.path) as f:
            return [json.loads(x) for x in f if x.strip()]


def default_parsers(log_globs=()):
    ps = [GPUParser(), CPUParser(), NICParser(), SensorsParser(), SMARTParser()]
    if log_globs:
        ps.append(LogParser(log_globs))
    return ps


def run_once(store: LocalStore, parsers=None) -> list:
    """RunOnce: query every parser, store and return the records."""
    recs = []
    for p in parsers or default_parsers():
        try:
            recs += p.query()
        except Exception as e:  # noqa: BLE001 - a broken parser never stops monitoring
            recs.append(event("FAILMON", "WARN", type(p).__name__, f"parser failed: {e}"))
    store.insert(recs)
    return recs


class Continuous:
    """Continuous: run_once every ``interval`` seconds on a daemon thread."""

    def __init__(self, store, parsers=None, interval=60.0):
        self.store, self.parsers, self.interval = store, parsers, interval
        self.rounds = 0
        self._stop = threading.Event()
        self._thread = None

    def _run(self):
        while not self._stop.is_set():
            run_once(self.store, self.parsers)
            self.rounds += 1
            self._stop.wait(self.interval)

    def start(self):
        self._thread = threading.Thread(target=self._run, daemon=True, name="failmon")
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=10)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(prog="hbmr failmon")
    ap.add_argument("--store", default="failmon/events.jsonl")
    ap.add_argument("--logs", nargs="*", default=[])
    ap.add_argument("--interval", type=float, default=0.0, help="0 = run once")
    ap.add_argument("--anonymize", action="store_true")
    a = ap.parse_args(argv)
    store = LocalStore(a.store, a.anonymize)
    parsers = default_parsers(a.logs)
    if a.interval <= 0:
        for r in run_once(store, parsers):
            if r["logLevel"] != "INFO":
                print(json.dumps(r, default=str))
        return 0
    c = Continuous(store, parsers, a.interval).start()
    try:
        while True:
            time.sleep(1.0)
    except KeyboardInterrupt:
        c.stop()
    return 0
