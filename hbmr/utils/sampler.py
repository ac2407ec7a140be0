"""A sampling profiler for the control plane: a daemon thread snapshots every
thread's Python stack (``sys._current_frames``) every ``interval`` seconds and
counts (thread-name prefix, function) samples — self time and inclusive time
— so the JobTracker's and TaskTracker's threads can be profiled inside a live
multi-rank run, where cProfile (one thread, heavy overhead) cannot.

``HBMR_SAMPLE_PROF=/path/prefix`` in a bench or node process starts it; the
report is written to ``<prefix>_<pid>.txt`` at exit."""
from __future__ import annotations

import atexit
import collections
import os
import sys
import threading
import time


class Sampler:
    def __init__(self, interval=0.0005):
        self.interval = interval
        self.self_counts = collections.Counter()
        self.incl_counts = collections.Counter()
        self.line_counts = collections.Counter()
        self.thread_counts = collections.Counter()
        self.samples = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="hbmr-sampler")

    def start(self):
        self._t.start()
        return self

    def stop(self):
        self._stop.set()

    def _run(self):
        me = threading.get_ident()
        while not self._stop.is_set():
            names = {t.ident: t.name for t in threading.enumerate()}
            for tid, frame in sys._current_frames().items():
                if tid == me:
                    continue
                tname = names.get(tid, "?")
                group = tname.split("-")[0] if "-" in tname else tname
                if _idle(frame):
                    continue
                self.thread_counts[group] += 1
                f = frame
                key = _key(f)
                self.self_counts[(group, key)] += 1
                self.line_counts[(group, f"{key} @{f.f_lineno}")] += 1
                seen = set()
                while f is not None:
                    k = _key(f)
                    if k not in seen:
                        self.incl_counts[(group, k)] += 1
                        seen.add(k)
                    f = f.f_back
            self.samples += 1
            time.sleep(self.interval)

    def mark(self):
        """Per-thread CPU is reported relative to now (e.g. a timed window)."""
        self.cpu_mark = _thread_cpu()

    def report(self, top=40):
        lines = [f"samples {self.samples} (interval {self.interval * 1e3:.2f} ms); busy "
                 f"samples per thread group:"]
        for g, n in self.thread_counts.most_common():
            lines.append(f"  {n:7d}  {g}")
        lines.append("\nself time (busy samples):")
        for (g, k), n in self.self_counts.most_common(top):
            lines.append(f"  {n:7d}  {g:<24} {k}")
        lines.append("\nself time by line (a line that blocks in C, e.g. a lock "
                     "acquire or the GIL, shows here):")
        for (g, k), n in self.line_counts.most_common(top // 2):
            lines.append(f"  {n:7d}  {g:<24} {k}")
        rpc = sys.modules.get("hbmr.mapred.rpc")
        if rpc is not None and rpc.RPC_STATS:
            lines.append("\nRPC server methods (calls, total s, mean us):")
            for m, (n, t) in sorted(rpc.RPC_STATS.items(), key=lambda kv: -kv[1][1]):
                lines.append(f"  {m:<28} {n:8d} {t:9.3f} {t / max(1, n) * 1e6:9.1f}")
        now = _thread_cpu()
        base = getattr(self, "cpu_mark", None)
        lines.append("\nCPU seconds per thread (/proc, by thread name)" +
                     (" since mark()" if base is not None else "") + ":")
        if base is not None:
            now = collections.Counter({g: t - base.get(g, 0.0) for g, t in now.items()})
        for g, t in sorted(now.items(), key=lambda kv: -kv[1])[:20]:
            lines.append(f"  {t:9.3f}  {g}")
        if rpc is not None and getattr(rpc, "_PROFS", None):
            import io, pstats
            buf = io.StringIO()
            ps = list(rpc._PROFS.values())
            st = pstats.Stats(ps[0], stream=buf)
            for p in ps[1:]:
                st.add(p)
            st.sort_stats("tottime").print_stats(45)
            lines.append(buf.getvalue())
        jt = sys.modules.get("hbmr.mapred.jobtracker")
        pl = getattr(getattr(jt, "_ProfLock", None), "STATS", None)
        if pl:
            lines.append("\nJT lock holds (calls, total ms):")
            for k2, (n2, t2) in sorted(pl.items(), key=lambda kv: -kv[1][1])[:25]:
                lines.append(f"  {k2:<40} {n2:7d} {t2 * 1e3:9.1f}")
        lines.append("\ninclusive time (busy samples):")
        for (g, k), n in self.incl_counts.most_common(top):
            lines.append(f"  {n:7d}  {g:<24} {k}")
        return "\n".join(lines)


_IDLE = {"wait", "_wait_for_tstate_lock", "select", "accept", "recv_into", "recv", "get",
         "sleep", "poll", "_recv_bytes", "readinto", "acquire", "_worker", "serve_forever",
         "wait_for", "result", "join", "_recv_exact", "barrier", "serve_until_shutdown",
         "recv_msg", "_wait"}


def _thread_cpu():
    """utime+stime of this process's threads from /proc, by thread name
    (threads that ended are not counted)."""
    names = {t.native_id: t.name for t in threading.enumerate()}
    tick = os.sysconf("SC_CLK_TCK")
    out = collections.Counter()
    try:
        tids = os.listdir("/proc/self/task")
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                parts = f.read().rsplit(")", 1)[1].split()
        except OSError:
            continue
        name = names.get(int(tid), "native")
        out[name] += (int(parts[11]) + int(parts[12])) / tick
    return out


def _idle(frame):
    """A thread blocked in a wait/recv/select (its innermost Python frame)."""
    return frame.f_code.co_name in _IDLE


def _key(f):
    c = f.f_code
    fn = c.co_filename
    i = fn.find("hbmr/")
    fn = fn[i:] if i >= 0 else os.path.basename(fn)
    return f"{fn}:{c.co_firstlineno} {c.co_name}"


def maybe_arm_stackdump():
    """``HBMR_STACKDUMP_S=<s>``: every s seconds write every thread's Python
    stack to stderr (faulthandler) — where a slow or stuck run is waiting."""
    s = os.environ.get("HBMR_STACKDUMP_S")
    if not s:
        return
    import faulthandler
    faulthandler.dump_traceback_later(float(s), repeat=True, file=sys.stderr)


def maybe_watch_jobtracker(jt):
    """With ``HBMR_STACKDUMP_S``: also print the JobTracker's view of its
    unfinished jobs and of each tracker every that many seconds (stderr)."""
    s = os.environ.get("HBMR_STACKDUMP_S")
    if not s or jt is None:
        return

    def loop():
        while True:
            time.sleep(float(s))
            try:
                lines = ["jt-watch:"]
                with jt.lock:
                    for jid, j in list(jt.jobs.items()):
                        if j.completed():
                            continue
                        ra = sum(1 for t in j.maps for a in t.running_attempts())
                        lines.append(
                            f"  {jid} state={j.status.state} maps={len(j.maps)} "
                            f"pending={len(j.pending_maps)} running_attempts={ra} "
                            f"running_gpu={j.running_gpu} running_cpu={j.running_cpu} "
                            f"done={j.maps_done} reduces_done="
                            f"{sum(1 for r in j.reduces if r.successful)}/{len(j.reduces)} "
                            f"staged_on={j.staged_on} expect={j.expect_mode}")
                        for r in j.reduces:
                            if r.successful is None:
                                lines.append("    reduce " + str(r.tid) + " attempts " + ", ".join(
                                    f"{a.aid[-12:]}@{a.tracker[-3:]}:{a.state}"
                                    for a in r.attempts.values()))
                    evs = [e for e in list(getattr(jt.history, "events", []))
                           if any(w in e.get("event", "") for w in ("FAILED", "RESTART", "LOST",
                                                                     "KILLED"))]
                    for e in evs[-6:]:
                        lines.append(f"  event {e.get('event')} {e.get('attempt') or e.get('job')}"
                                     f" {str(e.get('diag', ''))[:300]!r}")
                    for name, tr in jt.trackers.items():
                        lines.append(f"  tracker {name}: running={len(tr.running)} "
                                     f"gpu={dict(tr.running_gpu)} cpu={tr.running_cpu} "
                                     f"cached={len(tr.cached)} more={tr.more}")
                print("\n".join(lines), file=sys.stderr, flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"jt-watch: {e!r}", file=sys.stderr, flush=True)
    threading.Thread(target=loop, daemon=True, name="hbmr-jtwatch").start()


_PROFILES: list = []


def maybe_profile_threads():
    """``HBMR_CPROFILE=path``: every thread started from now on (and the
    caller's) runs under its own cProfile; ``dump_profiles`` merges them."""
    path = os.environ.get("HBMR_CPROFILE")
    if not path:
        return None
    import cProfile
    orig = threading.Thread.run

    def run(self):
        pr = cProfile.Profile(time.thread_time)
        _PROFILES.append(pr)
        pr.enable()
        try:
            orig(self)
        finally:
            pr.disable()
    threading.Thread.run = run
    main = cProfile.Profile(time.thread_time)
    _PROFILES.append(main)
    main.enable()
    return path


def dump_profiles(path):
    import io
    import pstats
    for pr in _PROFILES:
        try:
            pr.disable()
        except Exception:  # noqa: BLE001
            pass
    st = None
    for pr in _PROFILES:
        try:
            if st is None:
                st = pstats.Stats(pr, stream=io.StringIO())
            else:
                st.add(pr)
        except TypeError:      # a profile that never ran
            pass
    if st is None:
        return
    buf = io.StringIO()
    st.stream = buf
    st.sort_stats("tottime").print_stats(60)
    st.sort_stats("cumulative").print_stats(60)
    with open(f"{path}_{os.getpid()}.txt", "w") as f:
        f.write(buf.getvalue())
    st.dump_stats(f"{path}_{os.getpid()}.prof")     # raw, for pstats diffs


def maybe_start():
    prefix = os.environ.get("HBMR_SAMPLE_PROF")
    if not prefix:
        return None
    s = Sampler(float(os.environ.get("HBMR_SAMPLE_PROF_INTERVAL", "0.0005"))).start()

    def dump():
        if s._stop.is_set():
            return
        s.stop()
        with open(f"{prefix}_{os.getpid()}.txt", "w") as f:
            f.write(s.report())
    s.dump = dump
    atexit.register(dump)
    return s
