"""JobTracker web UI (the reference's webapps/job JSPs + TaskGraphServlet).

  /                         cluster summary: trackers (CPU slots, GPUs, running
                            tasks), running and completed jobs
  /jobdetails?jobid=ID      job status, counters, map/reduce task tables with
                            the placement of the successful attempt
  /taskgraph?jobid=ID&type=map|reduce
                            SVG progress bars — GPU tasks green (#00DD00), CPU
                            tasks blue (#AAAAFF) as TaskGraphServlet.java:113,
                            141-146, indexed correctly (the fork used
                            reports[barCnt])
  /timeline?jobid=ID        Chrome/Perfetto trace JSON of the job's attempts,
                            one track per tracker slot kind, CPU/GPU coloured
  /metrics                  Prometheus text exposition (hbmr.utils.metrics)
  /api/cluster, /api/jobs, /api/job?jobid=ID    JSON
  /jobconf.jsp?jobid=ID     the job's configuration
  /jobtasks.jsp?jobid=ID&type=map|reduce&pagenum=N&state=running|completed|killed|all
  /taskdetails.jsp?tipid=ID every attempt of a task (tracker, CPU/GPU, times, diagnostics)
  /jobfailures.jsp?jobid=ID failed and killed attempts, grouped by tracker
  /machines.jsp[?type=active|blacklisted]   trackers with slots, failures, health
  /jobqueue_details.jsp?queueName=Q         a queue's jobs (+ its ACLs)
  /jobhistory.jsp           completed-job history files; ?logFile=F → summary +
                            rule-based analysis (analysejobhistory.jsp / Vaidya)

:class:`DFSWebUI` serves the NameNode pages (webapps/hdfs): ``/dfshealth.jsp``
(capacity, safe mode, live/dead DataNodes), ``/dfsnodelist.jsp?whatNodes=LIVE|DEAD``
and ``/browseDirectory.jsp?dir=/path`` (nn_browsedfscontent; ``?filename=`` shows
the first 32 KB of a file).

Enabled by ``hbmr.webui.port`` (default 50030, the reference's
mapred.job.tracker.http.address port; 0 = any free port; -1 = off).
"""
from __future__ import annotations

import html
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

from ..utils.metrics import METRICS

GPU_COLOR, CPU_COLOR = "#00DD00", "#AAAAFF"

_CSS = ("body{font-family:sans-serif;margin:1.5em}table{border-collapse:collapse}"
        "td,th{border:1px solid #ccc;padding:2px 8px;font-size:13px}th{background:#eee}"
        ".gpu{color:#080}.cpu{color:#448}")


def _page(title, body):
    return (f"<html><head><title>{html.escape(title)}</title><style>{_CSS}</style></head>"
            f"<body><h1>{html.escape(title)}</h1>{body}</body></html>")


def _table(headers, rows):
    h = "".join(f"<th>{html.escape(str(x))}</th>" for x in headers)
    r = "".join("<tr>" + "".join(f"<td>{c}</td>" for c in row) + "</tr>" for row in rows)
    return f"<table><tr>{h}</tr>{r}</table>"


def _fmt_t(t):
    return time.strftime("%H:%M:%S", time.localtime(t)) if t else "-"


class WebUI:
    def __init__(self, jt, host="0.0.0.0", port=50030):
        self.jt = jt
        ui = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def do_GET(self):  # noqa: N802
                u = urlparse(self.path)
                q = {k: v[0] for k, v in parse_qs(u.query).items()}
                try:
                    ctype, body = ui.route(u.path, q)
                    code = 200
                except KeyError as e:
                    ctype, body, code = "text/plain", f"not found: {e}", 404
                except Exception as e:  # noqa: BLE001
                    ctype, body, code = "text/plain", f"error: {type(e).__name__}: {e}", 500
                data = body.encode() if isinstance(body, str) else body
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

        self.httpd = ThreadingHTTPServer((host, port), Handler)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self.url = f"http://127.0.0.1:{self.port}/"
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True,
                                       name="webui")

    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    # -- data -----------------------------------------------------------------------------
    def cluster(self):
        jt = self.jt
        with jt.lock:
            trackers = [{"name": n, "cpu_slots": t.status.max_cpu_map_slots,
                         "reduce_slots": t.status.max_reduce_slots,
                         "gpus": [{"device": g["device"], "slots": g["max_slots"],
                                   "name": g.get("name", "")} for g in t.status.gpus],
                         "running_cpu": t.running_cpu, "running_gpu": dict(t.running_gpu),
                         "running_reduce": t.running_reduce, "last_seen": t.last_seen,
                         "blacklisted": t.blacklisted, "cached_splits": len(t.cached)}
                        for n, t in sorted(jt.trackers.items())]
        return {"name": jt.name, "started": jt.start_time, "trackers": trackers,
                "cost_model": jt.cost_model.snapshot()}

    def jobs(self):
        return self.jt.rpc_list_jobs(True)

    def job(self, jid):
        jip = self.jt.jobs[jid]
        with self.jt.lock:
            counters = jip.fold_counters().to_dict()
            st = jip.status

            def rows(tips):
                out = []
                for tip in tips:
                    a = tip.successful or (max(tip.attempts.values(), key=lambda x: x.start)
                                           if tip.attempts else None)
                    out.append({"task": str(tip.tid), "state": a.state if a else "UNASSIGNED",
                                "progress": 1.0 if tip.successful else (a.progress if a else 0),
                                "gpu": bool(a and a.run_on_gpu), "device": a.device if a else -1,
                                "tracker": a.tracker if a else "", "start": a.start if a else 0,
                                "finish": a.finish if a else 0,
                                "attempts": len(tip.attempts)})
                return out
            return {"id": jid, "name": jip.conf.get_job_name(), "state": st.state,
                    "map_progress": st.map_progress, "reduce_progress": st.reduce_progress,
                    "submit": jip.submit_time, "finish": st.finish_time,
                    "failure": st.failure_info, "timeline": jip.timeline(),
                    "cpu_maps": jip.finished_cpu_maps, "gpu_maps": jip.finished_gpu_maps,
                    "counters": counters, "maps": rows(jip.maps), "reduces": rows(jip.reduces)}

    # -- routes ---------------------------------------------------------------------------
    def route(self, path, q):
        if path in ("/", "/jobtracker.jsp"):
            return "text/html", self.index_html()
        if path in ("/jobdetails", "/jobdetails.jsp"):
            return "text/html", self.job_html(q["jobid"])
        if path in ("/taskgraph",):
            return "image/svg+xml", self.taskgraph_svg(q["jobid"], q.get("type", "map"))
        if path == "/timeline":
            return "application/json", json.dumps(self.timeline(q["jobid"]))
        if path == "/metrics":
            return "text/plain; version=0.0.4", METRICS.prometheus_text()
        if path == "/api/cluster":
            return "application/json", json.dumps(self.cluster(), default=str)
        if path == "/api/jobs":
            return "application/json", json.dumps(self.jobs(), default=str)
        if path == "/api/job":
            return "application/json", json.dumps(self.job(q["jobid"]), default=str)
        extra = {"/jobconf.jsp": self.jobconf_html, "/jobtasks.jsp": self.jobtasks_html,
                 "/taskdetails.jsp": self.taskdetails_html, "/jobfailures.jsp":
                 self.jobfailures_html, "/machines.jsp": self.machines_html,
                 "/jobqueue_details.jsp": self.queue_html, "/jobhistory.jsp": self.history_html}
        if path in extra:
            return "text/html", extra[path](q)
        raise KeyError(path)

    # -- the remaining webapps/job pages ------------------------------------------------------
    def _jip(self, q):
        jid = q.get("jobid")
        if jid not in self.jt.jobs:
            raise KeyError(f"job {jid}")
        return jid, self.jt.jobs[jid]

    def jobconf_html(self, q):
        jid, jip = self._jip(q)
        rows = [[html.escape(k), html.escape(str(v))] for k, v in sorted(jip.conf.items())]
        return _page(f"Job Configuration: {jid}", _table(["name", "value"], rows))

    @staticmethod
    def _attempt_row(a):
        where = f"<span class=gpu>gpu{a.device}</span>" if a.run_on_gpu else \
            "<span class=cpu>cpu</span>"
        dur = f"{a.finish - a.start:.3f}s" if a.finish and a.start else "-"
        return [html.escape(str(a.aid)), a.state, where, html.escape(a.tracker or ""),
                _fmt_t(a.start), _fmt_t(a.finish), dur,
                f"{100 * (a.progress or 0):.0f}%", html.escape((a.diagnostic or "")[:300])]

    _ATTEMPT_HDR = ["attempt", "state", "ran on", "tracker", "start", "finish", "time",
                    "progress", "diagnostics"]

    def jobtasks_html(self, q):
        jid, jip = self._jip(q)
        typ = q.get("type", "map")
        want = q.get("state", "all")
        page, per = int(q.get("pagenum", 1)), 200
        with self.jt.lock:
            tips = jip.maps if typ == "map" else jip.reduces
            rows = []
            for tip in tips:
                st = ("completed" if tip.successful else "killed" if tip.killed else
                      "running" if tip.attempts else "pending")
                if want not in ("all", st):
                    continue
                a = tip.successful or (max(tip.attempts.values(), key=lambda x: x.start or 0)
                                       if tip.attempts else None)
                rows.append([f"<a href='/taskdetails.jsp?jobid={jid}&tipid={tip.tid}'>"
                             f"{tip.tid}</a>", st, len(tip.attempts), tip.failures]
                            + (self._attempt_row(a)[2:8] if a else ["-"] * 6))
        body = _table(["task", "status", "attempts", "failures", "ran on", "tracker", "start",
                       "finish", "time", "progress"], rows[(page - 1) * per:page * per])
        return _page(f"{typ} tasks of {jid} ({want})", body)

    def _tip(self, q):
        tipid = q.get("tipid")
        jids = [q["jobid"]] if q.get("jobid") else list(self.jt.jobs)
        for jid in jids:
            jip = self.jt.jobs.get(jid)
            for tip in (jip.maps + jip.reduces) if jip else []:
                if str(tip.tid) == tipid:
                    return jid, tip
        raise KeyError(f"task {tipid}")

    def taskdetails_html(self, q):
        jid, tip = self._tip(q)
        with self.jt.lock:
            rows = [self._attempt_row(a) for a in sorted(tip.attempts.values(),
                                                         key=lambda a: str(a.aid))]
        split = html.escape(str(getattr(tip.split, "path", tip.split))[:200]) if tip.split else "-"
        return _page(f"Task {tip.tid}", f"<p>job {jid}; input split: {split}</p>"
                     + _table(self._ATTEMPT_HDR, rows))

    def jobfailures_html(self, q):
        jid, jip = self._jip(q)
        by_tracker: dict = {}
        with self.jt.lock:
            for tip in jip.maps + jip.reduces:
                for a in tip.attempts.values():
                    if a.state in ("FAILED", "KILLED"):
                        by_tracker.setdefault(a.tracker or "?", []).append(self._attempt_row(a))
        body = "".join(f"<h2>{html.escape(t)}</h2>" + _table(self._ATTEMPT_HDR, rows)
                       for t, rows in sorted(by_tracker.items())) or "<p>no failures</p>"
        return _page(f"Failures of {jid}", body)

    def machines_html(self, q):
        typ = q.get("type", "active")
        with self.jt.lock:
            rows = [[html.escape(n), t.status.max_cpu_map_slots,
                     ", ".join(f"gpu{g['device']}" for g in t.status.gpus) or "-",
                     t.status.max_reduce_slots, t.failures,
                     "yes" if t.status.healthy else f"no: {html.escape(str(t.status.health_report))}",
                     f"{time.time() - t.last_seen:.1f}s ago"]
                    for n, t in sorted(self.jt.trackers.items())
                    if (typ == "blacklisted") == bool(t.blacklisted)]
        return _page(f"{typ.capitalize()} Task Trackers",
                     _table(["tracker", "CPU map slots", "GPUs", "reduce slots", "failures",
                             "healthy", "last heartbeat"], rows))

    def queue_html(self, q):
        from ..security import QueueManager
        name = q.get("queueName", "default")
        qm = QueueManager(self.jt.conf)
        acls = [[op, html.escape(str(qm.acl(name, op)))] for op in ("acl-submit-job",
                                                                    "acl-administer-jobs")]
        jobs = [[f"<a href='/jobdetails?jobid={j['id']}'>{j['id']}</a>", html.escape(j["name"]),
                 html.escape(str(j["user"])), j["state"]]
                for j in self.jobs()
                if self.jt.jobs[j["id"]].conf.get("mapred.job.queue.name", "default") == name]
        return _page(f"Queue {name}", _table(["acl", "value"], acls)
                     + _table(["job", "name", "user", "state"], jobs))

    def history_html(self, q):
        import os
        from .history import diagnose, history_dir, load_history, summarize_history
        d = history_dir(self.jt.conf)
        if q.get("logFile"):
            path = os.path.join(d, os.path.basename(q["logFile"]))
            job, attempts = load_history(path)
            summ = summarize_history(path)
            rules = diagnose(job, attempts)
            return _page(f"Analysis of {os.path.basename(path)}",
                         f"<pre>{html.escape(json.dumps(summ, indent=1, default=str))}</pre>"
                         "<h2>Diagnosis</h2><ul>" + "".join(
                             f"<li>{html.escape(str(r))}</li>" for r in rules) + "</ul>")
        files = sorted(os.listdir(d)) if d and os.path.isdir(d) else []
        rows = [[f"<a href='/jobhistory.jsp?logFile={f}'>{html.escape(f)}</a>"] for f in files
                if f.endswith(".jsonl")]
        return _page("Job History", _table(["history file"], rows))

    def index_html(self):
        c = self.cluster()
        trs = []
        for t in c["trackers"]:
            gpus = ", ".join(f"gpu{g['device']}×{g['slots']}" for g in t["gpus"]) or "-"
            trs.append([html.escape(t["name"]), t["cpu_slots"], gpus, t["running_cpu"],
                        sum(t["running_gpu"].values()), t["running_reduce"],
                        t["cached_splits"], "yes" if t["blacklisted"] else ""])
        jobs = self.jobs()
        jrows = [[f"<a href='/jobdetails?jobid={j['id']}'>{j['id']}</a>", html.escape(j["name"]),
                  j["state"], f"{100 * j['map_progress']:.0f}%",
                  f"{100 * j['reduce_progress']:.0f}%", j["maps"],
                  f"<span class=cpu>{j['cpu_maps']}</span>/<span class=gpu>{j['gpu_maps']}</span>",
                  _fmt_t(j["start"])] for j in reversed(jobs)]
        body = (f"<p>JobTracker {html.escape(c['name'])} — {len(c['trackers'])} trackers</p>"
                "<h2>Cluster</h2>" + _table(["tracker", "CPU map slots", "GPUs", "running CPU",
                                             "running GPU", "running reduce", "HBM splits",
                                             "blacklisted"], trs)
                + "<h2>Jobs</h2>" + _table(["job", "name", "state", "map %", "reduce %", "maps",
                                            "done cpu/gpu", "submitted"], jrows)
                + "<p><a href='/metrics'>metrics</a></p>")
        return _page("hbmr JobTracker", body)

    def job_html(self, jid):
        j = self.job(jid)

        def task_rows(ts):
            return [[t["task"], t["state"], f"{100 * t['progress']:.0f}%",
                     f"<span class=gpu>gpu{t['device']}</span>" if t["gpu"] else
                     "<span class=cpu>cpu</span>", html.escape(t["tracker"] or ""),
                     _fmt_t(t["start"]),
                     f"{t['finish'] - t['start']:.3f}s" if t["finish"] else "-", t["attempts"]]
                    for t in ts]
        crow = [[html.escape(g), html.escape(n), v] for g, cs in sorted(j["counters"].items())
                for n, v in sorted(cs.items())]
        hdr = ["task", "state", "progress", "ran on", "tracker", "start", "time", "attempts"]
        body = (f"<p>{html.escape(j['name'])}: <b>{j['state']}</b>, maps "
                f"{100 * j['map_progress']:.0f}% reduces {100 * j['reduce_progress']:.0f}%, "
                f"CPU/GPU maps {j['cpu_maps']}/{j['gpu_maps']}</p>"
                f"<p>timeline (s from submit): {html.escape(json.dumps(j['timeline']))}</p>"
                f"<p><a href='/timeline?jobid={jid}'>trace (Perfetto JSON)</a></p>"
                f"<embed src='/taskgraph?jobid={jid}&type=map' type='image/svg+xml'/>"
                "<h2>Map tasks</h2>" + _table(hdr, task_rows(j["maps"]))
                + "<h2>Reduce tasks</h2>" + _table(hdr, task_rows(j["reduces"]))
                + "<h2>Counters</h2>" + _table(["group", "counter", "value"], crow))
        return _page(f"Job {jid}", body)

    def taskgraph_svg(self, jid, typ="map"):
        j = self.job(jid)
        tasks = j["maps"] if typ == "map" else j["reduces"]
        w, bh = 600, 12
        h = max(1, len(tasks)) * (bh + 2) + 20
        parts = [f"<svg xmlns='http://www.w3.org/2000/svg' width='{w + 120}' height='{h}'>"]
        for i, t in enumerate(tasks):
            y = 10 + i * (bh + 2)
            color = GPU_COLOR if t["gpu"] else CPU_COLOR
            parts.append(f"<rect x='100' y='{y}' width='{w}' height='{bh}' fill='#eee'/>")
            parts.append(f"<rect x='100' y='{y}' width='{w * t['progress']:.1f}' height='{bh}' "
                         f"fill='{color}'/>")
            parts.append(f"<text x='2' y='{y + bh - 2}' font-size='10'>{t['task'][-8:]}</text>")
        parts.append("</svg>")
        return "".join(parts)

    def timeline(self, jid):
        j = self.job(jid)
        t0 = j["submit"]
        ev = []
        tids: dict = {}
        for kind, ts in (("map", j["maps"]), ("reduce", j["reduces"])):
            for t in ts:
                if not t["start"]:
                    continue
                track = f"{t['tracker']} {'gpu' + str(t['device']) if t['gpu'] else kind}"
                tid = tids.setdefault(track, len(tids) + 1)
                ev.append({"name": t["task"], "ph": "X", "pid": 1, "tid": tid,
                           "ts": (t["start"] - t0) * 1e6,
                           "dur": max(0.0, ((t["finish"] or time.time()) - t["start"]) * 1e6),
                           "cname": "good" if t["gpu"] else "rail_idle",
                           "args": {"state": t["state"], "tracker": t["tracker"]}})
        for track, tid in tids.items():
            ev.append({"name": "thread_name", "ph": "M", "pid": 1, "tid": tid,
                       "args": {"name": track}})
        return {"traceEvents": ev, "displayTimeUnit": "ms"}


class DFSWebUI(WebUI):
    """NameNode web UI (webapps/hdfs): health, node lists, directory browser."""

    def __init__(self, namenode, host="0.0.0.0", port=50070):
        self.nn = namenode
        super().__init__(None, host, port)

    def route(self, path, q):
        if path in ("/", "/dfshealth.jsp"):
            return "text/html", self.health_html()
        if path == "/dfsnodelist.jsp":
            return "text/html", self.nodelist_html(q.get("whatNodes", "LIVE"))
        if path in ("/browseDirectory.jsp", "/nn_browsedfscontent.jsp"):
            return "text/html", self.browse_html(q)
        if path == "/metrics":
            return "text/plain; version=0.0.4", METRICS.prometheus_text()
        raise KeyError(path)

    def health_html(self):
        nodes = self.nn.datanode_report()
        cap = sum(d["capacity"] or 0 for d in nodes if d["alive"])
        used = sum(d["used"] or 0 for d in nodes if d["alive"])
        fsck = self.nn.fsck("/")
        live = sum(1 for d in nodes if d["alive"])
        rows = [["Configured Capacity", cap], ["DFS Used", used],
                ["DFS Used%", f"{100 * used / cap:.2f}%" if cap else "-"],
                ["Files", fsck["files"]], ["Blocks", fsck["blocks"]],
                ["Missing blocks", fsck["missing_blocks"]],
                ["Under-replicated blocks", fsck["under_replicated_blocks"]],
                ["Safe mode", "ON" if self.nn.safemode("get") else "OFF"],
                ["<a href='/dfsnodelist.jsp?whatNodes=LIVE'>Live Nodes</a>", live],
                ["<a href='/dfsnodelist.jsp?whatNodes=DEAD'>Dead Nodes</a>", len(nodes) - live]]
        return _page("NameNode", _table(["", ""], rows) +
                     "<p><a href='/browseDirectory.jsp?dir=/'>Browse the filesystem</a></p>")

    def nodelist_html(self, what):
        alive = what.upper() == "LIVE"
        rows = [[html.escape(d["id"]), html.escape(d["host"]), html.escape(d["rack"]),
                 d["capacity"], d["used"], d["blocks"], d["decommission"] or "In Service"]
                for d in self.nn.datanode_report() if bool(d["alive"]) == alive]
        return _page(f"{what.capitalize()} Datanodes",
                     _table(["node", "host", "rack", "capacity", "used", "blocks",
                             "admin state"], rows))

    def browse_html(self, q):
        if q.get("filename"):
            f = q["filename"]
            locs = self.nn.get_block_locations(f, 0, 32768)
            from ..dfs.datanode import resolve_datanode
            data = b""
            for b in locs:
                if len(data) >= 32768:
                    break
                for dn in b["dns"]:
                    try:
                        data += resolve_datanode(self.nn, dn).read_block(b["block"], 0,
                                                                          32768 - len(data))
                        break
                    except Exception:  # noqa: BLE001
                        continue
            return _page(f"File: {f}", "<pre>" + html.escape(data.decode("utf-8", "replace"))
                         + "</pre>")
        d = q.get("dir", "/")
        rows = []
        for e in self.nn.list_status(d):
            name = html.escape(e["path"])
            link = (f"<a href='/browseDirectory.jsp?dir={name}'>{name}/</a>" if e["is_dir"] else
                    f"<a href='/browseDirectory.jsp?filename={name}'>{name}</a>")
            rows.append([link, "dir" if e["is_dir"] else "file", e["length"],
                         e.get("replication", 0), e.get("block_size", 0), _fmt_t(e["mtime"])])
        return _page(f"Contents of directory {d}",
                     _table(["name", "type", "size", "replication", "block size",
                             "modification time"], rows))


def maybe_start(jt, conf):
    port = conf.get_int("hbmr.webui.port", 50030)
    if port < 0:
        return None
    try:
        return WebUI(jt, port=port).start()
    except OSError:
        return WebUI(jt, port=0).start()   # port taken: any free port
