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
        raise KeyError(path)

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


def maybe_start(jt, conf):
    port = conf.get_int("hbmr.webui.port", 50030)
    if port < 0:
        return None
    try:
        return WebUI(jt, port=port).start()
    except OSError:
        return WebUI(jt, port=0).start()   # port taken: any free port
