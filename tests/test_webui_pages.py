"""The remaining webapps/job JSP pages and the NameNode web UI (webapps/hdfs)."""
from __future__ import annotations

import os
import urllib.request

from hbmr.dfs import MiniDFSCluster
from hbmr.examples.sleepjob import sleep_job_conf
from hbmr.mapred import JobClient, JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.webui.server import DFSWebUI, WebUI


def test_job_pages(tmp_path):
    conf = JobConf()
    conf.set("hbmr.history.dir", str(tmp_path / "hist"))
    conf.set("mapred.queue.names", "default,prod")
    with LocalCluster(conf, num_trackers=2, cpu_slots=2) as cl:
        job = sleep_job_conf(maps=3, reduces=1, map_ms=1, reduce_ms=1, base=conf)
        job.set("mapred.job.queue.name", "prod")
        rj = JobClient.runJob(job, cluster=cl, verbose=False)
        jid = str(rj.getID())
        ui = WebUI(cl.jt, host="127.0.0.1", port=0)
        _, page = ui.route("/jobconf.jsp", {"jobid": jid})
        assert "sleep.job.map.sleep.time" in page
        _, page = ui.route("/jobtasks.jsp", {"jobid": jid, "type": "map", "state": "completed"})
        assert page.count("taskdetails.jsp") == 3
        tip = str(cl.jt.jobs[jid].maps[0].tid)
        _, page = ui.route("/taskdetails.jsp", {"jobid": jid, "tipid": tip})
        assert "SUCCEEDED" in page and "tracker_" in page
        _, page = ui.route("/jobfailures.jsp", {"jobid": jid})
        assert "no failures" in page
        _, page = ui.route("/machines.jsp", {})
        assert "tracker_0" in page and "tracker_1" in page
        _, page = ui.route("/jobqueue_details.jsp", {"queueName": "prod"})
        assert jid in page
        _, page = ui.route("/jobhistory.jsp", {})
        assert f"{jid}.jsonl" in page
        _, page = ui.route("/jobhistory.jsp", {"logFile": f"{jid}.jsonl"})
        assert "Diagnosis" in page
        ui.start()
        try:
            with urllib.request.urlopen(f"{ui.url}jobtasks.jsp?jobid={jid}&type=reduce") as r:
                assert r.status == 200 and b"taskdetails" in r.read()
        finally:
            ui.stop()


def test_namenode_pages(tmp_path):
    with MiniDFSCluster(num_datanodes=2, base_dir=str(tmp_path / "dfs")) as dfs:
        fs = dfs.filesystem()
        with fs.create(f"{dfs.uri}/docs/readme.txt") as f:
            f.write(b"hello <hdfs>\n")
        ui = DFSWebUI(dfs.nn, host="127.0.0.1", port=0)
        _, page = ui.route("/dfshealth.jsp", {})
        assert "Live Nodes" in page and "Safe mode" in page
        _, page = ui.route("/dfsnodelist.jsp", {"whatNodes": "LIVE"})
        assert page.count("In Service") == 2
        _, page = ui.route("/browseDirectory.jsp", {"dir": "/docs"})
        assert "/docs/readme.txt" in page
        _, page = ui.route("/browseDirectory.jsp", {"filename": "/docs/readme.txt"})
        assert "hello &lt;hdfs&gt;" in page
        assert os.path.isdir(tmp_path / "dfs")
