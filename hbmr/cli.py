"""``hbmr`` command line (the reference's bin/hadoop, hadoop-1.0.3/bin/hadoop:
jar/pipes/job/fs/version/... dispatch).

  hbmr examples <program> [args]      example programs (ExampleDriver)
  hbmr pipes -input I -output O -cpubin C -gpubin G ...
  hbmr streaming -input I -output O -mapper CMD -reducer CMD ...
  hbmr dumptb PATH | hbmr loadtb PATH   typed bytes out of / into SequenceFiles
  hbmr job -jt host:port -list [all] | -status ID | -kill ID | -counter ID GROUP NAME
           | -tasks ID map|reduce | -history FILE
  hbmr fs -ls|-lsr|-cat|-text|-put|-get|-cp|-mv|-rm|-rmr|-mkdir|-du|-count [-q]|-setrep PATH...
                                      (local paths and hdfs://NAMENODE/... URIs)
  hbmr namenode -dir D [-port P] | datanode -nn HOST:PORT -dir D [-host H]
  hbmr fsck hdfs://NAMENODE/path | dfsadmin -nn NAMENODE -report|-safemode X|...
  hbmr balancer -nn NAMENODE [-threshold PCT] | secondarynamenode -nn NAMENODE -dir D
  hbmr distcp [-update|-overwrite|-delete|-i|-p|-m N] SRC... DST   (file:// / hdfs://)
  hbmr archive -archiveName NAME.har -p PARENT SRC... DEST        (read back as har://)
  hbmr rumen TRACE_OUT TOPOLOGY_OUT HISTORY...                     (job-history traces)
  hbmr logalyzer [-archive -logs URLS] -archiveDir D [-analysis OUT -grep P -sort COLS]
  hbmr distch [-i] PATH:OWNER:GROUP:PERM ...  |  hbmr failmon [--interval S] [--logs GLOB..]
  hbmr gridmix [-generate BYTES] [-jobtype LOADJOB|SLEEPJOB] [-policy REPLAY|STRESS|SERIAL] IOPATH TRACE
  hbmr test TestDFSIO|nnbench|mrbench|testbigmapoutput|threadedmapbench|sortvalidate ...
  hbmr node            start this process's TaskTracker (+ JobTracker on rank 0)
                       under torchrun: one process per GPU
  hbmr run module:function [args]     run a user program (the ``jar`` analogue)
  hbmr version
"""
from __future__ import annotations

import importlib
import json
import os
import shutil
import sys
import time

VERSION = "hbmr 0.1 (Hadoop 1.0.3 API, MI355X / ROCm)"


def _job(argv):
    from .mapred.rpc import RpcClient
    from .utils.tool import GenericOptionsParser
    from .mapred.jobconf import JobConf
    conf = JobConf()
    args = GenericOptionsParser(conf, argv).getRemainingArgs()
    if args and args[0] == "-history":
        from .webui.history import summarize_history
        print(json.dumps(summarize_history(args[1]), indent=1, default=str))
        return 0
    jt = conf.get("mapred.job.tracker")
    if not jt or jt in ("local", "inproc"):
        print("hbmr job needs -jt host:port of a running JobTracker", file=sys.stderr)
        return 2
    rpc = RpcClient(jt)
    if not args:
        print(__doc__, file=sys.stderr)
        return 2
    op = args[0]
    if op == "-list":
        jobs = rpc.call("rpc_list_jobs", len(args) > 1 and args[1] == "all")
        print(f"{len(jobs)} jobs currently running" if len(args) == 1 else f"{len(jobs)} jobs")
        print("JobId\tState\tStartTime\tUserName\tMaps(cpu/gpu)")
        for j in jobs:
            print(f"{j['id']}\t{j['state']}\t{int(j['start'] * 1000)}\t{j['user']}\t"
                  f"{j['maps']}({j['cpu_maps']}/{j['gpu_maps']})")
    elif op == "-status":
        st = rpc.call("rpc_job_status", args[1])
        print(f"Job: {args[1]}\nmap() completion: {st['map_progress']}\n"
              f"reduce() completion: {st['reduce_progress']}\nstate: {st['state']}")
        for g, cs in sorted(st["counters"].items()):
            print(f"\t{g}")
            for n, v in sorted(cs.items()):
                print(f"\t\t{n}={v}")
    elif op == "-kill":
        rpc.call("rpc_kill_job", args[1])
        print(f"Killed job {args[1]}")
    elif op == "-counter":
        st = rpc.call("rpc_job_status", args[1])
        print(st["counters"].get(args[2], {}).get(args[3], 0))
    elif op == "-tasks":
        for t in rpc.call("rpc_task_reports", args[1], args[2] == "map"):
            where = f"gpu{t['device']}" if t["gpu"] else "cpu"
            print(f"{t['task']}\t{t['state']}\t{where}\t{t['tracker']}")
    else:
        print(f"unknown job command {op}", file=sys.stderr)
        return 2
    return 0


def _fs(argv):
    """FsShell over the FileSystem layer: local paths and hdfs:// URIs."""
    from . import fs as F
    from .io import sequencefile as seqf
    if not argv:
        print("hbmr fs -ls|-lsr|-cat|-text|-put|-get|-cp|-mv|-rm|-rmr|-mkdir|-du|-count [-q]|-setrep PATH...",
              file=sys.stderr)
        return 2
    op, paths = argv[0], [p[5:] if p.startswith("file:") and not p.startswith("file://") else p
                          for p in argv[1:]]

    def _walk(p):
        fs = F.get_fs(p)
        st = fs.get_file_status(p)
        if not st.is_dir:
            return [st]
        out = []
        for c in fs.list_status(p, filter_hidden=False):
            out += _walk(c.path) if c.is_dir and op == "-lsr" else [c]
        return out

    def _copy(src, dst):
        if F.isdir(dst):
            dst = os.path.join(dst, os.path.basename(src.rstrip("/")))
        if F.isdir(src):
            F.makedirs(dst)
            for name in F.listdir(src):
                _copy(os.path.join(src, name), os.path.join(dst, name))
            return
        with F.fopen(src, "rb") as fi, F.fopen(dst, "wb") as fo:
            shutil.copyfileobj(fi, fo, 1 << 20)

    if op in ("-ls", "-lsr"):
        for p in paths or ["."]:
            entries = _walk(p)
            print(f"Found {len(entries)} items")
            for st in entries:
                kind = "d" if st.is_dir else "-"
                print(f"{kind}rw-r--r--   1 {st.length:>12} "
                      f"{time.strftime('%Y-%m-%d %H:%M', time.localtime(st.modification_time))} "
                      f"{st.path}")
    elif op == "-cat":
        for p in paths:
            with F.fopen(p, "rb") as f:
                shutil.copyfileobj(f, sys.stdout.buffer)
    elif op == "-text":
        for p in paths:
            with F.fopen(p, "rb") as f:
                magic = f.read(3)
            if magic == b"SEQ":
                with seqf.Reader(p) as r:
                    for k, v in r:
                        print(f"{k}\t{v}")
            else:
                with F.fopen(p, "rb") as f:
                    shutil.copyfileobj(f, sys.stdout.buffer)
    elif op in ("-put", "-copyFromLocal", "-get", "-copyToLocal", "-cp"):
        *srcs, dst = paths
        for src in srcs:
            _copy(src, dst)
    elif op == "-mv":
        if not F.get_fs(paths[0]).rename(paths[0], paths[1]):
            print(f"mv: cannot move {paths[0]}", file=sys.stderr)
            return 1
    elif op in ("-rm", "-rmr"):
        for p in paths:
            if F.isdir(p) and op != "-rmr":
                print(f"rm: cannot remove {p}: Is a directory", file=sys.stderr)
                return 1
            F.get_fs(p).delete(p, recursive=True)
            print(f"Deleted {p}")
    elif op == "-mkdir":
        for p in paths:
            F.makedirs(p)
    elif op in ("-du", "-dus"):
        for p in paths:
            op_ = op
            op = "-lsr"
            tot = sum(st.length for st in _walk(p) if not st.is_dir)
            op = op_
            print(f"{tot}\t{p}")
    elif op == "-count":
        quota = bool(paths) and paths[0] == "-q"
        for p in paths[1:] if quota else paths:
            fs = F.get_fs(p)
            if hasattr(fs, "get_content_summary"):
                c = fs.get_content_summary(p)
            else:
                sts = list(_walk(p))
                c = {"directoryCount": 1 + sum(st.is_dir for st in sts),
                     "fileCount": sum(not st.is_dir for st in sts),
                     "length": sum(st.length for st in sts if not st.is_dir),
                     "quota": -1, "spaceQuota": -1, "spaceConsumed": 0}
            cols = [c["directoryCount"], c["fileCount"], c["length"]]
            if quota:
                qn = c["quota"]
                qs = c["spaceQuota"]
                rem_n = "inf" if qn < 0 else qn - c["directoryCount"] - c["fileCount"]
                rem_s = "inf" if qs < 0 else qs - c["spaceConsumed"]
                cols = ["none" if qn < 0 else qn, rem_n, "none" if qs < 0 else qs, rem_s] + cols
            print("\t".join(str(x) for x in cols + [p]))
    elif op == "-setrep":
        r, p = int(paths[0]), paths[1]
        F.get_fs(p).set_replication(p, r)
        print(f"Replication {r} set: {p}")
    else:
        print(f"{op}: Unknown command", file=sys.stderr)
        return 2
    return 0


def _namenode(argv):
    """hbmr namenode -dir NAME_DIR [-port P]: serve a NameNode over RPC."""
    import argparse
    from .dfs.namenode import NameNode
    from .mapred.jobconf import JobConf
    from .mapred.rpc import RpcServer
    ap = argparse.ArgumentParser(prog="hbmr namenode")
    ap.add_argument("-dir", required=True)
    ap.add_argument("-port", type=int, default=8020)
    a = ap.parse_args(argv)
    nn = NameNode(JobConf(), a.dir)
    srv = RpcServer(nn, NameNode.METHODS, port=a.port).start()
    print(f"NameNode up: hdfs://127.0.0.1:{srv.port}", flush=True)
    try:
        while True:
            time.sleep(1.0)
    except KeyboardInterrupt:
        nn.save_namespace()
    return 0


def _datanode(argv):
    """hbmr datanode -nn HOST:PORT -dir DATA_DIR [-id ID] [-host H] [-rack R]."""
    import argparse
    import socket
    from .dfs.client import RpcProxy
    from .dfs.datanode import DataNode
    from .mapred.jobconf import JobConf
    ap = argparse.ArgumentParser(prog="hbmr datanode")
    ap.add_argument("-nn", required=True)
    ap.add_argument("-dir", required=True)
    ap.add_argument("-id", default=None)
    ap.add_argument("-host", default=socket.gethostname())
    ap.add_argument("-rack", default="/default-rack")
    a = ap.parse_args(argv)
    dn = DataNode(JobConf(), RpcProxy(a.nn), a.id or f"dn-{a.host}-{os.getpid()}", a.host, a.dir,
                  a.rack, serve_rpc=True)
    print(f"DataNode {dn.id} up, serving {dn.server.port}", flush=True)
    try:
        while True:
            time.sleep(1.0)
    except KeyboardInterrupt:
        dn.shutdown()
    return 0


def _fsck(argv):
    from .dfs.client import namenode_for, split_uri
    if not argv:
        print("hbmr fsck hdfs://NAMENODE/path", file=sys.stderr)
        return 2
    auth, path = split_uri(argv[0])
    rep = namenode_for(auth).fsck(path)
    for line in rep.pop("problems", []):
        print(line)
    print(json.dumps(rep, indent=1))
    return 0 if rep["status"] == "HEALTHY" else 1


def _dfsadmin(argv):
    """hbmr dfsadmin -nn AUTH -report | -safemode get|enter|leave | -saveNamespace
    | -decommission DN_ID | -setQuota N PATH.. | -clrQuota PATH.. | -setSpaceQuota BYTES PATH..
    | -clrSpaceQuota PATH.. | -rollEditLog"""
    from .dfs.client import namenode_for
    if len(argv) < 3 or argv[0] != "-nn":
        print(_dfsadmin.__doc__, file=sys.stderr)
        return 2
    nn = namenode_for(argv[1])
    op, rest = argv[2], argv[3:]
    if op == "-report":
        for d in nn.datanode_report():
            print(json.dumps(d))
    elif op == "-safemode":
        print("Safe mode is " + ("ON" if nn.safemode(rest[0] if rest else "get") else "OFF"))
    elif op == "-saveNamespace":
        print("Save namespace " + ("successful" if nn.save_namespace() else "failed"))
    elif op == "-decommission":
        print("Decommission " + ("started" if nn.decommission(rest[0]) else "failed"))
    elif op in ("-setQuota", "-setSpaceQuota"):
        n, paths = int(rest[0]), rest[1:]
        for p in paths:
            cur = nn.get_content_summary(p)
            ns, ds = cur["quota"], cur["spaceQuota"]
            nn.set_quota(p, n if op == "-setQuota" else ns, n if op == "-setSpaceQuota" else ds)
    elif op in ("-clrQuota", "-clrSpaceQuota"):
        for p in rest:
            cur = nn.get_content_summary(p)
            nn.set_quota(p, -1 if op == "-clrQuota" else cur["quota"],
                         -1 if op == "-clrSpaceQuota" else cur["spaceQuota"])
    elif op == "-rollEditLog":
        print(json.dumps(nn.roll_edit_log()))
    else:
        print(_dfsadmin.__doc__, file=sys.stderr)
        return 2
    return 0


def _balancer(argv):
    """hbmr balancer -nn AUTH [-threshold PCT]"""
    import argparse
    from .dfs.balancer import Balancer
    from .dfs.client import namenode_for
    ap = argparse.ArgumentParser(prog="hbmr balancer")
    ap.add_argument("-nn", required=True)
    ap.add_argument("-threshold", type=float, default=10.0)
    a = ap.parse_args(argv)
    b = Balancer(namenode_for(a.nn), a.threshold)
    rc = b.run()
    print(f"Balancing took effect: moved {b.moved_blocks} blocks ({b.moved_bytes} bytes); "
          f"exit status {rc}")
    return 0 if rc > 0 else 1


def _secondarynamenode(argv):
    """hbmr secondarynamenode -nn AUTH -dir CHECKPOINT_DIR [-period S] [-checkpoint]"""
    import argparse
    import time
    from .dfs.client import namenode_for
    from .dfs.secondary import SecondaryNameNode
    ap = argparse.ArgumentParser(prog="hbmr secondarynamenode")
    ap.add_argument("-nn", required=True)
    ap.add_argument("-dir", required=True)
    ap.add_argument("-period", type=float, default=3600.0)
    ap.add_argument("-checkpoint", action="store_true", help="one checkpoint, then exit")
    a = ap.parse_args(argv)
    snn = SecondaryNameNode(namenode_for(a.nn), a.dir, period_s=a.period)
    if a.checkpoint:
        return 0 if snn.do_checkpoint() else 1
    snn.start()
    try:
        while True:
            time.sleep(1.0)
    except KeyboardInterrupt:
        snn.shutdown()
    return 0


def _node(argv):
    import logging
    from .mapred.jobconf import JobConf
    from .mapred.node import Node
    from .utils.tool import GenericOptionsParser
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    conf = JobConf()
    GenericOptionsParser(conf, argv)
    node = Node(conf)
    if node.is_master:
        from .webui.server import maybe_start
        web = maybe_start(node.jt, conf)
        addr = node.server.port if node.server else None
        print(f"JobTracker up (rpc port {addr}, web {web.url if web else 'off'}); Ctrl-C to stop",
              flush=True)
        try:
            while True:
                time.sleep(1.0)
        except KeyboardInterrupt:
            pass
        node.shutdown()
    else:
        node.serve_until_shutdown()
        node.shutdown()
    return 0


def _run(argv):
    target, args = argv[0], argv[1:]
    mod, _, fn = target.partition(":")
    m = importlib.import_module(mod)
    rc = getattr(m, fn or "main")(args)
    return rc or 0


TOOLS = {  # src/tools + contrib commands of bin/hadoop
    "distcp": "hbmr.tools.distcp:main",
    "archive": "hbmr.tools.har:main",
    "rumen": "hbmr.tools.rumen:main",
    "gridmix": "hbmr.tools.gridmix:main",
    "logalyzer": "hbmr.tools.logalyzer:main",
    "distch": "hbmr.tools.distch:main",
    "failmon": "hbmr.utils.failmon:main",
    "isolationrunner": "hbmr.mapred.isolation:main",
    "org.apache.hadoop.mapred.IsolationRunner": "hbmr.mapred.isolation:main",
}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help", "help"):
        print(__doc__)
        return 0 if argv else 1
    cmd, rest = argv[0], argv[1:]
    if cmd == "examples":
        from .examples import driver
        return driver.main(rest)
    if cmd == "pipes":
        from .pipes import submitter
        return submitter.main(rest)
    if cmd == "streaming":
        from . import streaming
        return streaming.main(rest)
    if cmd in ("dumptb", "loadtb"):
        from .streaming import dumptb
        return (dumptb.dump_main if cmd == "dumptb" else dumptb.load_main)(rest)
    if cmd == "job":
        return _job(rest)
    if cmd in ("fs", "dfs"):
        return _fs(rest)
    if cmd == "node":
        return _node(rest)
    if cmd == "namenode":
        return _namenode(rest)
    if cmd == "datanode":
        return _datanode(rest)
    if cmd == "fsck":
        return _fsck(rest)
    if cmd == "dfsadmin":
        return _dfsadmin(rest)
    if cmd == "balancer":
        return _balancer(rest)
    if cmd == "secondarynamenode":
        return _secondarynamenode(rest)
    if cmd in ("run", "jar"):
        return _run(rest)
    if cmd == "test":
        from .benchmarks import driver as bdriver
        return bdriver.main(rest)
    if cmd in TOOLS:
        return _run([TOOLS[cmd], *rest])
    if cmd == "version":
        print(VERSION)
        return 0
    print(f"unknown command {cmd}\n{__doc__}", file=sys.stderr)
    return 1


if __name__ == "__main__":
    sys.exit(main())
