"""``hbmr`` command line (the reference's bin/hadoop, hadoop-1.0.3/bin/hadoop:
jar/pipes/job/fs/version/... dispatch).

  hbmr examples <program> [args]      example programs (ExampleDriver)
  hbmr pipes -input I -output O -cpubin C -gpubin G ...
  hbmr streaming -input I -output O -mapper CMD -reducer CMD ...
  hbmr job -jt host:port -list [all] | -status ID | -kill ID | -counter ID GROUP NAME
           | -tasks ID map|reduce | -history FILE
  hbmr fs -ls|-cat|-text|-put|-get|-rm|-rmr|-mkdir|-du PATH...
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
    from .io import sequencefile as seqf
    if not argv:
        print("hbmr fs -ls|-cat|-text|-put|-get|-rm|-rmr|-mkdir|-du PATH...", file=sys.stderr)
        return 2
    op, paths = argv[0], [p[5:] if p.startswith("file:") else p for p in argv[1:]]
    if op in ("-ls", "-lsr"):
        for p in paths or ["."]:
            entries = [p] if os.path.isfile(p) else sorted(
                os.path.join(d, f) for d, _s, fs in os.walk(p) for f in fs) if op == "-lsr" \
                else [os.path.join(p, f) for f in sorted(os.listdir(p))]
            print(f"Found {len(entries)} items")
            for e in entries:
                st = os.stat(e)
                kind = "d" if os.path.isdir(e) else "-"
                print(f"{kind}rw-r--r--   1 {st.st_size:>12} "
                      f"{time.strftime('%Y-%m-%d %H:%M', time.localtime(st.st_mtime))} {e}")
    elif op == "-cat":
        for p in paths:
            with open(p, "rb") as f:
                shutil.copyfileobj(f, sys.stdout.buffer)
    elif op == "-text":
        for p in paths:
            with open(p, "rb") as f:
                magic = f.read(3)
            if magic == b"SEQ":
                with seqf.Reader(p) as r:
                    for k, v in r:
                        print(f"{k}\t{v}")
            else:
                with open(p, "rb") as f:
                    shutil.copyfileobj(f, sys.stdout.buffer)
    elif op in ("-put", "-copyFromLocal", "-get", "-copyToLocal", "-cp"):
        *srcs, dst = paths
        for s in srcs:
            if os.path.isdir(s):
                shutil.copytree(s, os.path.join(dst, os.path.basename(s)) if os.path.isdir(dst)
                                else dst)
            else:
                shutil.copy(s, dst)
    elif op == "-mv":
        shutil.move(paths[0], paths[1])
    elif op in ("-rm", "-rmr"):
        for p in paths:
            if os.path.isdir(p):
                if op != "-rmr":
                    print(f"rm: cannot remove {p}: Is a directory", file=sys.stderr)
                    return 1
                shutil.rmtree(p)
            else:
                os.remove(p)
            print(f"Deleted {p}")
    elif op == "-mkdir":
        for p in paths:
            os.makedirs(p, exist_ok=True)
    elif op in ("-du", "-dus"):
        for p in paths:
            tot = sum(os.path.getsize(os.path.join(d, f)) for d, _s, fs in os.walk(p) for f in fs) \
                if os.path.isdir(p) else os.path.getsize(p)
            print(f"{tot}\t{p}")
    else:
        print(f"{op}: Unknown command", file=sys.stderr)
        return 2
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
    if cmd == "job":
        return _job(rest)
    if cmd in ("fs", "dfs"):
        return _fs(rest)
    if cmd == "node":
        return _node(rest)
    if cmd in ("run", "jar"):
        return _run(rest)
    if cmd == "version":
        print(VERSION)
        return 0
    print(f"unknown command {cmd}\n{__doc__}", file=sys.stderr)
    return 1


if __name__ == "__main__":
    sys.exit(main())
