"""CPU per call of the control plane's RPC layer (hbmr/mapred/rpc.py): a server
process with a method that returns a reply of the size a tracker's report gets
at 8 ranks (~6 KB of actions) for a ~2 KB request, called by N client threads
(one connection each, as the trackers hold).  Reports the server process's CPU
(user + sys) per call — the part of the JobTracker process's CPU per job that
is RPC rather than scheduling (tools/jt_microbench.py measures that part).

    python tools/rpc_microbench.py --clients 8 --calls 2000
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class Target:
    def __init__(self, reply_bytes):
        self.reply = {"actions": [{"type": "launch_batch", "tasks": [["attempt_x_%04d" % i, i,
                                                                      {"key": "k" * 40}]
                                                                     for i in range(
                                                                         reply_bytes // 80)]}]}

    def report(self, status, assign=False):
        return self.reply


def serve(port_file, reply_bytes):
    from hbmr.mapred.rpc import RpcServer
    srv = RpcServer(Target(reply_bytes), ["report"], host="127.0.0.1", secret=None).start()
    with open(port_file, "w") as f:
        f.write(str(srv.port))
    while True:
        time.sleep(3600)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--reply-bytes", type=int, default=6000)
    ap.add_argument("--serve", default=None)
    a = ap.parse_args()
    if a.serve:
        serve(a.serve, a.reply_bytes)
        return
    import subprocess
    import tempfile

    import psutil

    from hbmr.mapred.rpc import RpcClient
    pf = os.path.join(tempfile.mkdtemp(), "port")
    proc = subprocess.Popen([sys.executable, __file__, "--serve", pf, "--reply-bytes",
                             str(a.reply_bytes)])
    try:
        while not os.path.exists(pf) or not open(pf).read():
            time.sleep(0.05)
        port = int(open(pf).read())
        status = {"tracker_name": "t", "task_reports": [{"attempt_id": "a" * 30, "x": "y" * 200}
                                                         for _ in range(8)]}
        per = a.calls // a.clients

        def client():
            c = RpcClient(f"127.0.0.1:{port}", secret=None)
            for _ in range(per):
                c.call("report", status, True)
        warm = threading.Thread(target=client)
        warm.start()
        warm.join()
        p = psutil.Process(proc.pid)
        c0 = sum(p.cpu_times()[:2])
        t0 = time.perf_counter()
        ths = [threading.Thread(target=client) for _ in range(a.clients)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        wall = time.perf_counter() - t0
        cpu = sum(p.cpu_times()[:2]) - c0
        n = per * a.clients
        print(json.dumps({"clients": a.clients, "calls": n, "reply_bytes": a.reply_bytes,
                          "server_cpu_us_per_call": round(cpu / n * 1e6, 1),
                          "wall_us_per_call": round(wall / n * 1e6, 1)}), flush=True)
    finally:
        proc.kill()


if __name__ == "__main__":
    main()
