"""Offline look at the control plane's real request frames (HBMR_RPC_DUMP):
per method the frame count, mean size and the decode cost (msgpack unpack +
TaskTrackerStatus / TaskStatus construction), and the biggest fields of a
tracker status.  usage: python tools/rpc_payloads.py /tmp/rpcd_<pid>.bin"""
import collections
import json
import os
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msgpack  # noqa: E402

from hbmr.mapred import protocol as P  # noqa: E402


def frames(path):
    data = open(path, "rb").read()
    i = 0
    while i + 4 <= len(data):
        (n,) = struct.unpack(">I", data[i:i + 4])
        yield data[i + 4:i + 4 + n]
        i += 4 + n


def main():
    fr = list(frames(sys.argv[1]))
    by = collections.defaultdict(list)
    for b in fr:
        by[msgpack.unpackb(b, raw=False, strict_map_key=False).get("m")].append(b)
    out = {}
    for m, bs in by.items():
        t0 = time.perf_counter()
        objs = [msgpack.unpackb(b, raw=False, strict_map_key=False) for b in bs]
        t1 = time.perf_counter()
        n_st = 0
        for o in objs:
            a = o.get("a") or [None]
            if isinstance(a[0], dict) and "tracker_name" in a[0]:
                st = P.TaskTrackerStatus.from_dict(a[0])
                for r in st.task_reports:
                    P.TaskStatus.from_dict(r)
                n_st += 1
        t2 = time.perf_counter()
        out[m] = {"frames": len(bs), "mean_bytes": round(sum(map(len, bs)) / len(bs)),
                  "unpack_us": round((t1 - t0) / len(bs) * 1e6, 1),
                  "objects_us": round((t2 - t1) / max(1, n_st) * 1e6, 1) if n_st else None}
    print(json.dumps(out, indent=1))
    # field sizes of the biggest report
    rep = max(by.get("report", []) or [b""], key=len)
    if rep:
        st = msgpack.unpackb(rep, raw=False, strict_map_key=False)["a"][0]
        sizes = {k: len(msgpack.packb(v)) for k, v in st.items()}
        print(json.dumps(dict(sorted(sizes.items(), key=lambda kv: -kv[1])[:8])))
        for r in st.get("task_reports", [])[:1]:
            print(json.dumps({k: len(msgpack.packb(v)) for k, v in r.items()}))
            print(json.dumps(r.get("counters"))[:1500])
        for b in st.get("bulk_reports", [])[:1]:
            print(json.dumps({k: len(msgpack.packb(v)) for k, v in b.items()}))


if __name__ == "__main__":
    main()
