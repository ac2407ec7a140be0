"""MiniDFSCluster: a NameNode and N DataNodes in this process
(src/test/org/apache/hadoop/hdfs/MiniDFSCluster.java), addressed as
``hdfs://<name>/...``.  DataNode host names can match a LocalCluster's
TaskTracker hosts so split locations drive data-local scheduling."""
from __future__ import annotations

import os
import shutil
import tempfile
import uuid

from .client import DistributedFileSystem, register_namenode, unregister_namenode
from .datanode import DataNode
from .namenode import NameNode


class MiniDFSCluster:
    def __init__(self, conf=None, num_datanodes=3, hosts=None, racks=None, base_dir=None,
                 name=None, serve_rpc=False, format=True):  # noqa: A002
        self.conf = conf
        self.base = base_dir or tempfile.mkdtemp(prefix="hbmr-dfs-")
        self.name = name or f"mini-{uuid.uuid4().hex[:6]}"
        self.name_dir = os.path.join(self.base, "name")
        if format and os.path.exists(self.name_dir):
            shutil.rmtree(self.name_dir)
        self.serve_rpc = serve_rpc
        self.nn = NameNode(conf, self.name_dir)
        self.server = None
        if serve_rpc:
            from ..mapred.rpc import RpcServer
            self.server = RpcServer(self.nn, NameNode.METHODS, host="127.0.0.1").start()
        register_namenode(self.name, self.nn)
        self.datanodes = []
        hosts = hosts or [f"dnhost{i}" for i in range(num_datanodes)]
        racks = racks or ["/default-rack"] * len(hosts)
        for i, (h, r) in enumerate(zip(hosts, racks)):
            self.start_datanode(i, h, r)

    @property
    def uri(self):
        return f"hdfs://{self.name}"

    @property
    def rpc_address(self):
        return f"127.0.0.1:{self.server.port}" if self.server else None

    def start_datanode(self, i, host, rack="/default-rack"):
        dn = DataNode(self.conf, self.nn, f"dn{i}", host, os.path.join(self.base, f"data{i}"),
                      rack, serve_rpc=self.serve_rpc)
        if i < len(self.datanodes):
            self.datanodes[i] = dn
        else:
            self.datanodes.append(dn)
        return dn

    def stop_datanode(self, i):
        self.datanodes[i].shutdown()

    def restart_namenode(self):
        """Stop the NameNode and start a new one from its image + edit log; the
        DataNodes re-register on their next heartbeat and send block reports."""
        self.nn.shutdown()
        self.nn = NameNode(self.conf, self.name_dir)
        register_namenode(self.name, self.nn)
        for dn in self.datanodes:
            dn.nn = self.nn
        return self.nn

    def filesystem(self, host=None):
        return DistributedFileSystem(self.name, self.conf, host=host)

    def shutdown(self):
        for dn in self.datanodes:
            dn.shutdown()
        self.nn.shutdown()
        if self.server is not None:
            self.server.stop()
        unregister_namenode(self.name)
        shutil.rmtree(self.base, ignore_errors=True)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.shutdown()
