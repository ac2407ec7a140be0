"""hbmr DFS: an HDFS-style block file system for one GPU node.

The reference ships HDFS (hadoop-1.0.3/src/hdfs: NameNode, DataNode,
DFSClient, DataTransferProtocol).  hbmr keeps its model —
files as replicated, checksummed blocks with locations the scheduler uses for
data-local map placement — scaled to one node: one DataNode per storage
device (next to each GPU), a NameNode with an edit log + image, and the
``hdfs://`` FileSystem for jobs.

* :mod:`.namenode`  — namespace, edit log / image, block map, placement,
  safe mode, replication monitor, fsck
* :mod:`.datanode`  — block storage with CRC32 chunks, pipelined writes,
  heartbeat commands, block scanner
* :mod:`.client`    — DistributedFileSystem (FileSystem API), DFS streams
* :mod:`.cluster`   — MiniDFSCluster (in-process NameNode + DataNodes)
"""
from .client import DistributedFileSystem, register_namenode, unregister_namenode  # noqa: F401
from .cluster import MiniDFSCluster  # noqa: F401
from .namenode import NameNode, SafeModeException  # noqa: F401
