"""New-API partitioners (mapreduce/lib/partition/*.java)."""
from __future__ import annotations

from .. import api


class HashPartitioner(api.Partitioner):
    """(key.hashCode() & Integer.MAX_VALUE) % numReduceTasks."""

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        return (key.hash_code() & 0x7FFFFFFF) % num_partitions


class BinaryPartitioner(api.Partitioner):
    """Partition on a byte range of the key's bytes
    (mapreduce/lib/partition/BinaryPartitioner.java): offsets
    ``mapred.binary.partitioner.left.offset`` (default 0) and
    ``.right.offset`` (default -1), negative ones counted from the end;
    hash = WritableComparator.hashBytes over the range."""

    LEFT = "mapred.binary.partitioner.left.offset"
    RIGHT = "mapred.binary.partitioner.right.offset"

    @staticmethod
    def setOffsets(conf, left, right):  # noqa: N802
        conf = conf.getConfiguration() if hasattr(conf, "getConfiguration") else conf
        conf.set_int(BinaryPartitioner.LEFT, left)
        conf.set_int(BinaryPartitioner.RIGHT, right)

    @staticmethod
    def setLeftOffset(conf, off):  # noqa: N802
        conf = conf.getConfiguration() if hasattr(conf, "getConfiguration") else conf
        conf.set_int(BinaryPartitioner.LEFT, off)

    @staticmethod
    def setRightOffset(conf, off):  # noqa: N802
        conf = conf.getConfiguration() if hasattr(conf, "getConfiguration") else conf
        conf.set_int(BinaryPartitioner.RIGHT, off)

    def configure(self, conf):
        self.left = conf.get_int(self.LEFT, 0)
        self.right = conf.get_int(self.RIGHT, -1)

    setConf = configure  # noqa: N815

    @staticmethod
    def _bytes(key) -> bytes:
        if hasattr(key, "get") and isinstance(key.get(), (bytes, bytearray)):
            return bytes(key.get())        # BytesWritable
        if hasattr(key, "bytes"):
            return bytes(key.bytes)        # Text
        return bytes(key)

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        from ...io.writable import hash_bytes
        if not hasattr(self, "left"):
            self.left, self.right = 0, -1
        b = self._bytes(key)
        n = len(b)
        if n == 0:
            return 0
        lo, hi = (self.left + n) % n, (self.right + n) % n
        return (hash_bytes(b[lo:hi + 1]) & 0x7FFFFFFF) % num_partitions


class KeyFieldBasedPartitioner(api.Partitioner):
    """(mapreduce/lib/partition/KeyFieldBasedPartitioner.java)."""

    def configure(self, conf):
        from ...mapred.lib.keyfield import KeyFieldBasedPartitioner as _Old
        self._p = _Old()
        self._p.configure(conf)

    setConf = configure  # noqa: N815

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        return self._p.getPartition(key, value, num_partitions)


from ...mapred.lib.basic import TotalOrderPartitioner, InputSampler  # noqa: E402,F401
from ...mapred.lib.keyfield import KeyFieldBasedComparator  # noqa: E402,F401
