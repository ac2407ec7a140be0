"""New-API partitioners (mapreduce/lib/partition/*.java)."""
from __future__ import annotations

from .. import api


class HashPartitioner(api.Partitioner):
    """(key.hashCode() & Integer.MAX_VALUE) % numReduceTasks."""

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        return (key.hash_code() & 0x7FFFFFFF) % num_partitions
