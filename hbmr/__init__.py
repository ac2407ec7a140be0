"""hbmr — HBM-resident MapReduce: an MI355X-native GPU MapReduce runtime.

Provides the capabilities of millecker/hadoop-1.0.3-gpu (Hadoop 1.0.3 with
Shirahata et al.'s hybrid CPU/GPU map-task scheduling) re-designed for one node
of 8×MI355X: Hadoop-style JobConf/JobClient/Mapper/Reducer APIs, SequenceFile
I/O, a JobTracker/TaskTracker control plane with CPU and per-GPU map slots and a
profiled CPU-vs-GPU cost model, a Pipes-compatible C++ task bridge, HIP/CDNA4
kernels for the map/combine/sort hot paths and RCCL (xGMI) collectives for the
shuffle.  See SURVEY.md for the blueprint and README.md for usage.
"""

__version__ = "0.1.0"
