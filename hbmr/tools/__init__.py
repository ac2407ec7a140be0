"""Cluster tools (hadoop-1.0.3/src/tools/org/apache/hadoop/tools/): DistCp,
HadoopArchives (+ the har:// read side), Rumen job traces, Logalyzer, DistCh."""
