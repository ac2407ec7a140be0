"""Benchmarks and validators from the reference's test tree (AllTestDriver in
hadoop-1.0.3/src/test/org/apache/hadoop/test/AllTestDriver.java): TestDFSIO,
NNBench, MRBench, SortValidator, BigMapOutput, ThreadedMapBenchmark.
``hbmr test <program> [args]`` runs them."""
