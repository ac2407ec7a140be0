"""New-API library classes (hadoop-1.0.3 mapreduce/lib/{input,output,map,reduce,partition})."""
