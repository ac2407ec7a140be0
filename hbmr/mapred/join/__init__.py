"""Map-side joins over sorted, identically partitioned inputs
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/join/, 2,551 LoC of Java):
CompositeInputFormat + the ``mapred.join.expr`` parser, the inner / outer /
override join readers and TupleWritable."""
from .format import CompositeInputFormat, CompositeInputSplit
from .parser import CNode, Node, WNode, parse, tokenize
from .readers import (ArrayListBackedIterator, ComposableRecordReader, CompositeRecordReader,
                      InnerJoinRecordReader, JoinCollector, JoinRecordReader,
                      MultiFilterRecordReader, OuterJoinRecordReader, OverrideRecordReader,
                      ResetableIterator, StreamBackedIterator, WrappedRecordReader)
from .tuple import TupleWritable

__all__ = ["CompositeInputFormat", "CompositeInputSplit", "CNode", "Node", "WNode", "parse",
           "tokenize", "ArrayListBackedIterator", "ComposableRecordReader",
           "CompositeRecordReader", "InnerJoinRecordReader", "JoinCollector",
           "JoinRecordReader", "MultiFilterRecordReader", "OuterJoinRecordReader",
           "OverrideRecordReader", "ResetableIterator", "StreamBackedIterator",
           "WrappedRecordReader", "TupleWritable"]
