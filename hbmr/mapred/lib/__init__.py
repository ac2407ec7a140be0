from .basic import (HashPartitioner, IdentityMapper, IdentityReducer, IntSumReducer,  # noqa: F401
                    InputSampler, InverseMapper, KeyFieldBasedPartitioner, LongSumReducer,
                    RegexMapper, TokenCountMapper, TotalOrderPartitioner)
from .keyfield import KeyFieldBasedComparator  # noqa: F401,E402
from ...mapreduce.lib.partition import BinaryPartitioner  # noqa: F401,E402  (mapred.lib.BinaryPartitioner)
