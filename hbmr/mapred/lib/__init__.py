from .basic import (HashPartitioner, IdentityMapper, IdentityReducer, IntSumReducer,  # noqa: F401
                    InputSampler, InverseMapper, KeyFieldBasedPartitioner, LongSumReducer,
                    RegexMapper, TokenCountMapper, TotalOrderPartitioner)
