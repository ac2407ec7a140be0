"""New-API library reducers (mapreduce/lib/reduce/*.java)."""
from __future__ import annotations

from ...io.writable import IntWritable, LongWritable
from .. import api


class IntSumReducer(api.Reducer):
    def reduce(self, key, values, context):
        context.write(key, IntWritable(sum(v.get() for v in values)))


class LongSumReducer(api.Reducer):
    def reduce(self, key, values, context):
        context.write(key, LongWritable(sum(v.get() for v in values)))
