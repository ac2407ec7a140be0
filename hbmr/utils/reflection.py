"""Class references by name ("package.module:QualName"), the Python analogue of
Hadoop's ReflectionUtils / Configuration.getClass."""
from __future__ import annotations

import importlib


def class_name(obj) -> str:
    if isinstance(obj, str):
        return obj
    cls = obj if isinstance(obj, type) else type(obj)
    return f"{cls.__module__}:{cls.__qualname__}"


# the reference's class names of the formats/writables/partitioners hbmr
# provides, so configurations and join expressions written for Hadoop resolve
JAVA_ALIASES = {
    "org.apache.hadoop.mapred.TextInputFormat": "hbmr.mapred.formats:TextInputFormat",
    "org.apache.hadoop.mapred.KeyValueTextInputFormat":
        "hbmr.mapred.formats:KeyValueTextInputFormat",
    "org.apache.hadoop.mapred.SequenceFileInputFormat":
        "hbmr.mapred.formats:SequenceFileInputFormat",
    "org.apache.hadoop.mapred.SequenceFileAsTextInputFormat":
        "hbmr.mapred.formats:SequenceFileAsTextInputFormat",
    "org.apache.hadoop.mapred.SequenceFileAsBinaryInputFormat":
        "hbmr.mapred.formats:SequenceFileAsBinaryInputFormat",
    "org.apache.hadoop.mapred.SequenceFileInputFilter":
        "hbmr.mapred.formats:SequenceFileInputFilter",
    "org.apache.hadoop.mapred.lib.NLineInputFormat": "hbmr.mapred.formats:NLineInputFormat",
    "org.apache.hadoop.mapred.TextOutputFormat": "hbmr.mapred.formats:TextOutputFormat",
    "org.apache.hadoop.mapred.SequenceFileOutputFormat":
        "hbmr.mapred.formats:SequenceFileOutputFormat",
    "org.apache.hadoop.mapred.SequenceFileAsBinaryOutputFormat":
        "hbmr.mapred.formats:SequenceFileAsBinaryOutputFormat",
    "org.apache.hadoop.mapred.MapFileOutputFormat": "hbmr.mapred.formats:MapFileOutputFormat",
    "org.apache.hadoop.mapred.lib.NullOutputFormat": "hbmr.mapred.formats:NullOutputFormat",
    "org.apache.hadoop.mapred.join.CompositeInputFormat":
        "hbmr.mapred.join.format:CompositeInputFormat",
    "org.apache.hadoop.mapred.join.TupleWritable": "hbmr.mapred.join.tuple:TupleWritable",
    "org.apache.hadoop.mapred.lib.IdentityMapper": "hbmr.mapred.lib.basic:IdentityMapper",
    "org.apache.hadoop.mapred.lib.IdentityReducer": "hbmr.mapred.lib.basic:IdentityReducer",
    "org.apache.hadoop.mapred.lib.HashPartitioner": "hbmr.mapred.lib.basic:HashPartitioner",
    "org.apache.hadoop.mapred.lib.BinaryPartitioner": "hbmr.mapreduce.lib.partition:BinaryPartitioner",
    "org.apache.hadoop.mapred.lib.KeyFieldBasedPartitioner":
        "hbmr.mapred.lib.keyfield:KeyFieldBasedPartitioner",
    "org.apache.hadoop.mapred.lib.KeyFieldBasedComparator":
        "hbmr.mapred.lib.keyfield:KeyFieldBasedComparator",
    "org.apache.hadoop.mapred.lib.FieldSelectionMapReduce":
        "hbmr.mapred.lib.fieldsel:FieldSelectionMapReduce",
    "org.apache.hadoop.io.Text": "hbmr.io.writable:Text",
    "org.apache.hadoop.io.IntWritable": "hbmr.io.writable:IntWritable",
    "org.apache.hadoop.io.LongWritable": "hbmr.io.writable:LongWritable",
    "org.apache.hadoop.io.BytesWritable": "hbmr.io.writable:BytesWritable",
    "org.apache.hadoop.io.NullWritable": "hbmr.io.writable:NullWritable",
}


_LOADED: dict = {}


def load_class(name):
    """A class (or function) by ``module:Qual.name`` / dotted name / Java alias.
    Resolved names are memoised (a task resolves a few dozen class keys; the
    import machinery costs ~30 µs per lookup even for loaded modules)."""
    if not isinstance(name, str):
        return name
    hit = _LOADED.get(name)
    if hit is not None:
        return hit
    obj = _resolve(name)
    if len(_LOADED) < 4096:
        _LOADED[name] = obj
    return obj


def _resolve(name):
    name = JAVA_ALIASES.get(name.strip(), name)
    if ":" in name:
        mod, qual = name.split(":", 1)
    else:
        mod, _, qual = name.rpartition(".")
    m = importlib.import_module(mod)
    obj = m
    for part in qual.split("."):
        obj = getattr(obj, part)
    return obj


def new_instance(cls_or_name, conf=None):
    """ReflectionUtils.newInstance: construct and configure() if supported."""
    cls = load_class(cls_or_name)
    obj = cls()
    if conf is not None:
        for hook in ("configure", "setConf"):
            fn = getattr(obj, hook, None)
            if callable(fn):
                fn(conf)
                break
    return obj
