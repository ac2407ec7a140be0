"""Class references by name ("package.module:QualName"), the Python analogue of
Hadoop's ReflectionUtils / Configuration.getClass."""
from __future__ import annotations

import importlib


def class_name(obj) -> str:
    if isinstance(obj, str):
        return obj
    cls = obj if isinstance(obj, type) else type(obj)
    return f"{cls.__module__}:{cls.__qualname__}"


def load_class(name):
    if not isinstance(name, str):
        return name
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
