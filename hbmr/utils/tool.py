"""Tool / ToolRunner / GenericOptionsParser (hadoop-1.0.3 core/org/apache/hadoop/util/
{Tool,ToolRunner,GenericOptionsParser}.java).

Generic options, parsed before a tool's own arguments:
  -D key=value   set a configuration property (repeatable)
  -conf file     add an XML configuration resource
  -jt host:port  set mapred.job.tracker ("local" for the LocalJobRunner)
  -fs uri        set fs.default.name
  -files a,b     files for the DistributedCache (mapred.cache.files)
  -archives a,b  archives for the DistributedCache (mapred.cache.archives)
  -libjars a,b   accepted for compatibility (python modules are imported normally)
"""
from __future__ import annotations

import os


class GenericOptionsParser:
    def __init__(self, conf, args):
        self.conf = conf
        self.remaining = self._parse(list(args))

    def _parse(self, args):
        out = []
        i = 0
        while i < len(args):
            a = args[i]
            nxt = args[i + 1] if i + 1 < len(args) else None
            if a == "-D" and nxt is not None:
                k, _, v = nxt.partition("=")
                self.conf.set(k, v)
                i += 2
            elif a.startswith("-D") and "=" in a:
                k, _, v = a[2:].partition("=")
                self.conf.set(k, v)
                i += 1
            elif a == "-conf" and nxt is not None:
                self.conf.add_resource(nxt)
                i += 2
            elif a == "-jt" and nxt is not None:
                self.conf.set("mapred.job.tracker", nxt)
                i += 2
            elif a == "-fs" and nxt is not None:
                self.conf.set("fs.default.name", nxt)
                i += 2
            elif a in ("-files", "-archives", "-libjars") and nxt is not None:
                key = {"-files": "mapred.cache.files", "-archives": "mapred.cache.archives",
                       "-libjars": "tmpjars"}[a]
                vals = [os.path.abspath(p) for p in nxt.split(",") if p]
                old = self.conf.get(key)
                self.conf.set(key, ",".join(([old] if old else []) + vals))
                i += 2
            else:
                out.append(a)
                i += 1
        return out

    def getRemainingArgs(self):  # noqa: N802
        return list(self.remaining)

    def getConfiguration(self):  # noqa: N802
        return self.conf


class Tool:
    """run(args) -> int exit code; conf via setConf/getConf (Configured)."""

    conf = None

    def setConf(self, conf):  # noqa: N802
        self.conf = conf

    def getConf(self):  # noqa: N802
        return self.conf

    def run(self, args) -> int:
        raise NotImplementedError


class ToolRunner:
    @staticmethod
    def run(conf, tool: Tool, args) -> int:
        from ..mapred.jobconf import JobConf
        if conf is None:
            conf = JobConf()
        parser = GenericOptionsParser(conf, args)
        tool.setConf(conf)
        return tool.run(parser.getRemainingArgs())
