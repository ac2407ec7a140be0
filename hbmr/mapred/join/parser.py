"""The ``mapred.join.expr`` language (hadoop-1.0.3/src/mapred/org/apache/hadoop/
mapred/join/Parser.java):

    func  ::= <ident>([<func>,]*<func>)
    func  ::= tbl(<class>,"<path>")

``tbl`` nodes wrap an InputFormat over one input path; the other identifiers
are join operators: ``inner``, ``outer``, ``override`` and any user type named
by ``mapred.join.define.<ident>`` (a CompositeRecordReader subclass).  Class
names may be hbmr's (``package.module:Class``) or the reference's Java names
of the formats hbmr provides (``org.apache.hadoop.mapred.SequenceFileInputFormat``).

Parse nodes are composable input formats: ``getSplits`` builds, for a
composite, the i-th CompositeInputSplit from the i-th split of every child
(all children must give the same number: the inputs are partitioned alike);
``getRecordReader`` builds the reader tree for one composite split.
"""
from __future__ import annotations

import re

from ...utils.reflection import load_class, new_instance
from .readers import (InnerJoinRecordReader, OuterJoinRecordReader, OverrideRecordReader,
                      WrappedRecordReader, key_order)

_TOKEN = re.compile(r'\s*(?:(?P<str>"(?:[^"\\]|\\.)*")|(?P<num>-?\d+(?:\.\d*)?)|'
                    r'(?P<ident>[A-Za-z_$][\w$.:]*)|(?P<punct>[(),]))')

COMPOSITE_TYPES = {"inner": InnerJoinRecordReader, "outer": OuterJoinRecordReader,
                   "override": OverrideRecordReader}
WRAPPED_TYPES = {"tbl": WrappedRecordReader}


def tokenize(expr: str):
    pos, out = 0, []
    expr = expr.strip()
    while pos < len(expr):
        m = _TOKEN.match(expr, pos)
        if m is None or m.end() == pos:
            raise ValueError(f"join expression: unexpected {expr[pos:pos + 20]!r}")
        pos = m.end()
        if m.group("str") is not None:
            out.append(("QUOT", m.group("str")[1:-1].replace('\\"', '"')))
        elif m.group("num") is not None:
            out.append(("NUM", float(m.group("num"))))
        elif m.group("ident") is not None:
            out.append(("IDENT", m.group("ident")))
        else:
            out.append((m.group("punct"), m.group("punct")))
    return out


class Node:
    """A parse node: a composable InputFormat."""

    def __init__(self, ident):
        self.ident = ident
        self.id = 0
        self.order = key_order(None)

    def set_id(self, i):
        self.id = i

    def set_key_order(self, order):
        self.order = order


class WNode(Node):
    """``tbl(<InputFormat class>, "<path>")``: one join source."""

    def __init__(self, ident, fmt_cls, path, job):
        super().__init__(ident)
        self.fmt_cls = fmt_cls
        self.inf = new_instance(fmt_cls, job)
        self.indir = path

    def _conf(self, job):
        from ..formats import set_input_paths
        from ..jobconf import JobConf
        c = JobConf(job)
        set_input_paths(c, self.indir)
        return c

    def getSplits(self, job, num_splits):  # noqa: N802
        return list(self.inf.getSplits(self._conf(job), num_splits))

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        rcls = WRAPPED_TYPES[self.ident]
        return rcls(self.id, self.inf.getRecordReader(split, self._conf(job), reporter),
                    self.order)

    def __str__(self):
        name = self.fmt_cls if isinstance(self.fmt_cls, str) else \
            f"{self.fmt_cls.__module__}:{self.fmt_cls.__qualname__}"
        return f'{self.ident}({name},"{self.indir}")'


class CNode(Node):
    """``<op>(<node>, ...)``: a join of its children."""

    def __init__(self, ident, kids, reader_cls):
        super().__init__(ident)
        self.kids = kids
        self.reader_cls = reader_cls
        for i, k in enumerate(kids):
            k.set_id(i)

    def set_key_order(self, order):
        super().set_key_order(order)
        for k in self.kids:
            k.set_key_order(order)

    def getSplits(self, job, num_splits):  # noqa: N802
        from .format import CompositeInputSplit
        per = [k.getSplits(job, num_splits) for k in self.kids]
        for i, s in enumerate(per):
            if len(s) != len(per[0]):
                raise IOError(f"Inconsistent split cardinality from child {i} "
                              f"({len(s)}/{len(per[0])})")
        return [CompositeInputSplit([s[j] for s in per]) for j in range(len(per[0]))]

    def getRecordReader(self, split, job, reporter):  # noqa: N802
        if len(split.splits) != len(self.kids):
            raise IOError(f"split has {len(split.splits)} children, {self} expects "
                          f"{len(self.kids)}")
        kids = [k.getRecordReader(s, job, reporter) for k, s in zip(self.kids, split.splits)]
        return self.reader_cls(self.id, kids, self.order)

    def __str__(self):
        return f"{self.ident}(" + ",".join(str(k) for k in self.kids) + ")"


def _identifiers(job):
    comp = dict(COMPOSITE_TYPES)
    if job is not None:
        pat = re.compile(r"^mapred\.join\.define\.(\w+)$")
        for k, v in job:
            m = pat.match(k)
            if m:
                comp[m.group(1)] = load_class(v)
    return comp


def parse(expr: str, job=None) -> Node:
    """Parse a join expression into its node tree (Parser.parse)."""
    if not expr:
        raise ValueError("mapred.join.expr is not set")
    comp = _identifiers(job)
    toks = tokenize(expr)
    pos = 0

    def expect(kind):
        nonlocal pos
        if pos >= len(toks) or toks[pos][0] != kind:
            got = toks[pos][1] if pos < len(toks) else "end of expression"
            raise ValueError(f"join expression: expected {kind}, got {got!r}")
        pos += 1
        return toks[pos - 1][1]

    def node():
        nonlocal pos
        ident = expect("IDENT")
        expect("(")
        if ident in WRAPPED_TYPES:
            cls = expect("IDENT")
            expect(",")
            path = expect("QUOT")
            expect(")")
            return WNode(ident, cls, path, job)
        if ident not in comp:
            raise ValueError(f"join expression: no node type for {ident!r}")
        kids = [node()]
        while pos < len(toks) and toks[pos][0] == ",":
            pos += 1
            kids.append(node())
        expect(")")
        return CNode(ident, kids, comp[ident])

    root = node()
    if pos != len(toks):
        raise ValueError(f"join expression: trailing {toks[pos][1]!r}")
    cmp = job.get("mapred.join.keycomparator") if job is not None else None
    if cmp:
        root.set_key_order(key_order(new_instance(cmp, job)))
    return root
