"""Record readers of the map-side join framework.

Behaviour of hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/join/
{ComposableRecordReader, WrappedRecordReader, CompositeRecordReader,
JoinRecordReader, InnerJoinRecordReader, OuterJoinRecordReader,
MultiFilterRecordReader, OverrideRecordReader, ResetableIterator,
StreamBackedIterator, ArrayListBackedIterator}.java, as Python readers:

* every source is read in key order (the inputs are sorted and partitioned
  alike — the precondition of a map-side join); a *wrapped* reader looks one
  record ahead and hands all values of the current key to the collector;
* a *composite* reader keeps its children in a heap by (key, id), pops every
  child whose head key is the smallest and emits, for that key, the cross
  product of the children's value lists (the last source varying fastest, as
  the reference's JoinCollector odometer does) filtered by ``combine``:
  inner = every source present, outer = any;
* an *override* reader emits, per key, the values of the rightmost source that
  has it.

A composite reader is itself composable, so joins nest:
``outer(inner(tbl(...),tbl(...)),tbl(...))``.
"""
from __future__ import annotations

import functools
import heapq
import itertools

from ..api import RecordReader
from .tuple import TupleWritable


def key_order(comparator=None):
    """Sort key over join keys: the ``mapred.join.keycomparator`` object
    (``compare(a, b)`` or ``sort_key(k)``), else the keys' natural order."""
    if comparator is None:
        return lambda k: k
    if hasattr(comparator, "sort_key"):
        return comparator.sort_key
    return functools.cmp_to_key(comparator.compare)


# --------------------------------------------------------------------------- iterators
class ResetableIterator:
    """Values of one source for the current key, replayable (the reference's
    ResetableIterator / ArrayListBackedIterator / StreamBackedIterator)."""

    def __init__(self, values=()):
        self.values = list(values)
        self.pos = 0

    def hasNext(self):  # noqa: N802
        return self.pos < len(self.values)

    def next(self):
        v = self.values[self.pos]
        self.pos += 1
        return v

    def add(self, v):
        self.values.append(v)

    def reset(self):
        self.pos = 0

    def clear(self):
        self.values = []
        self.pos = 0

    def __iter__(self):
        return iter(self.values)

    def __len__(self):
        return len(self.values)


ArrayListBackedIterator = ResetableIterator
StreamBackedIterator = ResetableIterator


class JoinCollector:
    """The values of every source for one key (CompositeRecordReader.JoinCollector)."""

    def __init__(self, card):
        self.iters = [None] * card
        self.key = None

    def add(self, i, it: ResetableIterator):
        self.iters[i] = it

    def reset(self, key):
        self.key = key

    def clear(self):
        self.key = None
        self.iters = [None] * len(self.iters)

    def tuples(self):
        """Every combination of one value (or absence) per source; the last
        source varies fastest."""
        lists = [list(it) if it is not None and len(it) else [None] for it in self.iters]
        for combo in itertools.product(*lists):
            yield TupleWritable(combo)


# --------------------------------------------------------------------------- readers
class ComposableRecordReader(RecordReader):
    """A reader that can take part in a join: its records come in key order,
    and it can hand all values of a key to a :class:`JoinCollector`."""

    def __init__(self, rid: int, order):
        self._id = rid
        self.order = order          # sort key over join keys

    def id(self):
        return self._id

    def key(self):
        """The key of the next record (None at the end)."""
        raise NotImplementedError

    def hasNext(self):  # noqa: N802
        return self.key() is not None

    def skip(self, key):
        """Drop records whose key is at or below ``key``."""
        while self.hasNext() and self.order(self.key()) <= self.order(key):
            self._advance_key()

    def accept(self, jc: JoinCollector, key):
        raise NotImplementedError

    def _heap_key(self):
        return (self.order(self.key()), self._id)


class WrappedRecordReader(ComposableRecordReader):
    """A source: an ordinary RecordReader made composable by looking one
    record ahead (WrappedRecordReader.java)."""

    def __init__(self, rid, reader: RecordReader, order):
        super().__init__(rid, order)
        self.rr = reader
        self._head = reader.next()

    def key(self):
        return None if self._head is None else self._head[0]

    def next(self):
        kv = self._head
        if kv is not None:
            self._head = self.rr.next()
        return kv

    def _advance_key(self):
        self.next()

    def accept(self, jc, key):
        it = ResetableIterator()
        ok = self.order(key)
        while self._head is not None and self.order(self._head[0]) == ok:
            it.add(self._head[1])
            self._head = self.rr.next()
        jc.add(self._id, it)

    def getProgress(self):  # noqa: N802
        return self.rr.getProgress()

    def getPos(self):  # noqa: N802
        return self.rr.getPos()

    def close(self):
        self.rr.close()


class CompositeRecordReader(ComposableRecordReader):
    """Joins its children (CompositeRecordReader / JoinRecordReader.java).
    ``next()`` returns (key, TupleWritable) for every combination ``combine``
    accepts; as a child of another composite it contributes, per key, the list
    of those tuples."""

    def __init__(self, rid, kids, order):
        super().__init__(rid, order)
        self.kids = list(kids)
        self.jc = JoinCollector(len(self.kids))
        self._heap = []
        for k in self.kids:
            if k.hasNext():
                heapq.heappush(self._heap, (k._heap_key(), k.id(), k))
        self._pending = iter(())      # tuples of the current key not yet returned
        self._pkey = None
        self._peek = None             # (key, [tuples]) looked ahead for a parent

    def combine(self, srcs, value: TupleWritable) -> bool:
        raise NotImplementedError

    def _fill(self):
        """Collect every child whose head key is the smallest."""
        if not self._heap:
            return None
        hk, _, first = heapq.heappop(self._heap)
        key = first.key()
        ready = [first]
        while self._heap and self._heap[0][0][0] == hk[0]:
            ready.append(heapq.heappop(self._heap)[2])
        self.jc.clear()
        self.jc.reset(key)
        sel = self._select(ready)
        for k in sel:
            k.accept(self.jc, key)
        for k in ready:
            if k not in sel:
                k.skip(key)          # (override: the other sources' values drop)
        for k in ready:
            if k.hasNext():
                heapq.heappush(self._heap, (k._heap_key(), k.id(), k))
        return key

    def _select(self, ready):
        """Children whose values take part for this key (all of them here)."""
        return ready

    def _key_tuples(self):
        """(key, tuples accepted by combine) of the next key that has any."""
        while True:
            key = self._fill()
            if key is None:
                return None
            got = [t for t in self.jc.tuples() if self.combine(self.kids, t)]
            if got:
                return key, got

    def next(self):
        if self._peek is not None:
            self._pkey, tuples = self._peek
            self._peek = None
            self._pending = iter(tuples)
        while True:
            t = next(self._pending, None)
            if t is not None:
                return self._pkey, self.emit(t)
            kt = self._key_tuples()
            if kt is None:
                return None
            self._pkey, tuples = kt
            self._pending = iter(tuples)

    def emit(self, t: TupleWritable):
        return t

    # as the child of another composite: one key at a time
    def key(self):
        if self._peek is None:
            kt = self._key_tuples()
            if kt is None:
                return None
            self._peek = kt
        return self._peek[0]

    def _advance_key(self):
        self.key()
        self._peek = None

    def accept(self, jc, key):
        it = ResetableIterator()
        if self.key() is not None and self.order(self.key()) == self.order(key):
            for t in self._peek[1]:
                it.add(self.emit(t))
            self._peek = None
        jc.add(self._id, it)

    def getProgress(self):  # noqa: N802
        ps = [k.getProgress() for k in self.kids]
        return min(ps) if ps else 1.0

    def close(self):
        for k in self.kids:
            k.close()


class JoinRecordReader(CompositeRecordReader):
    """Base of the joins whose value is the TupleWritable of the sources."""


class InnerJoinRecordReader(JoinRecordReader):
    def combine(self, srcs, value):
        return all(value.has(i) for i in range(len(srcs)))


class OuterJoinRecordReader(JoinRecordReader):
    def combine(self, srcs, value):
        return True


class MultiFilterRecordReader(CompositeRecordReader):
    """A composite that emits one source value per combination
    (MultiFilterRecordReader.java): ``emit`` picks it from the tuple."""

    def combine(self, srcs, value):
        return True

    def emit(self, t):
        raise NotImplementedError


class OverrideRecordReader(MultiFilterRecordReader):
    """Per key, the values of the rightmost source that has it
    (OverrideRecordReader.java: later sources override earlier ones)."""

    def _select(self, ready):
        return [max(ready, key=lambda k: k.id())]

    def emit(self, t):
        for i in range(t.size() - 1, -1, -1):
            if t.has(i):
                return t.get(i)
        return None
