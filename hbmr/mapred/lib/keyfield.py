"""Unix-sort-style key fields for text keys: the ``-k pos1[,pos2]`` options
(pos = field[.char][n][r]; global -n / -r / -nr) of
hadoop-1.0.3/src/mapred/org/apache/hadoop/mapreduce/lib/partition/
{KeyFieldHelper, KeyFieldBasedComparator, KeyFieldBasedPartitioner}.java and
their old-API twins in mapred/lib.

* KeyFieldBasedComparator (``mapred.text.key.comparator.options``): compares
  the UTF-8 bytes of each key range in turn, lexically or numerically, and
  reversed on ``r``;
* KeyFieldBasedPartitioner (``mapred.text.key.partitioner.options``, or the
  older ``num.key.fields.for.partition``): hashes only the key ranges
  (h = 31·h + signed byte over every range), so records with equal ranges
  meet in one reduce.
Fields are split on ``map.output.key.field.separator`` (default tab)."""
from __future__ import annotations

import re
from decimal import Decimal, InvalidOperation

from ..api import Partitioner

SEP_KEY = "map.output.key.field.separator"
COMPARATOR_OPTIONS = "mapred.text.key.comparator.options"
PARTITIONER_OPTIONS = "mapred.text.key.partitioner.options"


class KeyDescription:
    __slots__ = ("begin_field", "begin_char", "end_field", "end_char", "numeric", "reverse")

    def __init__(self):
        self.begin_field, self.begin_char = 1, 1
        self.end_field, self.end_char = 0, 0
        self.numeric = self.reverse = False

    def __repr__(self):
        return (f"-k{self.begin_field}.{self.begin_char},{self.end_field}.{self.end_char}"
                f"{'n' if self.numeric else ''}{'r' if self.reverse else ''}")


_POS = re.compile(r"^(\d+)(?:\.(\d+))?([nr]*)$")


def _parse_pos(s):
    m = _POS.match(s)
    if m is None:
        raise ValueError("Invalid -k argument. Must be of the form -k pos1,[pos2], where pos "
                         "is of the form f[.c]nr")
    return int(m.group(1)), int(m.group(2) or 0), "n" in m.group(3), "r" in m.group(3)


class KeyFieldHelper:
    def __init__(self, separator="\t"):
        self.sep = separator.encode("utf-8")
        self.specs: list[KeyDescription] = []
        self.seen = False

    def set_key_field_spec(self, start, end):
        """Fields start..end (the ``num.key.fields.for.partition`` form)."""
        if end >= start:
            k = KeyDescription()
            k.begin_field, k.end_field = start, end
            self.specs.append(k)
            self.seen = True

    def parse_option(self, option):
        if not option:
            return
        toks = option.split()
        glob = KeyDescription()
        i = 0
        while i < len(toks):
            t = toks[i]
            if t in ("-n", "-nr", "-rn"):
                glob.numeric = True
            if t in ("-r", "-nr", "-rn"):
                glob.reverse = True
            if t.startswith("-k"):
                arg = t[2:]
                if not arg and i + 1 < len(toks):
                    i += 1
                    arg = toks[i]
                if arg:
                    k = KeyDescription()
                    first, _, second = arg.partition(",")
                    k.begin_field, c, n1, r1 = _parse_pos(first)
                    k.begin_char = c or 1
                    k.numeric, k.reverse = n1, r1
                    if second:
                        k.end_field, k.end_char, n2, r2 = _parse_pos(second)
                        k.numeric |= n2
                        k.reverse |= r2
                    self.specs.append(k)
                    self.seen = True
            i += 1
        for k in self.specs:
            if not (k.reverse or k.numeric):
                k.reverse, k.numeric = glob.reverse, glob.numeric
        if not self.specs:
            self.specs.append(glob)

    # -- byte ranges -------------------------------------------------------------------
    def word_lengths(self, b: bytes):
        """[field count, len(field 1), len(field 2), ...] (KeyFieldHelper.getWordLengths)."""
        if not self.seen:
            return [1]
        parts = b.split(self.sep)     # (a trailing separator makes an empty last field)
        return [len(parts)] + [len(p) for p in parts]

    def start_offset(self, b, lens, k):
        if lens[0] >= k.begin_field:
            pos = sum(lens[i] + len(self.sep) for i in range(1, k.begin_field))
            if pos + k.begin_char <= len(b):
                return pos + k.begin_char - 1
        return -1

    def end_offset(self, b, lens, k):
        if k.end_field == 0:
            return len(b) - 1
        if lens[0] >= k.end_field:
            pos = sum(lens[i] + len(self.sep) for i in range(1, k.end_field))
            if k.end_char == 0:
                pos += lens[k.end_field]
            if pos + k.end_char <= len(b):
                return pos + k.end_char - 1
        return len(b) - 1


def _key_bytes(key) -> bytes:
    if hasattr(key, "bytes") and isinstance(key.bytes, (bytes, bytearray)):
        return bytes(key.bytes)
    return str(key).encode("utf-8")


_NUM = re.compile(rb"^-?\d*(?:\.\d*)?")


def _number(b: bytes) -> Decimal:
    m = _NUM.match(b)
    s = m.group(0).decode() if m else ""
    if s in ("", "-", ".", "-."):
        return Decimal(0)
    try:
        return Decimal(s)
    except InvalidOperation:
        return Decimal(0)


def _cmp(a, b):
    return (a > b) - (a < b)


class KeyFieldBasedComparator:
    """Sort comparator over Text keys (``sort_key`` for the runtime's sort,
    ``compare`` for RawComparator users)."""

    def __init__(self, job=None):
        self.helper = None
        if job is not None:
            self.configure(job)

    def configure(self, job):
        self.helper = KeyFieldHelper(job.get(SEP_KEY, "\t"))
        self.helper.parse_option(job.get(COMPARATOR_OPTIONS))

    def _ensure(self):
        if self.helper is None:
            self.helper = KeyFieldHelper()

    def compare_bytes(self, b1: bytes, b2: bytes) -> int:
        self._ensure()
        h = self.helper
        if not h.specs:
            return _cmp(b1, b2)
        l1, l2 = h.word_lengths(b1), h.word_lengths(b2)
        for k in h.specs:
            s1, s2 = h.start_offset(b1, l1, k), h.start_offset(b2, l2, k)
            if s1 < 0 or s2 < 0:
                if s1 < 0 and s2 < 0:
                    r = -1          # (as the reference: the first absent side is smaller)
                else:
                    r = -1 if s1 < 0 else 1
                return -r if k.reverse else r
            e1, e2 = h.end_offset(b1, l1, k), h.end_offset(b2, l2, k)
            x, y = b1[s1:e1 + 1], b2[s2:e2 + 1]
            r = _cmp(_number(x), _number(y)) if k.numeric else _cmp(x, y)
            if k.reverse:
                r = -r
            if r:
                return r
        return 0

    def compare(self, a, b) -> int:
        return self.compare_bytes(_key_bytes(a), _key_bytes(b))

    def sort_key(self, raw: bytes):
        """Sort key of a serialised Text key (the runtime sorts serialised keys)."""
        from ...io.vint import decode_vint_size
        n = decode_vint_size(raw[0]) if raw else 0
        return _Keyed(self, raw[n:])


class _Keyed:
    __slots__ = ("c", "b")

    def __init__(self, c, b):
        self.c, self.b = c, b

    def __lt__(self, o):
        return self.c.compare_bytes(self.b, o.b) < 0

    def __eq__(self, o):
        return self.c.compare_bytes(self.b, o.b) == 0

    def __le__(self, o):
        return self.c.compare_bytes(self.b, o.b) <= 0

    def __gt__(self, o):
        return self.c.compare_bytes(self.b, o.b) > 0

    def __ge__(self, o):
        return self.c.compare_bytes(self.b, o.b) >= 0

    def __hash__(self):
        return hash(self.b)


def _java_string_hash(s: str) -> int:
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        for u in ([ord(ch)] if ord(ch) < 0x10000 else
                  [0xD800 + ((ord(ch) - 0x10000) >> 10), 0xDC00 + ((ord(ch) - 0x10000) & 0x3FF)]):
            h = (31 * h + u) & 0xFFFFFFFF
    return h - (1 << 32) if h & 0x80000000 else h


class KeyFieldBasedPartitioner(Partitioner):
    def configure(self, job):
        self.helper = KeyFieldHelper(job.get(SEP_KEY, "\t"))
        n = job.get_int("num.key.fields.for.partition", 0)
        if n > 0:
            self.helper.set_key_field_spec(1, n)
        else:
            self.helper.parse_option(job.get(PARTITIONER_OPTIONS))

    def getPartition(self, key, value, num_partitions):  # noqa: N802
        if not hasattr(self, "helper"):
            self.helper = KeyFieldHelper()
        h = self.helper
        if not h.specs or not h.seen:
            return (_java_string_hash(str(key)) & 0x7FFFFFFF) % num_partitions
        b = str(key).encode("utf-8")
        if not b:
            return 0
        lens = h.word_lengths(b)
        cur = 0
        for k in h.specs:
            s = h.start_offset(b, lens, k)
            if s < 0:
                continue
            e = h.end_offset(b, lens, k)
            for x in b[s:e + 1]:
                cur = (31 * cur + (x - 256 if x > 127 else x)) & 0xFFFFFFFF
        if cur & 0x80000000:
            cur -= 1 << 32
        return (cur & 0x7FFFFFFF) % num_partitions
