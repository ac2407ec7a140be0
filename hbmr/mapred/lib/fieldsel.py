"""Field selection: a mapper/reducer that cuts records into fields and
re-assembles a key and a value from chosen fields, like Unix ``cut``
(hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/lib/FieldSelectionMapReduce.java
and mapreduce/lib/fieldsel/FieldSelectionHelper.java).

Spec ``"keyFields:valueFields"``, each a comma list of field numbers, ranges
``n-m`` and open ranges ``n-`` (all fields from n on), e.g. ``"4,3,0,1:6,5,1-3,7-"``.
Fields are split on a separator (``mapred.data.field.separator``, default tab;
a regular expression, as Java's String.split) with Java's trailing-empty-field
removal."""
from __future__ import annotations

import re

from ...io.writable import Text
from ..api import Mapper, Reducer

SEP_KEY = "mapred.data.field.separator"
MAP_SPEC_KEY = "map.output.key.value.fields.spec"
REDUCE_SPEC_KEY = "reduce.output.key.value.fields.spec"


def java_split(s: str, sep: str) -> list[str]:
    """String.split(regex): trailing empty strings removed."""
    parts = re.split(sep, s) if len(sep) != 1 else s.split(sep)
    while parts and parts[-1] == "":
        parts.pop()
    return parts or [""] if s == "" else parts


def extract_fields(spec: list[str], out: list) -> int:
    """Append the listed field numbers to ``out``; return the n of an open
    range ``n-`` (all fields from n on), else -1."""
    all_from = -1
    for f in spec:
        if not f:
            continue
        if "-" not in f:
            out.append(int(f))
            continue
        start, end = f.split("-", 1)
        start = start or "0"
        if not end:
            all_from = int(start)
            continue
        out.extend(range(int(start), int(end) + 1))
    return all_from


def parse_key_value_spec(spec: str):
    """(key fields, value fields, value fields from) of a ``key:value`` spec."""
    kv = spec.split(":")
    keys, vals = [], []
    extract_fields(kv[0].split(","), keys)
    from_ = extract_fields(kv[1].split(",") if len(kv) > 1 else [], vals)
    return keys, vals, from_


def select_fields(fields, field_list, all_from, sep):
    """The selected fields joined by ``sep`` (None if nothing was selected);
    a listed field past the end contributes an empty field."""
    parts = None
    if field_list:
        parts = [fields[i] if i < len(fields) else "" for i in field_list]
    if all_from >= 0:
        parts = (parts or []) + list(fields[all_from:])
    return None if parts is None else sep.join(parts)


class FieldSelectionMapReduce(Mapper, Reducer):
    """Old-API field-selection mapper and reducer.  The map input key is part
    of the record unless the job reads TextInputFormat (whose key is a byte
    offset)."""

    def configure(self, job):
        self.sep = job.get(SEP_KEY, "\t")
        self.map_spec = job.get(MAP_SPEC_KEY, "0-:")
        self.mk, self.mv, self.m_from = parse_key_value_spec(self.map_spec)
        self.red_spec = job.get(REDUCE_SPEC_KEY, "0-:")
        self.rk, self.rv, self.r_from = parse_key_value_spec(self.red_spec)
        fmt = job.get("mapred.input.format.class") or "hbmr.mapred.formats:TextInputFormat"
        self.ignore_key = fmt.endswith("TextInputFormat") and "KeyValue" not in fmt

    def map(self, key, value, output, reporter):
        fields = java_split(str(value), self.sep)
        if not self.ignore_key:
            fields = java_split(str(key), self.sep) + fields
        nk = select_fields(fields, self.mk, -1, self.sep)
        nv = select_fields(fields, self.mv, self.m_from, self.sep)
        if nk is None:
            nk, nv = nv, None
        output.collect(Text(nk or ""), Text(nv or ""))

    def reduce(self, key, values, output, reporter):
        ks = str(key) + self.sep
        for v in values:
            fields = java_split(ks + str(v), self.sep)
            nk = select_fields(fields, self.rk, -1, self.sep)
            nv = select_fields(fields, self.rv, self.r_from, self.sep)
            output.collect(Text(nk or ""), Text(nv or ""))
