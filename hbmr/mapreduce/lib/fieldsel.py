"""New-API field selection (mapreduce/lib/fieldsel/FieldSelectionMapper.java,
FieldSelectionReducer.java, FieldSelectionHelper.java): the same ``key:value``
field specs as mapred.lib.FieldSelectionMapReduce under the new-API keys."""
from __future__ import annotations

from ...io.writable import Text
from ...mapred.lib.fieldsel import java_split, parse_key_value_spec, select_fields
from .. import api

DATA_FIELD_SEPARATOR = "mapreduce.fieldsel.data.field.separator"
MAP_OUTPUT_KEY_VALUE_SPEC = "mapreduce.fieldsel.map.output.key.value.fields.spec"
REDUCE_OUTPUT_KEY_VALUE_SPEC = "mapreduce.fieldsel.reduce.output.key.value.fields.spec"


class FieldSelectionHelper:
    @staticmethod
    def parseOutputKeyValueSpec(spec, key_fields, value_fields):  # noqa: N802
        k, v, from_ = parse_key_value_spec(spec)
        key_fields.extend(k)
        value_fields.extend(v)
        return from_

    @staticmethod
    def extract(key, val, sep, kf, vf, all_from, ignore_key, is_map):
        """(new key, new value) as extractOutputKeyValue: the record is the
        value, prefixed by the key unless ``ignore_key``."""
        line = str(val) if ignore_key else str(key) + str(val)
        fields = java_split(line, sep)
        nk = select_fields(fields, kf, -1, sep)
        nv = select_fields(fields, vf, all_from, sep)
        if is_map and nk is None:
            nk, nv = nv, None
        return Text(nk if nk is not None else ""), Text(nv if nv is not None else "")


class FieldSelectionMapper(api.Mapper):
    def setup(self, context):
        conf = context.getConfiguration()
        self.sep = conf.get(DATA_FIELD_SEPARATOR, "\t")
        self.kf, self.vf = [], []
        self.from_ = FieldSelectionHelper.parseOutputKeyValueSpec(
            conf.get(MAP_OUTPUT_KEY_VALUE_SPEC, "0-:"), self.kf, self.vf)
        fmt = conf.get("mapreduce.inputformat.class") or ""
        self.ignore = fmt == "" or (fmt.endswith("TextInputFormat") and "KeyValue" not in fmt)

    def map(self, key, value, context):
        context.write(*FieldSelectionHelper.extract(key, value, self.sep, self.kf, self.vf,
                                                    self.from_, self.ignore, True))


class FieldSelectionReducer(api.Reducer):
    def setup(self, context):
        conf = context.getConfiguration()
        self.sep = conf.get(DATA_FIELD_SEPARATOR, "\t")
        self.kf, self.vf = [], []
        self.from_ = FieldSelectionHelper.parseOutputKeyValueSpec(
            conf.get(REDUCE_OUTPUT_KEY_VALUE_SPEC, "0-:"), self.kf, self.vf)

    def reduce(self, key, values, context):
        ks = str(key) + self.sep
        for v in values:
            context.write(*FieldSelectionHelper.extract(ks, v, self.sep, self.kf, self.vf,
                                                        self.from_, False, False))
