"""Layered key/value configuration with Hadoop XML resources.

Behaviour follows hadoop-1.0.3/src/core/org/apache/hadoop/conf/Configuration.java:
default resources are loaded first (core-default.xml then core-site.xml,
Configuration.java:198-199; JobConf adds mapred-default/mapred-site,
JobConf.java:112-113), later resources override earlier ones unless a property
was marked ``<final>true</final>``, values expand ``${var}`` from other keys or
from the environment, and programmatic ``set`` always wins.

Site files are looked up in ``$HBMR_CONF_DIR`` (or ``$HADOOP_CONF_DIR``).
Deprecated/misspelled keys are mapped to their canonical names; notably the
reference's GPU-runner getter read the typo ``mapred.map.runnner.gpu.class``
while the setter wrote ``mapred.map.runner.gpu.class`` (JobConf.java:977-1002,
SURVEY.md B2) — here both spellings address one key.
"""
from __future__ import annotations

import functools
import getpass
import os
import re
import threading
import xml.etree.ElementTree as ET
from pathlib import Path

from ..utils.reflection import class_name, load_class

_DEFAULTS_DIR = Path(__file__).resolve().parent / "defaults"
_VAR = re.compile(r"\$\{([^}$ ]+)\}")
_MAX_SUBST = 20

DEPRECATED_KEYS = {
    "mapred.map.runnner.gpu.class": "mapred.map.runner.gpu.class",
    "fs.default.name": "fs.defaultFS",
}


def _conf_dir() -> Path | None:
    for var in ("HBMR_CONF_DIR", "HADOOP_CONF_DIR"):
        v = os.environ.get(var)
        if v:
            return Path(v)
    return None



@functools.lru_cache(maxsize=1)
def _login_user():
    """getpass.getuser() once per process (``${user.name}`` in every
    hadoop.tmp.dir lookup called it on each job's hot path)."""
    return getpass.getuser()

class Configuration:
    _default_resources = ["core-default.xml", "core-site.xml"]
    _lock = threading.RLock()

    def __init__(self, other: "Configuration | None" = None, load_defaults: bool = True):
        self._props: dict[str, str] = {}
        self._final: set[str] = set()
        self._overlay: dict[str, str] = {}
        self._resources: list = []
        self.load_defaults = load_defaults
        if other is not None:
            self._props = dict(other._props)
            self._final = set(other._final)
            self._overlay = dict(other._overlay)
            self._resources = list(other._resources)
            self.load_defaults = other.load_defaults
        elif load_defaults:
            self._load_defaults()

    # the layered default resources, shared by every new Configuration: a
    # TaskTracker builds a JobConf per job on the launch path, and re-layering
    # the XML files (two stat()s per resource and a _put per property) cost
    # ~0.4 ms there.  The packaged defaults never change under a running
    # process; site files in the conf dir are keyed by their mtimes.
    _defaults_snap = None   # (key, props, final)

    def _load_defaults(self):
        cdir = _conf_dir()
        site = []
        if cdir is not None:
            for r in self._default_resources:
                try:
                    site.append(os.stat(cdir / r).st_mtime_ns)
                except OSError:
                    site.append(None)
        key = (tuple(self._default_resources), str(cdir), tuple(site))
        snap = Configuration._defaults_snap
        if snap is not None and snap[0] == key:
            self._props = dict(snap[1])
            self._final = set(snap[2])
            return
        for r in self._default_resources:
            self._load_named(r)
        Configuration._defaults_snap = (key, dict(self._props), frozenset(self._final))

    # -- resources -----------------------------------------------------------
    @classmethod
    def add_default_resource(cls, name: str):
        with cls._lock:
            if name not in cls._default_resources:
                cls._default_resources.append(name)

    addDefaultResource = add_default_resource  # noqa: N815

    def _load_named(self, name: str):
        for d in (_DEFAULTS_DIR, _conf_dir()):
            if d is None:
                continue
            p = d / name
            if p.exists():
                self._load_file(p)

    def add_resource(self, resource):
        """Add an XML file path, a dict, or a named resource on the conf path."""
        self._resources.append(resource)
        if isinstance(resource, dict):
            for k, v in resource.items():
                self._put(k, str(v), final=False)
        elif isinstance(resource, (str, Path)) and os.path.exists(str(resource)):
            self._load_file(Path(resource))
        else:
            self._load_named(str(resource))
        # programmatic overrides always win
        self._props.update(self._overlay)

    addResource = add_resource  # noqa: N815

    _parsed: dict = {}   # path -> (mtime_ns, [(name, value, final), ...])

    def _load_file(self, path: Path):
        # parsed XML is cached per (path, mtime): every JobConf() re-layers the
        # default resources, and re-parsing them cost ~1 ms per job
        key = str(path)
        mt = os.stat(key).st_mtime_ns
        hit = Configuration._parsed.get(key)
        if hit is None or hit[0] != mt:
            props = []
            root = ET.parse(key).getroot()
            for prop in root.iter("property"):
                name = prop.findtext("name")
                if not name:
                    continue
                value = prop.findtext("value") or ""
                final = (prop.findtext("final") or "").strip().lower() == "true"
                props.append((name.strip(), value, final))
            hit = (mt, props)
            Configuration._parsed[key] = hit
        for name, value, final in hit[1]:
            self._put(name, value, final)

    def _put(self, name, value, final):
        name = DEPRECATED_KEYS.get(name, name)
        if name in self._final:
            return
        self._props[name] = value
        self._gen += 1
        if final:
            self._final.add(name)

    # -- raw access ----------------------------------------------------------
    def _substitute(self, value):
        if value is None or "${" not in value:
            return value
        for _ in range(_MAX_SUBST):
            m = _VAR.search(value)
            if not m:
                return value
            var = m.group(1)
            rep = os.environ.get(var)
            if rep is None:
                rep = self.get_raw(var)
            if rep is None and var in ("USER", "user.name"):
                rep = _login_user()
            if rep is None:
                return value
            value = value[:m.start()] + rep + value[m.end():]
        raise ValueError(f"variable substitution depth too large: {value}")

    def get_raw(self, name):
        name = DEPRECATED_KEYS.get(name, name)
        return self._props.get(name)

    getRaw = get_raw  # noqa: N815

    def get(self, name, default=None):
        v = self.get_raw(name)
        if v is None:
            return default
        return self._substitute(v)

    #: mutation count (set / unset): lets a reader cache values derived from
    #: this conf (MapOutputBuffer's per-job settings) and see a later change
    _gen = 0

    def set(self, name, value):
        name = DEPRECATED_KEYS.get(name, name)
        v = "" if value is None else (str(value).lower() if isinstance(value, bool) else str(value))
        self._props[name] = v
        self._overlay[name] = v
        self._gen += 1

    def unset(self, name):
        name = DEPRECATED_KEYS.get(name, name)
        self._props.pop(name, None)
        self._overlay.pop(name, None)
        self._gen += 1

    def set_if_unset(self, name, value):
        if self.get_raw(name) is None:
            self.set(name, value)

    setIfUnset = set_if_unset  # noqa: N815

    # -- typed accessors -----------------------------------------------------
    def get_int(self, name, default=0) -> int:
        v = self.get(name)
        if v is None or v.strip() == "":
            return default
        v = v.strip()
        return int(v, 16) if v.lower().startswith(("0x", "-0x")) else int(v)

    getInt = get_int  # noqa: N815
    get_long = get_int
    getLong = get_int  # noqa: N815

    def set_int(self, name, value):
        self.set(name, int(value))

    setInt = set_int  # noqa: N815
    set_long = set_int
    setLong = set_int  # noqa: N815

    def get_float(self, name, default=0.0) -> float:
        v = self.get(name)
        return default if v is None or v.strip() == "" else float(v)

    getFloat = get_float  # noqa: N815

    def set_float(self, name, value):
        self.set(name, float(value))

    setFloat = set_float  # noqa: N815

    def get_boolean(self, name, default=False) -> bool:
        v = self.get(name)
        if v is None:
            return default
        v = v.strip().lower()
        if v == "true":
            return True
        if v == "false":
            return False
        return default

    getBoolean = get_boolean  # noqa: N815

    def set_boolean(self, name, value):
        self.set(name, bool(value))

    setBoolean = set_boolean  # noqa: N815

    def get_strings(self, name, default=None) -> list[str] | None:
        v = self.get(name)
        if v is None:
            return default
        return [s.strip() for s in v.split(",") if s.strip() != ""]

    getStrings = get_strings  # noqa: N815

    def set_strings(self, name, values):
        self.set(name, ",".join(str(v) for v in values))

    setStrings = set_strings  # noqa: N815

    def get_class(self, name, default=None):
        v = self.get(name)
        if v is None or v == "":
            return load_class(default) if default is not None else None
        return load_class(v.strip())

    getClass = get_class  # noqa: N815

    def set_class(self, name, cls):
        if cls is None:
            self.unset(name)
            return
        self.set(name, class_name(cls))

    setClass = set_class  # noqa: N815

    # -- iteration / export ----------------------------------------------------
    def __iter__(self):
        for k in sorted(self._props):
            yield k, self.get(k)

    def __contains__(self, name):
        return self.get_raw(name) is not None

    def __len__(self):
        return len(self._props)

    def items(self):
        return list(iter(self))

    def to_dict(self) -> dict:
        sub = self._substitute
        return {k: (sub(v) if "${" in v else v) for k, v in sorted(self._props.items())}

    def write_xml(self, out):
        root = ET.Element("configuration")
        for k, v in self:
            p = ET.SubElement(root, "property")
            ET.SubElement(p, "name").text = k
            ET.SubElement(p, "value").text = v
            if k in self._final:
                ET.SubElement(p, "final").text = "true"
        data = ET.tostring(root, encoding="unicode")
        text = '<?xml version="1.0"?>\n' + data
        if hasattr(out, "write"):
            out.write(text)
        else:
            Path(out).write_text(text)

    writeXml = write_xml  # noqa: N815

    def copy(self):
        return type(self)(self)

    def __repr__(self):
        return f"{type(self).__name__}({len(self._props)} props)"
