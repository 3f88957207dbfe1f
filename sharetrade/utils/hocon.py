"""A HOCON subset reader, so an Akka-style ``application.conf`` configures the engine.

The reference is configured through Typesafe Config (HOCON) auto-loaded from
``application.conf`` (`src/main/resources/application.conf:1-25`, test profile
`src/test/resources/application.conf:1-11`).  Supported here: nested objects, dotted
keys (``a.b.c = 1``), ``=`` / ``:`` / no separator before ``{``, quoted and unquoted
strings, numbers, booleans, ``null``, arrays, ``#`` and ``//`` comments, newline- or
comma-separated fields, and object merging of repeated keys.  Not supported:
substitutions (``${...}``), ``include`` and multi-line strings.

:func:`akka_to_config` maps the Akka keys the reference uses onto :class:`Config`
fields; a ``sharetrade { ... }`` block sets any field directly.
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Tuple

_NUM = re.compile(r"^-?(\d+\.?\d*([eE][-+]?\d+)?|\.\d+)$")


class HoconError(ValueError):
    pass


class _Parser:
    def __init__(self, text: str):
        self.s = text
        self.i = 0

    # ------------------------------------------------------------------ lexing helpers
    def _skip(self, newlines: bool = True) -> None:
        s = self.s
        while self.i < len(s):
            c = s[self.i]
            if c in " \t\r" or (newlines and c in "\n,"):
                self.i += 1
            elif c == "#" or s.startswith("//", self.i):
                while self.i < len(s) and s[self.i] != "\n":
                    self.i += 1
            else:
                break

    def _peek(self) -> str:
        return self.s[self.i] if self.i < len(self.s) else ""

    def _quoted(self) -> str:
        assert self.s[self.i] == '"'
        self.i += 1
        out = []
        while self.i < len(self.s):
            c = self.s[self.i]
            if c == "\\":
                nxt = self.s[self.i + 1]
                out.append({"n": "\n", "t": "\t", '"': '"', "\\": "\\"}.get(nxt, nxt))
                self.i += 2
                continue
            if c == '"':
                self.i += 1
                return "".join(out)
            out.append(c)
            self.i += 1
        raise HoconError("unterminated string")

    def _key(self) -> List[str]:
        parts: List[str] = []
        cur = ""
        while self.i < len(self.s):
            c = self._peek()
            if c == '"':
                cur += self._quoted()
            elif c == ".":
                parts.append(cur)
                cur = ""
                self.i += 1
            elif c in " \t=:{\n\r":
                break
            else:
                cur += c
                self.i += 1
        parts.append(cur.strip())
        if not all(parts):
            raise HoconError(f"bad key near offset {self.i}")
        return parts

    # ------------------------------------------------------------------ grammar
    def parse_root(self) -> Dict[str, Any]:
        self._skip()
        if self._peek() == "{":
            self.i += 1
            obj = self._fields(closing="}")
        else:
            obj = self._fields(closing="")
        self._skip()
        if self.i != len(self.s):
            raise HoconError(f"trailing input at offset {self.i}")
        return obj

    def _fields(self, closing: str) -> Dict[str, Any]:
        obj: Dict[str, Any] = {}
        while True:
            self._skip()
            c = self._peek()
            if closing and c == closing:
                self.i += 1
                return obj
            if not c:
                if closing:
                    raise HoconError("unterminated object")
                return obj
            path = self._key()
            self._skip(newlines=False)
            c = self._peek()
            if c in "=:":
                self.i += 1
                self._skip(newlines=False)
            elif c != "{":
                raise HoconError(f"expected '=', ':' or '{{' after key {'.'.join(path)}")
            val = self._value()
            _set_path(obj, path, val)

    def _value(self) -> Any:
        c = self._peek()
        if c == "{":
            self.i += 1
            return self._fields(closing="}")
        if c == "[":
            self.i += 1
            arr = []
            while True:
                self._skip()
                if self._peek() == "]":
                    self.i += 1
                    return arr
                arr.append(self._value())
        if c == '"':
            return self._quoted()
        start = self.i
        while self.i < len(self.s) and self.s[self.i] not in "\n,}]#":
            if self.s.startswith("//", self.i):
                break
            self.i += 1
        raw = self.s[start:self.i].strip()
        if raw == "":
            raise HoconError(f"missing value at offset {start}")
        if raw in ("true", "yes", "on"):
            return True
        if raw in ("false", "no", "off"):
            return False
        if raw == "null":
            return None
        if _NUM.match(raw):
            return float(raw) if any(ch in raw for ch in ".eE") else int(raw)
        if "${" in raw:
            raise HoconError("substitutions are not supported")
        return raw


def _set_path(obj: Dict[str, Any], path: List[str], val: Any) -> None:
    for k in path[:-1]:
        nxt = obj.get(k)
        if not isinstance(nxt, dict):
            nxt = {}
            obj[k] = nxt
        obj = nxt
    last = path[-1]
    if isinstance(val, dict) and isinstance(obj.get(last), dict):
        _merge_dicts(obj[last], val)
    else:
        obj[last] = val


def _merge_dicts(dst: Dict[str, Any], src: Dict[str, Any]) -> None:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge_dicts(dst[k], v)
        else:
            dst[k] = v


def loads(text: str) -> Dict[str, Any]:
    return _Parser(text).parse_root()


def get(tree: Dict[str, Any], dotted: str, default: Any = None) -> Any:
    cur: Any = tree
    for k in dotted.split("."):
        if not isinstance(cur, dict) or k not in cur:
            return default
        cur = cur[k]
    return cur


_JOURNALS = {"akka.persistence.journal.leveldb": "file", "inmemory-journal": "inmemory",
             "akka.persistence.journal.inmem": "inmemory"}


def akka_to_config(tree: Dict[str, Any]) -> Tuple[Dict[str, Any], List[str]]:
    """(Config overrides as a nested dict, list of recognised-but-ignored keys)."""
    out: Dict[str, Any] = {}
    ignored: List[str] = []
    lvl = get(tree, "akka.loglevel")
    if lvl is not None:
        out.setdefault("log", {})["loglevel"] = str(lvl).upper()
    loggers = get(tree, "akka.loggers")
    if loggers is not None:
        out.setdefault("log", {})["test_listener"] = any("TestEventListener" in str(x) for x in loggers)
    plugin = get(tree, "akka.persistence.journal.plugin")
    if plugin is not None:
        if plugin not in _JOURNALS:
            raise HoconError(f"unsupported journal plugin {plugin!r}")
        out.setdefault("persist", {})["journal_plugin"] = _JOURNALS[plugin]
    d = get(tree, "akka.persistence.journal.leveldb.dir")
    if d is not None:
        out.setdefault("persist", {})["journal_dir"] = str(d)
    d = get(tree, "akka.persistence.snapshot-store.local.dir")
    if d is not None:
        out.setdefault("persist", {})["snapshot_dir"] = str(d)
    for k in ("akka.persistence.journal.leveldb.compaction-intervals", "akka.actor.serializers",
              "akka.persistence.snapshot-store.plugin"):
        if get(tree, k) is not None:
            ignored.append(k)
    own = tree.get("sharetrade")
    if isinstance(own, dict):
        _merge_dicts(out, own)
    return out, ignored
