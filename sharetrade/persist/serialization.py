"""Deterministic binary serialization of persisted events / snapshots.

Akka persists the reference's ``Event(stockName, HashMap[LocalDate, Double])``
with default Java serialization (a ``proto`` serializer is registered but bound
to nothing, `application.conf:20-24`).  Here every persisted object is encoded
as ``[u16 type-id][body]`` with a fixed little-endian layout and canonical
ordering (map entries sorted by key), so equal values always encode to equal
bytes — the property the journal and checkpoint CRCs rely on.

Built-in codecs: ``None``, bool, int (i64), float (f64), str, bytes, date,
list/tuple, dict (keys sorted by their encoding), registered dataclasses.
"""
from __future__ import annotations

import dataclasses
import datetime as _dt
import struct
from typing import Any, Callable, Dict, Tuple, Type

_T_NONE, _T_BOOL, _T_INT, _T_FLOAT, _T_STR, _T_BYTES, _T_DATE, _T_LIST, _T_DICT, _T_TUPLE = range(10)
_T_USER = 64

_EPOCH = _dt.date(1970, 1, 1)

_registry_by_type: Dict[type, int] = {}
_registry_by_id: Dict[int, Tuple[type, Callable[[Any], Any], Callable[[Any], Any]]] = {}


def register(cls: Type, type_id: int, to_plain: Callable[[Any], Any] = None,
             from_plain: Callable[[Any], Any] = None) -> Type:
    """Register a class under ``type_id`` (>= 64).  Dataclasses default to a
    field-tuple encoding."""
    if type_id < _T_USER:
        raise ValueError("user type ids start at 64")
    if type_id in _registry_by_id and _registry_by_id[type_id][0] is not cls:
        raise ValueError(f"type id {type_id} already registered")
    if to_plain is None:
        if not dataclasses.is_dataclass(cls):
            raise TypeError("non-dataclass types need to_plain/from_plain")
        names = [f.name for f in dataclasses.fields(cls)]
        to_plain = lambda o: tuple(getattr(o, n) for n in names)  # noqa: E731
        from_plain = lambda t: cls(*t)  # noqa: E731
    _registry_by_type[cls] = type_id
    _registry_by_id[type_id] = (cls, to_plain, from_plain)
    return cls


def serializable(type_id: int):
    def deco(cls):
        return register(cls, type_id)
    return deco


def _enc(o: Any, out: bytearray) -> None:
    if o is None:
        out += struct.pack("<H", _T_NONE)
    elif isinstance(o, bool):
        out += struct.pack("<HB", _T_BOOL, int(o))
    elif isinstance(o, int):
        out += struct.pack("<Hq", _T_INT, o)
    elif isinstance(o, float):
        out += struct.pack("<Hd", _T_FLOAT, o)
    elif isinstance(o, str):
        b = o.encode("utf-8")
        out += struct.pack("<HI", _T_STR, len(b)) + b
    elif isinstance(o, (bytes, bytearray, memoryview)):
        b = bytes(o)
        out += struct.pack("<HQ", _T_BYTES, len(b)) + b
    elif isinstance(o, _dt.date) and not isinstance(o, _dt.datetime):
        out += struct.pack("<Hi", _T_DATE, (o - _EPOCH).days)
    elif type(o) in _registry_by_type:
        tid = _registry_by_type[type(o)]
        out += struct.pack("<H", tid)
        _enc(_registry_by_id[tid][1](o), out)
    elif isinstance(o, dict):
        items = [(encode(k), v) for k, v in o.items()]
        items.sort(key=lambda kv: kv[0])
        out += struct.pack("<HI", _T_DICT, len(items))
        for kb, v in items:
            out += kb
            _enc(v, out)
    elif isinstance(o, tuple):
        out += struct.pack("<HI", _T_TUPLE, len(o))
        for v in o:
            _enc(v, out)
    elif isinstance(o, list):
        out += struct.pack("<HI", _T_LIST, len(o))
        for v in o:
            _enc(v, out)
    else:
        # numpy scalars and the like
        try:
            import numpy as np

            if isinstance(o, np.integer):
                return _enc(int(o), out)
            if isinstance(o, np.floating):
                return _enc(float(o), out)
        except ImportError:  # pragma: no cover
            pass
        raise TypeError(f"no serializer for {type(o).__name__}")


def encode(o: Any) -> bytes:
    out = bytearray()
    _enc(o, out)
    return bytes(out)


def _dec(b: memoryview, i: int) -> Tuple[Any, int]:
    (t,) = struct.unpack_from("<H", b, i)
    i += 2
    if t == _T_NONE:
        return None, i
    if t == _T_BOOL:
        return bool(b[i]), i + 1
    if t == _T_INT:
        return struct.unpack_from("<q", b, i)[0], i + 8
    if t == _T_FLOAT:
        return struct.unpack_from("<d", b, i)[0], i + 8
    if t == _T_STR:
        (n,) = struct.unpack_from("<I", b, i)
        i += 4
        return bytes(b[i:i + n]).decode("utf-8"), i + n
    if t == _T_BYTES:
        (n,) = struct.unpack_from("<Q", b, i)
        i += 8
        return bytes(b[i:i + n]), i + n
    if t == _T_DATE:
        (d,) = struct.unpack_from("<i", b, i)
        return _EPOCH + _dt.timedelta(days=d), i + 4
    if t in (_T_LIST, _T_TUPLE):
        (n,) = struct.unpack_from("<I", b, i)
        i += 4
        vals = []
        for _ in range(n):
            v, i = _dec(b, i)
            vals.append(v)
        return (tuple(vals) if t == _T_TUPLE else vals), i
    if t == _T_DICT:
        (n,) = struct.unpack_from("<I", b, i)
        i += 4
        d = {}
        for _ in range(n):
            k, i = _dec(b, i)
            v, i = _dec(b, i)
            d[k] = v
        return d, i
    if t in _registry_by_id:
        cls, _, from_plain = _registry_by_id[t]
        plain, i = _dec(b, i)
        return from_plain(plain), i
    raise ValueError(f"unknown type id {t}")


def decode(data: bytes) -> Any:
    mv = memoryview(data)
    v, i = _dec(mv, 0)
    if i != len(mv):
        raise ValueError(f"trailing bytes: {len(mv) - i}")
    return v
