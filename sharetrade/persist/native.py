"""ctypes bindings to the host runtime library ``libsharetrade_rt.so``
(`csrc/runtime/*.cpp`: CRC32C, append-only journal, snapshot store,
deterministic checkpoint writer)."""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
RT_LIB_PATH = os.path.join(os.path.dirname(_HERE), "_native", "libsharetrade_rt.so")

_lib: Optional[C.CDLL] = None

REPLAY_CB = C.CFUNCTYPE(C.c_int, C.c_int64, C.c_void_p, C.c_size_t, C.c_void_p)


def available() -> bool:
    return os.path.exists(RT_LIB_PATH)


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(RT_LIB_PATH):
        # the runtime library is pure host C++: build it on demand (g++, seconds)
        import importlib
        import sys

        root = os.path.dirname(os.path.dirname(_HERE))
        if root not in sys.path:
            sys.path.insert(0, root)
        importlib.import_module("build").build_rt()
    L = C.CDLL(RT_LIB_PATH)
    L.st_crc32c.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
    L.st_crc32c.restype = C.c_uint32
    L.st_crc32c_sw.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
    L.st_crc32c_sw.restype = C.c_uint32
    L.st_journal_open.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    L.st_journal_open.restype = C.c_void_p
    L.st_journal_append.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.st_journal_append.restype = C.c_int64
    L.st_journal_append_batch.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.st_journal_append_batch.restype = C.c_int64
    for fn in ("st_journal_highest", "st_journal_deleted_to", "st_journal_truncated_bytes"):
        getattr(L, fn).argtypes = [C.c_void_p]
        getattr(L, fn).restype = C.c_int64
    L.st_journal_delete_to.argtypes = [C.c_void_p, C.c_int64]
    L.st_journal_delete_to.restype = C.c_int
    L.st_journal_replay.argtypes = [C.c_void_p, C.c_int64, C.c_int64, REPLAY_CB, C.c_void_p]
    L.st_journal_replay.restype = C.c_int64
    L.st_journal_sync.argtypes = [C.c_void_p]
    L.st_journal_sync.restype = C.c_int
    L.st_journal_close.argtypes = [C.c_void_p]
    L.st_journal_close.restype = None
    L.st_snapshot_save.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_int64, C.c_void_p, C.c_size_t]
    L.st_snapshot_save.restype = C.c_int
    L.st_snapshot_latest.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64),
                                     C.POINTER(C.c_int64), C.c_char_p, C.c_size_t]
    L.st_snapshot_latest.restype = C.c_int
    L.st_snapshot_read.argtypes = [C.c_char_p, C.c_void_p, C.c_size_t]
    L.st_snapshot_read.restype = C.c_int64
    L.st_snapshot_delete_to.argtypes = [C.c_char_p, C.c_char_p, C.c_int64]
    L.st_snapshot_delete_to.restype = C.c_int
    L.st_ckpt_write.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int),
                                C.POINTER(C.c_int), C.POINTER(C.c_int64), C.POINTER(C.c_void_p),
                                C.POINTER(C.c_uint64), C.c_char_p, C.c_uint64, C.c_int]
    L.st_ckpt_write.restype = C.c_int64
    _lib = L
    return L


def crc32c(data: bytes, init: int = 0) -> int:
    buf = C.create_string_buffer(bytes(data), len(data))
    return int(lib().st_crc32c(buf, len(data), init))


def crc32c_ptr(ptr: int, n: int, init: int = 0) -> int:
    return int(lib().st_crc32c(C.c_void_p(ptr), n, init))


def crc_mask(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF
