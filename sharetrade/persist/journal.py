"""Journal and snapshot-store plugins.

Mirrors Akka Persistence's plugin split configured in the reference
(`src/main/resources/application.conf:5-18` — LevelDB journal at
``target/my/journal``, local snapshot store at ``target/my/snapshots``; the test
profile swaps in in-memory plugins, `src/test/resources/application.conf:7-10`):

* :class:`FileJournal` / :class:`LocalSnapshotStore` — the native C++ store
  (`csrc/runtime/journal.cpp`): CRC32C-framed append-only records, torn-write
  truncation on recovery, atomic snapshot publication;
* :class:`InMemoryJournal` / :class:`InMemorySnapshotStore` — process-global
  dictionaries with ``clear()`` (the ``InMemoryCleanup`` trait of
  `QDecisionPolicyActorSpec.scala:75-87`).

Payloads are encoded with :mod:`sharetrade.persist.serialization`.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

from . import native, serialization


@dataclass(frozen=True)
class SnapshotMetadata:
    persistence_id: str
    sequence_nr: int
    timestamp: int


@dataclass(frozen=True)
class SelectedSnapshot:
    metadata: SnapshotMetadata
    snapshot: Any


class Journal:
    def append(self, pid: str, events: List[Any]) -> int:
        raise NotImplementedError

    def replay(self, pid: str, from_seq: int = 1, to_seq: int = -1) -> List[Tuple[int, Any]]:
        raise NotImplementedError

    def highest_sequence_nr(self, pid: str) -> int:
        raise NotImplementedError

    def delete_to(self, pid: str, seq: int) -> None:
        raise NotImplementedError

    def close(self) -> None:
        pass


class SnapshotStore:
    def save(self, pid: str, seq: int, snapshot: Any, timestamp: Optional[int] = None) -> SnapshotMetadata:
        raise NotImplementedError

    def load_latest(self, pid: str, max_seq: int = -1) -> Optional[SelectedSnapshot]:
        raise NotImplementedError

    def delete_to(self, pid: str, max_seq: int) -> int:
        raise NotImplementedError


# ---------------------------------------------------------------------- native file plugins
class FileJournal(Journal):
    """One ``<pid>.journal`` file per persistence id under ``directory``."""

    def __init__(self, directory: str, fsync: bool = False):
        self.dir = directory
        self.fsync = fsync
        self._handles: Dict[str, int] = {}
        self._lock = threading.Lock()

    def _h(self, pid: str) -> int:
        with self._lock:
            h = self._handles.get(pid)
            if h is None:
                h = native.lib().st_journal_open(self.dir.encode(), _safe(pid).encode(), int(self.fsync))
                if not h:
                    raise OSError(f"cannot open journal {self.dir}/{pid}")
                self._handles[pid] = h
            return h

    def append(self, pid: str, events: List[Any]) -> int:
        h = self._h(pid)
        blobs = [serialization.encode(e) for e in events]
        bufs = [C.create_string_buffer(b, len(b)) for b in blobs]
        ptrs = (C.c_void_p * len(bufs))(*[C.cast(b, C.c_void_p) for b in bufs])
        sizes = (C.c_size_t * len(bufs))(*[len(b) for b in blobs])
        r = native.lib().st_journal_append_batch(h, len(bufs), ptrs, sizes)
        if r < 0:
            raise OSError("journal append failed")
        return int(r)

    def replay(self, pid: str, from_seq: int = 1, to_seq: int = -1) -> List[Tuple[int, Any]]:
        h = self._h(pid)
        out: List[Tuple[int, Any]] = []

        def cb(seq, ptr, n, _user):
            out.append((int(seq), serialization.decode(C.string_at(ptr, n))))
            return 0

        r = native.lib().st_journal_replay(h, from_seq, to_seq, native.REPLAY_CB(cb), None)
        if r < 0:
            raise OSError("journal replay failed")
        return out

    def highest_sequence_nr(self, pid: str) -> int:
        return int(native.lib().st_journal_highest(self._h(pid)))

    def truncated_bytes(self, pid: str) -> int:
        return int(native.lib().st_journal_truncated_bytes(self._h(pid)))

    def delete_to(self, pid: str, seq: int) -> None:
        if native.lib().st_journal_delete_to(self._h(pid), seq) != 0:
            raise OSError("journal delete failed")

    def close(self) -> None:
        with self._lock:
            for h in self._handles.values():
                native.lib().st_journal_close(h)
            self._handles.clear()


class LocalSnapshotStore(SnapshotStore):
    def __init__(self, directory: str):
        self.dir = directory

    def save(self, pid: str, seq: int, snapshot: Any, timestamp: Optional[int] = None) -> SnapshotMetadata:
        ts = int(time.time() * 1000) if timestamp is None else int(timestamp)
        b = serialization.encode(snapshot)
        if native.lib().st_snapshot_save(self.dir.encode(), _safe(pid).encode(), seq, ts, b, len(b)) != 0:
            raise OSError("snapshot save failed")
        return SnapshotMetadata(pid, seq, ts)

    def load_latest(self, pid: str, max_seq: int = -1) -> Optional[SelectedSnapshot]:
        L = native.lib()
        s, t = C.c_int64(), C.c_int64()
        path = C.create_string_buffer(4096)
        r = L.st_snapshot_latest(self.dir.encode(), _safe(pid).encode(), max_seq, C.byref(s), C.byref(t), path, 4096)
        if r <= 0:
            return None
        n = L.st_snapshot_read(path.value, None, 0)
        if n < 0:
            return None
        buf = C.create_string_buffer(max(1, n))
        L.st_snapshot_read(path.value, buf, n)
        return SelectedSnapshot(SnapshotMetadata(pid, int(s.value), int(t.value)),
                                serialization.decode(buf.raw[:n]))

    def delete_to(self, pid: str, max_seq: int) -> int:
        return int(native.lib().st_snapshot_delete_to(self.dir.encode(), _safe(pid).encode(), max_seq))


# ---------------------------------------------------------------------- in-memory plugins
class InMemoryJournal(Journal):
    """Process-global in-memory journal (``inmemory-journal``)."""

    _data: Dict[str, List[Tuple[int, bytes]]] = {}
    _deleted: Dict[str, int] = {}
    _lock = threading.Lock()

    def append(self, pid: str, events: List[Any]) -> int:
        with self._lock:
            log = self._data.setdefault(pid, [])
            seq = log[-1][0] if log else 0
            for e in events:
                seq += 1
                log.append((seq, serialization.encode(e)))
            return seq

    def replay(self, pid: str, from_seq: int = 1, to_seq: int = -1) -> List[Tuple[int, Any]]:
        with self._lock:
            log = list(self._data.get(pid, []))
            dead = self._deleted.get(pid, 0)
        return [(s, serialization.decode(b)) for s, b in log
                if s > dead and s >= from_seq and (to_seq < 0 or s <= to_seq)]

    def highest_sequence_nr(self, pid: str) -> int:
        with self._lock:
            log = self._data.get(pid, [])
            return log[-1][0] if log else 0

    def delete_to(self, pid: str, seq: int) -> None:
        with self._lock:
            self._deleted[pid] = max(seq, self._deleted.get(pid, 0))

    @classmethod
    def clear(cls) -> None:
        with cls._lock:
            cls._data.clear()
            cls._deleted.clear()


class InMemorySnapshotStore(SnapshotStore):
    _data: Dict[str, List[Tuple[SnapshotMetadata, bytes]]] = {}
    _lock = threading.Lock()

    def save(self, pid: str, seq: int, snapshot: Any, timestamp: Optional[int] = None) -> SnapshotMetadata:
        md = SnapshotMetadata(pid, seq, int(time.time() * 1000) if timestamp is None else int(timestamp))
        with self._lock:
            self._data.setdefault(pid, []).append((md, serialization.encode(snapshot)))
        return md

    def load_latest(self, pid: str, max_seq: int = -1) -> Optional[SelectedSnapshot]:
        with self._lock:
            cands = [x for x in self._data.get(pid, []) if max_seq < 0 or x[0].sequence_nr <= max_seq]
        if not cands:
            return None
        md, b = max(cands, key=lambda x: (x[0].sequence_nr, x[0].timestamp))
        return SelectedSnapshot(md, serialization.decode(b))

    def delete_to(self, pid: str, max_seq: int) -> int:
        with self._lock:
            old = self._data.get(pid, [])
            keep = [x for x in old if x[0].sequence_nr > max_seq]
            self._data[pid] = keep
            return len(old) - len(keep)

    @classmethod
    def clear(cls) -> None:
        with cls._lock:
            cls._data.clear()


def _safe(pid: str) -> str:
    return "".join(c if (c.isalnum() or c in "-_.") else "_" for c in pid)


def make_plugins(persist_cfg) -> Tuple[Journal, SnapshotStore]:
    """Journal + snapshot store from a :class:`sharetrade.config.PersistConfig`."""
    if persist_cfg.journal_plugin == "inmemory":
        return InMemoryJournal(), InMemorySnapshotStore()
    if persist_cfg.journal_plugin == "file":
        return FileJournal(persist_cfg.journal_dir), LocalSnapshotStore(persist_cfg.snapshot_dir)
    raise KeyError(f"unknown journal plugin {persist_cfg.journal_plugin}")
