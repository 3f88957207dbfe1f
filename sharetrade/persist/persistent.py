"""Event-sourced actors (``akka.persistence.PersistentActor``).

The reference's ``SharePriceGetter`` is a ``PersistentActor`` with
``persistenceId = "Share-price-getter"`` that ``persist``s an ``Event`` after
each query and rebuilds its state in ``receiveRecover`` on restart
(`SharePriceGetter.scala:21-62`).  :class:`PersistentActor` here runs recovery
in ``pre_start`` — latest snapshot (``SnapshotOffer``), then the journal tail,
then ``RecoveryCompleted`` — before the first command is processed, and makes
``persist`` durable (journal append) before its handler runs.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, List, Optional

from ..actors.runtime import Actor, NotHandled, singleton
from .journal import InMemoryJournal, InMemorySnapshotStore, Journal, SnapshotMetadata, SnapshotStore

RecoveryCompleted = singleton("RecoveryCompleted")


@dataclass(frozen=True)
class SnapshotOffer:
    metadata: SnapshotMetadata
    snapshot: Any


@dataclass(frozen=True)
class SaveSnapshotSuccess:
    metadata: SnapshotMetadata


@dataclass(frozen=True)
class SaveSnapshotFailure:
    metadata: SnapshotMetadata
    cause: BaseException


@dataclass(frozen=True)
class DeleteMessagesSuccess:
    to_sequence_nr: int


class PersistentActor(Actor):
    """Subclasses define ``persistence_id``, :meth:`receive_command` and
    :meth:`receive_recover`; ``context.become`` swaps the *command* behaviour."""

    persistence_id: str = "persistent-actor"

    def __init__(self, journal: Optional[Journal] = None, snapshot_store: Optional[SnapshotStore] = None):
        self.journal = journal if journal is not None else InMemoryJournal()
        self.snapshot_store = snapshot_store if snapshot_store is not None else InMemorySnapshotStore()
        self.last_sequence_nr = 0
        self.recovery_running = False

    # ------------------------------------------------------------ to override
    def receive_command(self, msg: Any) -> Any:
        return NotHandled

    def receive_recover(self, msg: Any) -> Any:
        return None

    # ------------------------------------------------------------ lifecycle
    def receive(self, msg: Any) -> Any:
        return self.receive_command(msg)

    def pre_start(self) -> None:
        self.recover()

    def recover(self) -> None:
        self.recovery_running = True
        try:
            snap = self.snapshot_store.load_latest(self.persistence_id)
            from_seq = 1
            if snap is not None:
                self.last_sequence_nr = snap.metadata.sequence_nr
                self.receive_recover(SnapshotOffer(snap.metadata, snap.snapshot))
                from_seq = snap.metadata.sequence_nr + 1
            for seq, ev in self.journal.replay(self.persistence_id, from_seq):
                self.last_sequence_nr = seq
                self.receive_recover(ev)
            self.last_sequence_nr = max(self.last_sequence_nr, self.journal.highest_sequence_nr(self.persistence_id))
        finally:
            self.recovery_running = False
        self.receive_recover(RecoveryCompleted)

    # ------------------------------------------------------------ persistence ops
    def persist(self, event: Any, handler: Callable[[Any], Any]) -> None:
        self.last_sequence_nr = self.journal.append(self.persistence_id, [event])
        handler(event)

    def persist_all(self, events: List[Any], handler: Callable[[Any], Any]) -> None:
        if not events:
            return
        self.last_sequence_nr = self.journal.append(self.persistence_id, list(events))
        for e in events:
            handler(e)

    def delete_messages(self, to_sequence_nr: int) -> None:
        self.journal.delete_to(self.persistence_id, to_sequence_nr)
        self.self_ref.tell(DeleteMessagesSuccess(to_sequence_nr), self.self_ref)

    def save_snapshot(self, snapshot: Any) -> None:
        md = SnapshotMetadata(self.persistence_id, self.last_sequence_nr, 0)
        try:
            md = self.snapshot_store.save(self.persistence_id, self.last_sequence_nr, snapshot)
            self.self_ref.tell(SaveSnapshotSuccess(md), self.self_ref)
        except Exception as e:  # noqa: BLE001
            self.self_ref.tell(SaveSnapshotFailure(md, e), self.self_ref)
