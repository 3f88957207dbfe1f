"""``SharePriceGetter`` — the persistent price-data service.

Reference (`SharePriceGetter.scala:20-108`): ``RequestStockPrice(name, from,
to)`` runs a (faked) query in a ``Future``, pipes ``(originalSender,
Event(name, prices))`` back to itself, replies
``StockDataResponse(name, TreeMap(prices))`` and *then* persists the event;
after the first query it ``become``s ``queried(stockMap)`` and merges only the
new dates of later queries into the stored map; recovery replays events.

Defaults fix the reference's quirks: the query honours ticker and date range
(pluggable :class:`~sharetrade.data.prices.PriceSource`; the spec's synthetic
linear source is one of them, `SharePriceGetterSpec.scala:18-55`) and recovery
merges tickers instead of keeping only the last one (Q10).
``persist_before_reply`` switches off the reference's reply-before-persist
ordering (Q11).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, Optional

from ..actors.runtime import ActorRef, NotHandled, Props, pipe_to
from ..config import Config, preset_config
from ..persist.journal import Journal, SnapshotStore, make_plugins
from ..persist.persistent import PersistentActor, RecoveryCompleted, SnapshotOffer
from ..protocol import Event, RequestStockPrice, StockDataResponse, TreeMap
from .prices import PriceSource, make_source


@dataclass(frozen=True)
class _Queried:
    original_sender: Optional[ActorRef]
    event: Event


def merge_new_dates(stored: Dict[str, Dict], e: Event) -> Dict[str, Dict]:
    """``updateStockMapIfTheresChange`` (`SharePriceGetter.scala:64-73`): only
    dates not yet stored are added; existing dates keep their old value."""
    out = dict(stored)
    cur = stored.get(e.stock_name)
    if cur is None:
        out[e.stock_name] = dict(e.share_prices)
    else:
        merged = dict(cur)
        for d, p in e.share_prices.items():
            if d not in merged:
                merged[d] = p
        out[e.stock_name] = merged
    return out


class SharePriceGetter(PersistentActor):
    persistence_id = "Share-price-getter"

    def __init__(self, source: Optional[PriceSource] = None, cfg: Optional[Config] = None,
                 journal: Optional[Journal] = None, snapshot_store: Optional[SnapshotStore] = None):
        self.cfg = cfg or preset_config("reference_compat")
        if journal is None or snapshot_store is None:
            j, s = make_plugins(self.cfg.persist)
            journal = journal or j
            snapshot_store = snapshot_store or s
        super().__init__(journal, snapshot_store)
        self.source = source or make_source(self.cfg.data)
        self.stock_map: Dict[str, Dict] = {}
        self.recovered_events = 0

    @classmethod
    def props(cls, source: Optional[PriceSource] = None, cfg: Optional[Config] = None, **kw) -> Props:
        return Props(cls, source, cfg, **kw)

    # ------------------------------------------------------------------ recovery
    def receive_recover(self, msg: Any) -> Any:
        if msg is RecoveryCompleted:
            self.log.info("Recovery is finished")
            return None
        if isinstance(msg, SnapshotOffer):
            self.stock_map = {k: dict(v) for k, v in msg.snapshot.items()}
            return None
        if isinstance(msg, Event):
            self.recovered_events += 1
            self.log.info(f"Recovery for stock name : {msg.stock_name}")
            if self.cfg.persist.merge_on_recovery:
                self.stock_map = merge_new_dates(self.stock_map, msg)
            else:
                self.stock_map = {msg.stock_name: dict(msg.share_prices)}   # quirk Q10: last ticker wins
        return None

    # ------------------------------------------------------------------ commands
    def receive_command(self, msg: Any) -> Any:
        if isinstance(msg, RequestStockPrice):
            original = self.sender
            name, frm, to = msg.stock_name, msg.from_, msg.to
            fut = self.context.system.future(lambda: self.source.query(name, frm, to))
            pipe_to(fut.map(lambda prices: _Queried(original, Event(name, dict(prices)))), self.self_ref)
            return None
        if isinstance(msg, _Queried):
            e = msg.event
            reply = StockDataResponse(e.stock_name, TreeMap(e.share_prices))
            if not self.cfg.persist.persist_before_reply and msg.original_sender is not None:
                msg.original_sender.tell(reply, self.self_ref)
            self.persist(e, self._on_persisted)
            if self.cfg.persist.persist_before_reply and msg.original_sender is not None:
                msg.original_sender.tell(reply, self.self_ref)
            return None
        return NotHandled

    def _on_persisted(self, e: Event) -> None:
        self.stock_map = merge_new_dates(self.stock_map, e)
        self.log.info(f"Receive command, persisted stock name : {e.stock_name} & shareprices :"
                      f"{len(e.share_prices)} rows")

    def stored(self) -> Dict[str, Dict]:
        return self.stock_map
