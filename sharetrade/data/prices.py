"""Price sources.

Reference behaviour (`SharePriceGetter.scala:83-108`): the "query" reads a
bundled CSV of ``price, yyyy-MM-dd`` rows, splits on ``,``, trims, keeps rows
whose first two fields parse as (Double, LocalDate) and silently drops the rest
(shapeless HList match at :92-101).  Ticker and date range are ignored (quirk
Q10).  The test spec (`SharePriceGetterSpec.scala:18-55`) expects a *synthetic
linear* source filtered to an inclusive ``[from, to]`` range whose value is
``10 * (day - from)``; both are provided here as pluggable sources, plus a
seeded geometric random walk used for synthetic benchmark data.
"""
from __future__ import annotations

import datetime as _dt
import math
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, List, Optional, Tuple

import numpy as np

Date = _dt.date


def parse_date(s: str) -> Optional[Date]:
    """``yyyy-MM-dd`` strictly (DateTimeFormatter.ofPattern, SharePriceGetter.scala:105-108)."""
    s = s.strip()
    if len(s) != 10 or s[4] != "-" or s[7] != "-":
        return None
    try:
        return _dt.date(int(s[0:4]), int(s[5:7]), int(s[8:10]))
    except ValueError:
        return None


def parse_double(s: str) -> Optional[float]:
    """Java ``String.toDouble`` subset; rejects empty / non-numeric strings."""
    s = s.strip()
    if not s:
        return None
    try:
        v = float(s)
    except ValueError:
        return None
    return v


def parse_price_lines(lines: Iterable[str]) -> Dict[Date, float]:
    """Parse ``price, date[, ...]`` rows; rows that do not parse are dropped."""
    out: Dict[Date, float] = {}
    for line in lines:
        fields = [f.strip() for f in line.rstrip("\n").split(",")]
        if len(fields) < 2:
            continue
        d = parse_date(fields[1])
        p = parse_double(fields[0])
        if d is None or p is None:
            continue
        out[d] = p  # HashMap semantics: a later duplicate date wins
    return out


def load_csv(path: str) -> Dict[Date, float]:
    """``price, yyyy-MM-dd`` rows (the reference's file), or a parsed ``.npz`` series
    (``days``: date ordinals, ``prices``; ``tools/make_msft_fixture.py``)."""
    if path.endswith(".npz"):
        z = np.load(path)          # arrays only (allow_pickle stays False)
        return {Date.fromordinal(int(d)): float(p) for d, p in zip(z["days"], z["prices"])}
    with open(path, "r", encoding="utf-8") as f:
        return parse_price_lines(f)


def filter_range(prices: Dict[Date, float], start: Date, end: Date) -> Dict[Date, float]:
    """Inclusive ``[start, end]`` filter (SharePriceGetterSpec.scala:22-28)."""
    return {d: p for d, p in prices.items() if start <= d <= end}


def sorted_series(prices: Dict[Date, float]) -> Tuple[List[Date], np.ndarray]:
    """TreeMap ordering (StockDataResponse carries a TreeMap[LocalDate, Double])."""
    dates = sorted(prices)
    return dates, np.asarray([prices[d] for d in dates], dtype=np.float64)


def linear_source(name: str, start: Date, end: Date, step: float = 10.0) -> Dict[Date, float]:
    """Synthetic linear series of the test spec: value = step * days since ``start``."""
    n = (end - start).days
    return {start + _dt.timedelta(days=i): step * i for i in range(n + 1)}


def random_walk(length: int, start_price: float = 50.0, volatility: float = 0.02,
                seed: int = 7, n_series: int = 1, drift: float = 0.0) -> np.ndarray:
    """Seeded geometric random walk(s), shape ``[n_series, length]`` (float64)."""
    rng = np.random.default_rng(seed)
    steps = rng.standard_normal((n_series, length - 1)) * volatility + drift
    logp = np.concatenate([np.zeros((n_series, 1)), np.cumsum(steps, axis=1)], axis=1)
    return start_price * np.exp(logp)


def ar1_walk(length: int, start_price: float = 50.0, volatility: float = 0.02, phi: float = 0.3,
             seed: int = 7, n_series: int = 1) -> np.ndarray:
    """Seeded geometric walk(s) whose log-returns follow AR(1): r_t = phi * r_{t-1} + vol * eps_t,
    shape ``[n_series, length]`` (float64).  phi > 0 is momentum: yesterday's move predicts today's,
    a signal a Q-learner can exploit (a plain random walk has none)."""
    rng = np.random.default_rng(seed)
    eps = rng.standard_normal((n_series, length - 1)) * volatility
    r = np.empty_like(eps)
    prev = np.zeros(n_series)
    for t in range(length - 1):
        prev = phi * prev + eps[:, t]
        r[:, t] = prev
    logp = np.concatenate([np.zeros((n_series, 1)), np.cumsum(r, axis=1)], axis=1)
    return start_price * np.exp(logp)


def tick16_quantize(prices: np.ndarray) -> np.ndarray:
    """Every row on its own 16-bit power-of-two tick grid: ``tick * 2**x`` with ``0 < tick <= 65535`` and ``x``
    the smallest exponent that fits the row's largest price (the host mirror of csrc/series.hip tick16_kernel,
    mode 0; float32 in and out).  On such a bank the flagship kernel reads windows as u16 ticks and computes
    bit-identical relative features (w / last - 1 = tick_w / tick_last - 1 exactly); a tick is at most 2**-16
    of the row's largest price -- far below the bf16 resolution of the features (2**-8 relative)."""
    p = np.ascontiguousarray(prices, dtype=np.float32)
    if p.ndim == 1:
        return tick16_quantize(p[None])[0]
    m = p.max(axis=1)
    x = np.frexp(m)[1].astype(np.int64) - 16
    for _ in range(40):   # smallest x with m * 2**-x <= 65535
        dn = (x > -126) & (np.ldexp(m, -(x - 1)).astype(np.float32) <= 65535.0)
        up = np.ldexp(m, -x).astype(np.float32) > 65535.0
        if not dn.any() and not up.any():
            break
        x = np.where(dn, x - 1, np.where(up, x + 1, x))
    t = np.clip(np.rint(np.ldexp(p, -x[:, None]).astype(np.float32)), 1.0, 65535.0).astype(np.float32)
    return np.ldexp(t, x[:, None]).astype(np.float32)


def random_walk_dates(length: int, start: Date = _dt.date(2000, 1, 3)) -> List[Date]:
    return [start + _dt.timedelta(days=i) for i in range(length)]


@dataclass
class PriceQuery:
    """A request ``RequestStockPrice(stockName, from, to)`` (SharePriceGetter.scala:14)."""

    stock_name: str
    start: Date
    end: Date


class PriceSource:
    """Pluggable source: ``query(name, start, end) -> {date: price}``."""

    def query(self, name: str, start: Date, end: Date) -> Dict[Date, float]:
        raise NotImplementedError


class CsvPriceSource(PriceSource):
    """The reference's faked HTTP query over a bundled CSV.

    ``filter_range=False`` reproduces quirk Q10 (name/from/to ignored,
    the whole file is returned)."""

    def __init__(self, path: str, filter_range: bool = False):
        self.path = path
        self.filter = filter_range
        self._cache: Optional[Dict[Date, float]] = None

    def query(self, name: str, start: Date, end: Date) -> Dict[Date, float]:
        if self._cache is None:
            self._cache = load_csv(self.path)
        data = dict(self._cache)
        return filter_range(data, start, end) if self.filter else data


class LinearPriceSource(PriceSource):
    def __init__(self, step: float = 10.0):
        self.step = step

    def query(self, name: str, start: Date, end: Date) -> Dict[Date, float]:
        return linear_source(name, start, end, self.step)


class RandomWalkSource(PriceSource):
    """Deterministic per-ticker random walk, date-filtered."""

    def __init__(self, length: int = 6047, start_price: float = 50.0,
                 volatility: float = 0.02, seed: int = 7,
                 origin: Date = _dt.date(1992, 7, 22)):
        self.length, self.start_price, self.vol, self.seed = length, start_price, volatility, seed
        self.origin = origin

    def query(self, name: str, start: Date, end: Date) -> Dict[Date, float]:
        salt = sum(ord(c) * (i + 1) for i, c in enumerate(name)) & 0xFFFF
        p = random_walk(self.length, self.start_price, self.vol, self.seed + salt)[0]
        dates = random_walk_dates(self.length, self.origin)
        return {d: float(v) for d, v in zip(dates, p) if start <= d <= end}


class CallableSource(PriceSource):
    def __init__(self, fn: Callable[[str, Date, Date], Dict[Date, float]]):
        self.fn = fn

    def query(self, name: str, start: Date, end: Date) -> Dict[Date, float]:
        return self.fn(name, start, end)


def make_source(cfg) -> PriceSource:
    """Build a source from a :class:`sharetrade.config.DataConfig`."""
    from ..config import default_csv_path

    if cfg.source == "csv":
        return CsvPriceSource(cfg.csv_path or default_csv_path(), filter_range=cfg.filter_range)
    if cfg.source == "linear":
        return LinearPriceSource()
    if cfg.source == "random_walk":
        return RandomWalkSource(cfg.length, cfg.start_price, cfg.volatility, cfg.seed)
    raise KeyError(f"unknown price source {cfg.source}")


def to_date(x) -> Date:
    if isinstance(x, Date):
        return x
    return _dt.date.fromisoformat(str(x))
