#!/usr/bin/env python3
"""Write ``sharetrade/data/msft_prices.npz`` from the reference's bundled MSFT price file.

The reference reads ``src/main/resources/MSFT-stock-prices-revised.txt`` as a classpath resource
(`SharePriceGetter.scala:83-102`).  Parity tests need that series on every machine that runs them --
the GPU boxes included, where the reference checkout does not exist -- so the parsed series (the rows
`sharetrade.data.prices.parse_price_lines` keeps, as the reference's HList match keeps them) is stored
here as two arrays: ``days`` (proleptic Gregorian ordinals, int32, ascending) and ``prices`` (float64),
plus the SHA-256 of the source file.  ``tests/test_app.py`` re-derives it from the CSV whenever the
CSV is present and checks that the fixture is identical.

Usage: python tools/make_msft_fixture.py [csv] [out]
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sharetrade.config import REFERENCE_CSV  # noqa: E402
from sharetrade.data.prices import load_csv  # noqa: E402


def main() -> int:
    src = sys.argv[1] if len(sys.argv) > 1 else REFERENCE_CSV
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "sharetrade", "data", "msft_prices.npz")
    data = load_csv(src)
    dates = sorted(data)
    days = np.asarray([d.toordinal() for d in dates], dtype=np.int32)
    prices = np.asarray([data[d] for d in dates], dtype=np.float64)
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()
    np.savez_compressed(out, days=days, prices=prices, source_sha256=np.asarray(sha))
    print(out, len(days), sha)
    return 0


if __name__ == "__main__":
    sys.exit(main())
