"""The ws step kernel's LDS images are bank-conflict-free where the design says so
(tools/lds_bank_sim.py --ws: MI355X_MICROARCH.md lane groups per instruction).  Pins the slot swizzle
of csrc/qstep_ws.hip (a_off) and the weight-image swizzle (w1_off) against regressions."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_ws_lds_accesses(capsys):
    import lds_bank_sim

    lds_bank_sim.ws_report()
    rows = [l for l in capsys.readouterr().out.splitlines() if l.startswith("| ") and "access" not in l]
    got = {}
    for l in rows:
        c = [x.strip() for x in l.strip("|").split("|")]
        got[c[0]] = (int(c[2]), int(c[3]))
    conflict_free = ["data: layer-1 W0 fragments (b128)", "data: H1 / H2 -> slot (write b64)",
                     "data: layer-2 W1 fragments (b128)", "data: H2 mask re-read (b64)", "grad: dZ2 rows (b128)",
                     "grad: H1 / H2 (tr)", "grad: X (tr)"]
    for k in conflict_free:
        ideal, cyc = got[k]
        assert cyc == ideal, (k, cyc, ideal)
    # the transposed W1 reads are 2-way by construction (one half-unit per lane), never worse
    assert got["grad: W1^T (tr)"][1] <= 2 * got["grad: W1^T (tr)"][0]
