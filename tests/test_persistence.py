"""Native journal / snapshot store / checkpoint writer (csrc/runtime/*.cpp)."""
import datetime as dt
import os
import struct
import zlib

import numpy as np
import pytest
import torch

from sharetrade import protocol as P
from sharetrade.persist import checkpoint as ck
from sharetrade.persist import native, serialization
from sharetrade.persist.journal import FileJournal, InMemoryJournal, LocalSnapshotStore


def test_crc32c_known_answers():
    # RFC 3720 / iSCSI test vectors
    assert native.crc32c(b"123456789") == 0xE3069283
    assert native.crc32c(bytes(32)) == 0x8A9136AA
    assert native.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43
    data = os.urandom(1000)
    L = native.lib()
    buf = bytes(data)
    assert L.st_crc32c(buf, len(buf), 0) == L.st_crc32c_sw(buf, len(buf), 0)
    # incremental == one-shot
    assert native.crc32c(data[500:], native.crc32c(data[:500])) == native.crc32c(data)


def test_serialization_roundtrip_and_determinism():
    e1 = P.Event("MSFT", {dt.date(2001, 7, 11): 10.0, dt.date(2001, 7, 10): 0.0})
    e2 = P.Event("MSFT", {dt.date(2001, 7, 10): 0.0, dt.date(2001, 7, 11): 10.0})
    b1, b2 = serialization.encode(e1), serialization.encode(e2)
    assert b1 == b2                                  # canonical map order
    assert serialization.decode(b1) == e1
    v = {"a": [1, 2.5, "x", None, True, (3, b"\x00")], "d": dt.date(1992, 7, 22)}
    assert serialization.decode(serialization.encode(v)) == v


def test_file_journal_append_replay_recover(tmp_path):
    d = str(tmp_path / "journal")
    j = FileJournal(d)
    assert j.append("pid", [P.Event("A", {dt.date(2000, 1, 1): 1.0})]) == 1
    assert j.append("pid", [P.Event("B", {dt.date(2000, 1, 2): 2.0}), P.Event("C", {})]) == 3
    j.close()
    j2 = FileJournal(d)
    evs = j2.replay("pid")
    assert [s for s, _ in evs] == [1, 2, 3]
    assert [e.stock_name for _, e in evs] == ["A", "B", "C"]
    assert j2.highest_sequence_nr("pid") == 3
    j2.delete_to("pid", 2)
    assert [s for s, _ in j2.replay("pid")] == [3]
    j2.close()
    # deletion marker survives reopen
    j3 = FileJournal(d)
    assert [s for s, _ in j3.replay("pid")] == [3]
    j3.close()


def test_journal_torn_write_is_truncated(tmp_path):
    d = str(tmp_path / "j")
    j = FileJournal(d)
    for i in range(5):
        j.append("p", [P.Event(f"S{i}", {})])
    j.close()
    path = os.path.join(d, "p.journal")
    size = os.path.getsize(path)
    with open(path, "r+b") as f:            # crash mid-append: chop the last record in half
        f.truncate(size - 7)
    j2 = FileJournal(d)
    assert j2.highest_sequence_nr("p") == 4
    assert j2.truncated_bytes("p") > 0
    assert j2.append("p", [P.Event("S4b", {})]) == 5
    assert [e.stock_name for _, e in j2.replay("p")] == ["S0", "S1", "S2", "S3", "S4b"]
    j2.close()


def test_journal_corruption_stops_replay(tmp_path):
    d = str(tmp_path / "j")
    j = FileJournal(d)
    for i in range(3):
        j.append("p", [P.Event(f"S{i}", {dt.date(2000, 1, 1): float(i)})])
    j.close()
    path = os.path.join(d, "p.journal")
    raw = bytearray(open(path, "rb").read())
    raw[-3] ^= 0xFF                          # flip a payload byte of the last record
    open(path, "wb").write(bytes(raw))
    j2 = FileJournal(d)
    assert [s for s, _ in j2.replay("p")] == [1, 2]
    j2.close()


def test_journal_bytes_are_deterministic(tmp_path):
    blobs = []
    for k in range(2):
        d = str(tmp_path / f"j{k}")
        j = FileJournal(d)
        j.append("p", [P.Event("MSFT", {dt.date(2001, 1, i + 1): i * 1.5 for i in range(20)})])
        j.close()
        blobs.append(open(os.path.join(d, "p.journal"), "rb").read())
    assert blobs[0] == blobs[1]


def test_snapshot_store(tmp_path):
    s = LocalSnapshotStore(str(tmp_path / "snaps"))
    s.save("pid", 5, {"x": 1}, timestamp=100)
    s.save("pid", 9, {"x": 2}, timestamp=200)
    got = s.load_latest("pid")
    assert got.metadata.sequence_nr == 9 and got.snapshot == {"x": 2}
    assert s.load_latest("pid", max_seq=6).snapshot == {"x": 1}
    # a corrupt newest snapshot is skipped
    p = [f for f in os.listdir(tmp_path / "snaps") if "-00000000000000000009-" in f][0]
    raw = bytearray(open(tmp_path / "snaps" / p, "rb").read())
    raw[-1] ^= 1
    open(tmp_path / "snaps" / p, "wb").write(bytes(raw))
    assert s.load_latest("pid").metadata.sequence_nr == 5
    assert s.delete_to("pid", 9) == 2
    assert s.load_latest("pid") is None


def test_checkpoint_roundtrip_bit_identical(tmp_path):
    t = {
        "params": torch.randn(1000),
        "acc": torch.rand(17, 3, dtype=torch.float64),
        "bf": torch.randn(33).to(torch.bfloat16),
        "step": torch.tensor([12345], dtype=torch.int64),
        "flags": torch.tensor([True, False]),
        "empty": torch.zeros(0, 4),
    }
    p1, p2 = str(tmp_path / "a.stck"), str(tmp_path / "b.stck")
    n1 = ck.save(p1, t, {"iteration": 500, "b": [1, 2]})
    n2 = ck.save(p2, dict(t), {"b": [1, 2], "iteration": 500})
    assert n1 == n2 == os.path.getsize(p1)
    assert open(p1, "rb").read() == open(p2, "rb").read()   # same state -> same bytes
    back, meta = ck.load(p1)
    assert meta == {"iteration": 500, "b": [1, 2]}
    assert list(back) == list(t)
    for k in t:
        assert back[k].dtype == t[k].dtype and back[k].shape == t[k].shape
        assert torch.equal(back[k], t[k])
    # data blobs are 64-byte aligned
    raw = open(p1, "rb").read()
    assert raw[:8] == b"STCKPT01" and raw[-8:] == b"STCKEND1"


def test_checkpoint_detects_corruption(tmp_path):
    p = str(tmp_path / "c.stck")
    ck.save(p, {"w": torch.arange(100, dtype=torch.float32)})
    raw = bytearray(open(p, "rb").read())
    raw[200] ^= 0x40
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ck.CheckpointError):
        ck.load(p)


def test_checkpoint_manager_interval_and_retention(tmp_path):
    m = ck.CheckpointManager(str(tmp_path / "ck"), keep=2, interval=500)
    assert not m.should_save(0) and m.should_save(500) and not m.should_save(501)
    for step in (500, 1000, 1500):
        m.save(step, {"w": torch.full((4,), float(step))})
    assert len(m.list()) == 2
    st, meta = ck.load(m.latest())
    assert meta["step"] == 1500 and float(st["w"][0]) == 1500.0


def test_policy_snapshot_every_500_updates_and_resume(tmp_path):
    """Quirk Q13 fixed: the policy actor really checkpoints on the reference's schedule
    (`iteration % 500 == 0 && iteration != 0`, checked before the increment) and a new
    incarnation resumes bit-exactly."""
    from sharetrade.config import preset_config
    from sharetrade.policy.actor import QDecisionPolicyActor
    from sharetrade.actors.runtime import ActorSystem

    cfg = preset_config("test")
    cfg.agent.snapshot_interval = 5
    d = str(tmp_path / "policy")
    sysm = ActorSystem("ck")
    try:
        a = sysm.actor_of(QDecisionPolicyActor.props(cfg, checkpoint_dir=d))
        rng = np.random.default_rng(1)
        states = [rng.uniform(10, 60, 203).astype(np.float32) for _ in range(13)]
        for i in range(12):
            assert a.ask(P.UpdateQ(states[i], 1.0, states[i + 1]), 5).result(10) is P.Updated
        files = sorted(os.listdir(d))
        assert files == ["ckpt-000000000006.stck", "ckpt-000000000011.stck"]
        cont = a.ask(P.SelectionAction(states[0], 2000), 5).result(10)
        b = sysm.actor_of(QDecisionPolicyActor.props(cfg, checkpoint_dir=d))
        # b resumed at iteration 11 -> one more update brings it to a's state at 12
        assert b.ask(P.UpdateQ(states[11], 1.0, states[12]), 5).result(10) is P.Updated
        sa, _ = ck.load(os.path.join(d, "ckpt-000000000011.stck"))
        assert int(sa["iteration"][0]) == 11
    finally:
        sysm.terminate()


def test_price_getter_file_journal_recovery(tmp_path):
    from sharetrade.actors.runtime import ActorSystem
    from sharetrade.config import preset_config
    from sharetrade.data.getter import SharePriceGetter
    from sharetrade.data.prices import LinearPriceSource
    from sharetrade.actors.testkit import TestKit, await_assert

    cfg = preset_config("reference_compat")
    cfg.persist.journal_dir = str(tmp_path / "journal")
    cfg.persist.snapshot_dir = str(tmp_path / "snaps")
    s = ActorSystem("pg")
    try:
        kit = TestKit(s)
        g = s.actor_of(SharePriceGetter.props(LinearPriceSource(), cfg))
        kit.tell(g, P.RequestStockPrice("lloy", dt.date(2001, 7, 10), dt.date(2001, 7, 12)))
        kit.expect_msg_type(P.StockDataResponse)
        kit.tell(g, P.RequestStockPrice("capita", dt.date(2002, 7, 10), dt.date(2002, 7, 11)))
        kit.expect_msg_type(P.StockDataResponse)
        kit.tell(g, P.RequestStockPrice("lloy", dt.date(2001, 7, 11), dt.date(2001, 7, 14)))
        kit.expect_msg_type(P.StockDataResponse)
        s.stop(g)
        await_assert(lambda: _true(g.is_terminated()), 2, 0.01)
        g2 = SharePriceGetter(LinearPriceSource(), cfg)
        g2.context = kit.ref._cell.context
        g2.recover()
        st = g2.stored()
        assert set(st) == {"lloy", "capita"}            # merged on recovery (Q10 fixed)
        # later query only ADDED dates 13, 14; existing dates keep their first values
        assert st["lloy"][dt.date(2001, 7, 11)] == 10.0
        assert st["lloy"][dt.date(2001, 7, 14)] == 30.0
        assert len(st["lloy"]) == 5
    finally:
        s.terminate()


def _true(c):
    assert c


def test_snapshot_names_do_not_collide_across_pids(tmp_path):
    """pid "x" must not load or delete the snapshots of pid "x-1" (exact name match)."""
    s = LocalSnapshotStore(str(tmp_path / "snaps"))
    s.save("x-1", 7, {"who": "x-1"}, timestamp=10)
    assert s.load_latest("x") is None
    s.save("x", 3, {"who": "x"}, timestamp=11)
    assert s.load_latest("x").snapshot == {"who": "x"}
    assert s.delete_to("x", 100) == 1
    assert s.load_latest("x-1").snapshot == {"who": "x-1"}


_FSIZE_CHILD = r"""
import os, resource, signal, sys
sys.path.insert(0, sys.argv[2])
from sharetrade import protocol as P
from sharetrade.persist.journal import FileJournal
d = sys.argv[1]
j = FileJournal(d)
j.append("p", [P.Event("S0", {})])
size = os.path.getsize(os.path.join(d, "p.journal"))
signal.signal(signal.SIGXFSZ, signal.SIG_IGN)
soft, hard = resource.getrlimit(resource.RLIMIT_FSIZE)
resource.setrlimit(resource.RLIMIT_FSIZE, (size + 40, hard))   # the next big record is cut part-way (EFBIG)
import datetime as dt
try:
    j.append("p", [P.Event("BIG", {dt.date(2000, 1, 1) + dt.timedelta(days=i): float(i) for i in range(200)})])
    print("no-error")
except Exception:
    print("append-failed")
assert os.path.getsize(os.path.join(d, "p.journal")) == size, "torn bytes left behind"
resource.setrlimit(resource.RLIMIT_FSIZE, (soft, hard))
j.append("p", [P.Event("S1", {})])
j.close()
"""


def test_failed_append_is_rolled_back(tmp_path):
    """A write that fails part-way (file-size limit ~ ENOSPC) leaves no torn record: the next
    acknowledged append survives recovery."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = str(tmp_path / "j")
    r = subprocess.run([sys.executable, "-c", _FSIZE_CHILD, d, root], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "append-failed" in r.stdout
    j = FileJournal(d)
    assert [e.stock_name for _, e in j.replay("p")] == ["S0", "S1"]
    assert j.truncated_bytes("p") == 0
    j.close()
