"""The reference's own run at full length on the GPU (`ShareTradeHelper.scala:20-48`): 10 workers x the
whole MSFT series (5,846 steps each, `TrainerChildActor.scala:64-71`) as lanes of the vector engine on
the exact-fp32 row kernels (csrc/mlp_f32.hip) -> exactly avg 2400.0 / std 0.0 (quirk Q1 makes every
reward 0, `TrainerChildActor.scala:118-123`).  The series is the bundled parsed copy when the reference
checkout is absent (config.default_csv_path)."""
import pytest

pytestmark = pytest.mark.gpu


def test_full_length_compat_run_gpu_fp32_rows(native_built):
    from sharetrade.app import run
    from sharetrade.config import preset_config

    cfg = preset_config("test")
    cfg.router.poll_interval_s = 0.25
    cfg.env.progress_every = 0
    res = run(cfg, engine="vector", device="cuda:0", quiet=True)
    assert res["completed"] == 1.0, res
    assert res["avg"] == 2400.0 and res["std"] == 0.0, res


def test_full_length_intended_run_gpu_trades(native_built):
    """Same run with the quirks fixed (intended preset): the env trades, every worker completes."""
    from sharetrade.app import run
    from sharetrade.config import preset_config

    cfg = preset_config("intended")
    cfg.persist.journal_plugin = "inmemory"
    cfg.router.poll_interval_s = 0.25
    cfg.env.progress_every = 0
    res = run(cfg, engine="vector", device="cuda:0", quiet=True)
    assert res["completed"] == 1.0, res
    assert res["avg"] != 2400.0
