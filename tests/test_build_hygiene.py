"""The production native library ships production kernels only (VERDICT r3 'production-build hygiene').

The timing / debug builds of the flagship step kernel (csrc/ab/: per-phase stamps, phases skipped or
run twice to price them, several computing WRONG results by design) build into their own opt-in
library, and ``engine.step_variant`` refuses them unless SHARETRADE_AB_BUILDS=1."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_production_sources_exclude_ab_builds():
    prod = sorted(os.path.basename(p) for p in glob.glob(os.path.join(ROOT, "csrc", "*.hip")))
    assert not any(p.startswith("qstep_ws_") for p in prod), prod
    assert "qstep_pair.hip" not in prod
    assert "qstep_pipe.hip" not in prod   # measured 2.6x slower than ws: retired to the opt-in A/B library
    ab = sorted(os.path.basename(p) for p in glob.glob(os.path.join(ROOT, "csrc", "ab", "*.hip")))
    assert "qstep_ws_stamps.hip" in ab and "qstep_ws_gskip.hip" in ab


def test_variant_refused_without_opt_in(monkeypatch):
    from sharetrade.ops import native

    monkeypatch.delenv("SHARETRADE_AB_BUILDS", raising=False)
    for v in sorted(native.WRONG_RESULT_VARIANTS) + ["stamps"]:
        with pytest.raises(RuntimeError, match="SHARETRADE_AB_BUILDS"):
            native.variant_launch(v)
    with pytest.raises(RuntimeError, match="WRONG"):
        native.variant_launch("gskip")


@pytest.mark.skipif(shutil.which("nm") is None, reason="binutils nm not available")
def test_production_library_has_no_timing_builds():
    from sharetrade.ops import native

    if not os.path.exists(native.HIP_LIB_PATH):
        pytest.skip("native library not built")
    out = subprocess.run(["nm", "-D", native.HIP_LIB_PATH], stdout=subprocess.PIPE, text=True, check=True).stdout
    syms = [ln.split()[-1] for ln in out.splitlines() if ln.strip()]
    step = [s for s in syms if s.startswith("st_qstep")]
    assert "st_qstep_ws_launch" in step
    bad = [s for s in step if s.startswith("st_qstep_ws_launch_") or "pair" in s or "pipe" in s]
    assert not bad, bad
    assert not [s for s in syms if "qstep_pipe" in s], "csrc/ab/qstep_pipe.hip leaked into the production library"
