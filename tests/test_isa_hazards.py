"""Every production kernel's gfx950 ISA is free of the MFMA result hazards hipcc under-pads
(tools/mfma_hazard_scan.py; measured minima in profiles/r5_mfma_hazards.md): a 16x16x16 MFMA reading a
16x16x32 result as its accumulator within 4 wait states, or an accvgpr read of an MFMA result too early.
CPU only (hipcc -S); slow: compiles every csrc/*.hip once more."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_no_under_padded_mfma_result_reads():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_hazard_scan.py")], capture_output=True,
                       text=True, timeout=1500)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "total: 0" in r.stdout


def test_scanner_flags_the_qtarget_pattern():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from mfma_hazard_scan import scan

    bad = """k:
\tv_mfma_f32_16x16x32_bf16 a[56:59], v[164:167], v[88:91], a[56:59]
\tv_cvt_pk_bf16_f32 v88, 1.0, v80
\tv_mfma_f32_16x16x16_bf16 a[56:59], v[150:151], v[152:153], a[56:59]
"""
    ok = bad.replace("\tv_cvt_pk_bf16_f32", "\ts_nop 3\n\tv_cvt_pk_bf16_f32")
    chain = bad.replace("16x16x16_bf16 a[56:59], v[150:151]", "16x16x32_bf16 a[56:59], v[150:153]")
    assert len(scan(bad)) == 1 and scan(ok) == [] and scan(chain) == []


def test_scanner_follows_the_loop_exit_fall_through():
    """The w4k GEMM's first form: the loop exit read an accumulator two instructions after the loop's last
    (inline-asm) MFMA, behind a conditional branch."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from mfma_hazard_scan import scan

    bad = """k:
\tv_mfma_f32_16x16x32_bf16 a[252:255], v[66:69], v[70:73], a[252:255]
\ts_cbranch_scc1 .LBB24_74
\tv_accvgpr_read_b32 v1, a254
"""
    ok = bad.replace("\tv_accvgpr_read_b32", "\ts_nop 7\n\tv_accvgpr_read_b32")
    jump = bad.replace("s_cbranch_scc1", "s_branch")
    mov = bad.replace("v_accvgpr_read_b32 v1, a254", "v_accvgpr_mov_b32 a0, a254")
    assert len(scan(bad)) == 1 and scan(ok) == [] and scan(jump) == [] and len(scan(mov)) == 1
