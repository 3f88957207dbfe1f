"""The ctypes mirrors of the launch-parameter structs match the C++ structs' sizes (CPU: the HIP library is only
loaded, no HIP call is made).  A field added on one side only shows up here instead of as a wrong kernel argument."""
import ctypes as C

import pytest

from sharetrade.ops import native


def _sizes(fn_name):
    L = native.lib()
    fn = getattr(L, fn_name)
    fn.argtypes, fn.restype = [C.POINTER(C.c_int), C.c_int], C.c_int
    n = fn(None, 0)
    out = (C.c_int * n)()
    assert fn(out, n) == n
    return list(out)


@pytest.fixture(scope="module")
def lib_available():
    try:
        native.lib()
    except native.NativeUnavailable as e:   # (not built in this checkout)
        pytest.skip(str(e))


def test_deep_structs_match(lib_available):
    from sharetrade.trainer import deep

    mirrors = [deep._Replay, deep._Gather, deep._Env, deep._TD, deep._Head, deep._QHead, deep._Adam, deep._AdamSeg,
               deep._AdamMulti]
    assert _sizes("st_deep_abi") == [C.sizeof(m) for m in mirrors]


def test_gemm_structs_match(lib_available):
    from sharetrade.ops import gemm as gm

    assert _sizes("st_gemm_abi") == [C.sizeof(gm.GemmArgs), C.sizeof(gm.GemmArgs) * gm.GEMM_MAXB + 4 + 4]


@pytest.mark.parametrize("fn,mirrors", [
    ("st_abi_optim", ["sharetrade.ops.native:OptimParams"]),
    ("st_abi_qtarget", ["sharetrade.ops.native:QStepParams", "sharetrade.ops.native:QTargetParams"]),
    ("st_abi_gru", ["sharetrade.ops.gru:MinuteBarsArgs", "sharetrade.ops.gru:PackArgs", "sharetrade.ops.gru:ActArgs"]),
    ("st_abi_gru_learn", ["sharetrade.ops.gru:GatherArgs", "sharetrade.ops.gru:NetW", "sharetrade.ops.gru:SeqFwdArgs",
                          "sharetrade.ops.gru:TDArgs", "sharetrade.ops.gru:SeqBwdArgs"]),
    ("st_abi_mlp_f32", ["sharetrade.ops.mlp_f32:F32Net", "sharetrade.ops.mlp_f32:F32Rows",
                        "sharetrade.ops.mlp_f32:F32Optim"]),
    ("st_abi_mlp_f32_mfma", ["sharetrade.ops.mlp_f32:GemmF32", "sharetrade.ops.mlp_f32:Fwd2F32",
                             "sharetrade.ops.mlp_f32:F32Batch"]),
    ("st_abi_qserve", ["sharetrade.serve.kernel:ServeParams"]),
])
def test_launch_structs_match(lib_available, fn, mirrors):
    """Every other launch file: its structs against their ctypes mirrors (the fused and the wide / ws step kernels
    each define QStepParams; both must match the one mirror both launchers take)."""
    import importlib

    sizes = []
    for m in mirrors:
        mod, name = m.split(":")
        sizes.append(C.sizeof(getattr(importlib.import_module(mod), name)))
    assert _sizes(fn) == sizes


def test_fused_step_params_are_the_prefix(lib_available):
    """csrc/qstep_fused.hip reads the leading fields of the QStepParams mirror (its FusedStepParams ends at td_clip):
    its size is the offset of the first field it does not have."""
    from sharetrade.ops.native import QStepParams

    assert _sizes("st_abi_qstep_fused") == [QStepParams.err.offset]
    assert [f for f, _ in QStepParams._fields_].index("err") == [f for f, _ in QStepParams._fields_].index("td_clip") + 1
