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
