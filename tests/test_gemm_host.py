"""Host-side GEMM dispatch (CPU): tile selection and the shape checks that run before any launch."""
import pytest
import torch

from sharetrade.ops import gemm as gm


def _t(*shape, dtype=torch.bfloat16):
    return torch.zeros(*shape, dtype=dtype)


def test_auto_tile_prefers_pingpong_for_big_plain_products():
    assert gm.auto_tile(16384, 1024, gm.EPI_BF16, {}) == (256, 256, "pp")
    assert gm.auto_tile(16384, 1024, gm.EPI_F32, {"splitk": "auto"}) == (256, 256, "pp")
    # C^T, relu-grad masks and explicit split-K stay on the 128-family kernels
    assert gm.auto_tile(16384, 1024, gm.EPI_BF16, {"outT": _t(1024, 16384)}) == gm.pick_tile(16384, 1024)
    assert gm.auto_tile(16384, 1024, gm.EPI_RELU_GRAD, {}) == gm.pick_tile(16384, 1024)
    assert gm.auto_tile(16384, 1024, gm.EPI_F32, {"splitk": 4}) == gm.pick_tile(16384, 1024)
    # too few 256x256 tiles to fill 256 CUs
    assert gm.auto_tile(4096, 1024, gm.EPI_BF16, {}) == gm.pick_tile(4096, 1024)
    old = gm.PINGPONG
    try:
        gm.PINGPONG = False
        assert gm.auto_tile(16384, 1024, gm.EPI_BF16, {}) == gm.pick_tile(16384, 1024)
    finally:
        gm.PINGPONG = old


def test_pick_splitk_fills_the_chip():
    assert gm.pick_splitk(1024, 1024, 4096, (128, 128)) == 4        # 64 tiles -> 256 workgroups
    assert gm.pick_splitk(1024, 256, 4096, (64, 64)) == 4           # 64 tiles -> 256
    assert gm.pick_splitk(4096, 1024, 1024, (128, 128)) == 1        # already 256 tiles


def test_batched_and_dual_reject_bad_shapes_before_launch():
    A, B = _t(256, 128), _t(256, 128)
    ok = (A, B, _t(256, 256), {})
    with pytest.raises(ValueError):   # second problem not a multiple of the tile
        gm.gemm_nt_batched([ok, (_t(192, 128), _t(256, 128), _t(192, 256), {})], gm.EPI_BF16, (128, 128))
    with pytest.raises(ValueError):   # more than GEMM_MAXB problems
        gm.gemm_nt_batched([ok] * (gm.GEMM_MAXB + 1), gm.EPI_BF16, (128, 128))
    with pytest.raises(ValueError):   # 64-row product on 128x128 tiles
        gm.gemm_dual(ok, gm.EPI_BF16, (_t(64, 128), _t(256, 128), _t(64, 256, dtype=torch.float32), {}), gm.EPI_F32)
    with pytest.raises(ValueError):   # split-K needs the fp32 epilogue
        gm.make_args(A, B, _t(256, 256), gm.EPI_BF16, splitk=2)


def test_epilogue_side_outputs_are_validated_before_launch():
    """colpart (bias-gradient column partials) and qhead (the next layer's head folded into the bf16 epilogue) are
    refused on the host when their epilogue, dtype or shape does not fit; a fitting qhead fills the ABI fields the
    kernel checks against the tile (csrc/gemm_bf16.hip gemm_args_ok)."""
    A, B = _t(256, 128), _t(256, 128)
    out16, out32 = _t(256, 256), _t(256, 256, dtype=torch.float32)
    with pytest.raises(ValueError):   # column partials only with the relu-grad epilogue
        gm.make_args(A, B, out16, gm.EPI_BF16, colpart=_t(4, 256, dtype=torch.float32))
    with pytest.raises(ValueError):   # too narrow
        gm.make_args(A, B, out16, gm.EPI_RELU_GRAD, auxT=_t(256, 256), colpart=_t(4, 128, dtype=torch.float32))
    qw = _t(3, 256)
    qp = _t(4, 256, 4, dtype=torch.float32)
    with pytest.raises(ValueError):   # the head rides on the bf16 epilogue only
        gm.make_args(A, B, out32, gm.EPI_F32, qhead=(qw, qp))
    with pytest.raises(ValueError):   # at most 4 head rows
        gm.make_args(A, B, out16, gm.EPI_BF16, qhead=(_t(5, 256), qp))
    with pytest.raises(ValueError):   # partials must be fp32 [parts, M, 4]
        gm.make_args(A, B, out16, gm.EPI_BF16, qhead=(qw, _t(4, 256, 3, dtype=torch.float32)))
    with pytest.raises(ValueError):   # head rows shorter than N
        gm.make_args(A, B, out16, gm.EPI_BF16, qhead=(_t(3, 128), qp))
    g = gm.make_args(A, B, out16, gm.EPI_BF16, qhead=(qw, qp))
    assert (g.nq, g.nqp, g.ldqw) == (3, 4, 256) and g.qpart == qp.data_ptr() and g.qw == qw.data_ptr()
    plain = gm.make_args(A, B, out16, gm.EPI_BF16)
    assert not plain.qpart and not plain.colpart and plain.nqp == 0
