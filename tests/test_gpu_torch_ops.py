"""``torch.ops.sharetrade.*`` on the GPU: each registered operator runs its HIP kernel and matches a plain
PyTorch fp32 reference (or the module-level wrapper it registers), shows under its own name in a
torch.profiler trace, and runs inside a torch.compile'd function."""
import numpy as np
import pytest
import torch

import sharetrade.ops  # noqa: F401

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def test_gemm_nt_op_matches_fp32_reference(native_built):
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(512, 256, device="cuda", generator=g).bfloat16()
    B = torch.randn(256, 256, device="cuda", generator=g).bfloat16()
    bias = torch.randn(256, device="cuda", generator=g)
    lin = A.float() @ B.float().t() + bias
    out = torch.ops.sharetrade.gemm_nt(A, B, bias, False, True)      # fp32 epilogue: bias
    assert out.dtype == torch.float32 and _rel(out, lin) < 1e-5
    outb = torch.ops.sharetrade.gemm_nt(A, B, bias, True, False)     # bf16 epilogue: bias + ReLU
    assert outb.dtype == torch.bfloat16 and _rel(outb, torch.relu(lin)) < 1e-2
    with pytest.raises(Exception, match="ReLU"):
        torch.ops.sharetrade.gemm_nt(A, B, bias, True, True)


def test_qnet_select_op_matches_reference(native_built):
    from sharetrade.config import preset_config
    from sharetrade.models import qnet as qn
    from sharetrade.serve import kernel as K

    cfg = preset_config("flagship")
    layout = qn.QNetLayout.from_config(cfg.model)
    params = qn.init_params(layout, cfg.model, seed=3, device="cuda")
    pbf = params.bfloat16()
    rng = np.random.default_rng(1)
    B = 300
    st = torch.from_numpy(np.concatenate([rng.uniform(40, 60, (B, 201)), rng.uniform(0, 4800, (B, 1)),
                                          rng.integers(0, 9, (B, 1))], 1).astype(np.float32)).cuda()
    a, q = torch.ops.sharetrade.qnet_select(st, params, pbf, None, 201, True, False, cfg.env.budget, 0.9, 1000.0,
                                            11, 12, 0)
    ra, rq = K.reference_select(params, layout, st, history=201, feat_mode="relative", output_relu=False,
                                budget0=cfg.env.budget, epsilon=0.9, ramp=1000.0, key_seed=0)
    assert _rel(q, rq) < 2e-2
    near_tie = (rq.topk(2, dim=1).values[:, 0] - rq.topk(2, dim=1).values[:, 1]) < 1e-3 * rq.abs().max()
    assert torch.equal(a[~near_tie], ra[~near_tie])


def test_bank_ops(native_built):
    from sharetrade.data.prices import tick16_quantize
    from sharetrade.ops import native

    dev = torch.device("cuda", 0)
    w = torch.ops.sharetrade.random_walk(64, 700, 50.0, 0.02, 0.0, 5, 6, dev)
    ref = torch.empty(64, 700, device=dev)
    native.random_walk(ref, 50.0, 0.02, 0.0, 5, 6)
    assert torch.equal(w, ref)
    t, s = torch.ops.sharetrade.tick16(w)
    assert t.shape[0] == 0                                 # a plain random walk is off the tick grid
    torch.ops.sharetrade.tick16_quantize_(w)
    assert torch.equal(w.cpu(), torch.from_numpy(tick16_quantize(ref.cpu().numpy())))
    t, s = torch.ops.sharetrade.tick16(w)
    back = t.cpu().numpy().view(np.uint16)[:, :700].astype(np.float32) * s.cpu().numpy()[:, None]
    assert np.array_equal(back, w.cpu().numpy())
    blk = torch.zeros(8, 16, device=dev)
    torch.ops.sharetrade.init_normal_(blk, 8, 16, 1.0, 1, 2, 3)
    ref = torch.zeros(8, 16, device=dev)
    native.init_normal(ref, 8, 16, 1.0, 1, 2, 3)
    assert torch.equal(blk, ref) and blk.abs().sum() > 0


def test_ops_in_profiler_and_compile(native_built):
    A = torch.randn(256, 128, device="cuda").bfloat16()
    B = torch.randn(256, 128, device="cuda").bfloat16()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        torch.ops.sharetrade.gemm_nt(A, B, None, True, False)
    assert any("sharetrade::gemm_nt" in e.name for e in prof.events())

    def f(a, b):
        return torch.ops.sharetrade.gemm_nt(a, b, None, False, True) * 2.0

    cf = torch.compile(f, backend="eager", fullgraph=True)
    assert torch.allclose(cf(A, B), f(A, B))
