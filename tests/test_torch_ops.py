"""``torch.ops.sharetrade.*`` registration (sharetrade/ops/torch_ops.py): every op has a schema and a fake
implementation, so shapes propagate without a GPU (FakeTensorMode) and torch.compile can trace through it."""
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import sharetrade.ops  # noqa: F401  (registers the ops)
from sharetrade.ops import torch_ops


def test_every_op_registered_with_schema():
    for name in torch_ops.OPS:
        op = getattr(torch.ops.sharetrade, name)
        assert str(op.default._schema).startswith(f"sharetrade::{name}(")


def test_fake_shapes():
    with FakeTensorMode():
        A = torch.empty(512, 256, dtype=torch.bfloat16)
        B = torch.empty(128, 256, dtype=torch.bfloat16)
        C = torch.ops.sharetrade.gemm_nt(A, B, None, True, False)
        assert C.shape == (512, 128) and C.dtype == torch.bfloat16
        assert torch.ops.sharetrade.gemm_nt(A, B, torch.empty(128), False, True).dtype == torch.float32
        st = torch.empty(33, 203)
        p = torch.empty(4096)
        a, q = torch.ops.sharetrade.qnet_select(st, p, p.bfloat16(), None, 201, True, False, 2400.0, 0.9, 1000.0,
                                                1, 2, 0)
        assert a.shape == (33,) and a.dtype == torch.int32 and q.shape == (33, 3)
        bank = torch.empty(7, 300)
        t, s = torch.ops.sharetrade.tick16(bank)
        assert t.shape == (7, 312) and t.dtype == torch.int16 and s.shape == (7,)
        w = torch.ops.sharetrade.random_walk(5, 100, 50.0, 0.02, 0.0, 1, 2, torch.device("cpu"))
        assert w.shape == (5, 100)
