"""``torch.ops.sharetrade.*``: the HIP kernels as registered PyTorch operators.

The kernels are reached through the C ABI of ``libsharetrade_hip.so`` (``sharetrade.ops.native``); this module
registers the ones with a tensor-in / tensor-out contract with ``torch.library.custom_op``, so they carry a
schema, show under their own names in ``torch.profiler`` traces, run inside ``torch.compile`` graphs as opaque
nodes (each has a fake implementation for shape propagation) and compose with HIP-graph capture like any op
on the current stream.  The engine's fused step kernels keep their ctypes launch path: they act on an engine's
many resident buffers at once (env state, slabs, weight images), not on a few tensors.

    sharetrade::gemm_nt(A, B, bias?, relu, out_fp32) -> C           bf16 MFMA GEMM, C = A . B^T (+ bias, ReLU)
    sharetrade::qnet_select(states, params, params_bf, ...) -> (actions, q)
                                                                    batched SelectionAction (csrc/qserve.hip)
    sharetrade::random_walk(E, T, start, vol, drift, key0, key1, device) -> bank [E, T]
    sharetrade::tick16_quantize_(bank) -> ()                         bank onto its 16-bit tick grid, in place
    sharetrade::tick16(bank) -> (ticks [E, T16] int16, scale [E])   (empty when the bank is off the grid)
    sharetrade::init_normal_(block, rows, cols, std, key0, key1, stream) -> ()

``import sharetrade.ops.torch_ops`` (done by ``sharetrade.ops``) registers them.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch.library import custom_op

from . import native

NS = "sharetrade"


# ---------------------------------------------------------------------------------------------- GEMM
@custom_op(f"{NS}::gemm_nt", mutates_args=())
def gemm_nt(A: torch.Tensor, B: torch.Tensor, bias: Optional[torch.Tensor], relu: bool, out_fp32: bool) -> torch.Tensor:
    """``C = A . B^T`` on the bf16 MFMA GEMM (csrc/gemm_bf16.hip): A [M, K], B [N, K] bf16 (K-contiguous),
    optional fp32 bias [N] fused into the epilogue; C bf16 with an optional fused ReLU, or fp32 (``out_fp32``,
    no ReLU).  Tile choice as the engines' (``ops.gemm.auto_tile``); M, N, K must fit whole tiles (K % 64 == 0)."""
    from . import gemm as gm

    if relu and out_fp32:
        raise ValueError("sharetrade::gemm_nt: the fp32 epilogue has bias (and alpha / accumulate) but no ReLU")
    M, N = A.shape[0], B.shape[0]
    out = torch.empty(M, N, dtype=torch.float32 if out_fp32 else torch.bfloat16, device=A.device)
    gm.gemm_nt(A.contiguous(), B.contiguous(), out, gm.EPI_F32 if out_fp32 else gm.EPI_BF16,
               bias=None if bias is None else bias.float().contiguous(), relu=relu)
    return out


@gemm_nt.register_fake
def _(A, B, bias, relu, out_fp32):
    return A.new_empty(A.shape[0], B.shape[0], dtype=torch.float32 if out_fp32 else torch.bfloat16)


# ---------------------------------------------------------------------------------------------- serving
@custom_op(f"{NS}::qnet_select", mutates_args=())
def qnet_select(states: torch.Tensor, params: torch.Tensor, params_bf: torch.Tensor, steps: Optional[torch.Tensor],
                history: int, relative_features: bool, output_relu: bool, budget0: float, epsilon: float,
                ramp: float, key0: int, key1: int, seq: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Batched ``SelectionAction`` (csrc/qserve.hip): raw request rows [B, >= history + 2] fp32 (window prices,
    budget, shares) -> features -> the flagship 2x128 Q-net (flat ``params`` fp32 + its bf16 copy) -> greedy
    argmax, or epsilon-greedy at ``steps`` [B] (Philox counters (row, seq)).  Returns (actions int32 [B],
    q fp32 [B, 3])."""
    from ..config import preset_config
    from ..models import qnet as qn
    from ..serve import kernel as K

    cfg = preset_config("flagship")
    cfg.model.history = int(history)
    cfg.model.output_relu = bool(output_relu)
    layout = qn.QNetLayout.from_config(cfg.model)
    kern = K.ServeKernel(layout, params, params_bf, history=int(history), feat_mode=int(bool(relative_features)),
                         output_relu=bool(output_relu), budget0=float(budget0), epsilon=float(epsilon),
                         ramp=float(ramp), key=(int(key0), int(key1)))
    B = states.shape[0]
    actions = torch.empty(B, dtype=torch.int32, device=states.device)
    q = torch.empty(B, 3, dtype=torch.float32, device=states.device)
    kern.launch(states.float().contiguous(), actions, q_out=q,
                steps=None if steps is None else steps.float().contiguous(), seq=int(seq))
    return actions, q


@qnet_select.register_fake
def _(states, params, params_bf, steps, history, relative_features, output_relu, budget0, epsilon, ramp, key0,
      key1, seq):
    B = states.shape[0]
    return states.new_empty(B, dtype=torch.int32), states.new_empty(B, 3, dtype=torch.float32)


# ---------------------------------------------------------------------------------------------- price banks
@custom_op(f"{NS}::random_walk", mutates_args=())
def random_walk(E: int, T: int, start: float, vol: float, drift: float, key0: int, key1: int,
                device: torch.device) -> torch.Tensor:
    """[E, T] fp32 geometric random walks generated on the device (csrc/series.hip, Philox normals, one wave
    per series): the engines' synthetic price banks."""
    out = torch.empty(E, T, dtype=torch.float32, device=device)
    native.random_walk(out, float(start), float(vol), float(drift), int(key0), int(key1))
    return out


@random_walk.register_fake
def _(E, T, start, vol, drift, key0, key1, device):
    return torch.empty(E, T, dtype=torch.float32, device=device)


@custom_op(f"{NS}::tick16_quantize_", mutates_args=("bank",))
def tick16_quantize_(bank: torch.Tensor) -> None:
    """Every row of an [E, T] fp32 device bank onto its own 16-bit power-of-two tick grid, in place
    (csrc/series.hip tick16 mode 0; host mirror ``data.prices.tick16_quantize``)."""
    native.tick16_quantize_(bank)


@tick16_quantize_.register_fake
def _(bank):
    return None


@custom_op(f"{NS}::tick16", mutates_args=())
def tick16(bank: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """The 16-bit tick copy of an [E, T] fp32 bank that is on its tick grid: (ticks [E, T16] int16 holding
    u16, scale [E] fp32, price = tick * scale).  Both come back empty (0 rows) when some value is off the grid
    (the engine's fp32-window fallback)."""
    r = native.tick16(bank.contiguous(), quantize=False)
    if r is None:
        T16 = native.tick16_stride(bank.shape[1])
        return (torch.empty(0, T16, dtype=torch.int16, device=bank.device),
                torch.empty(0, dtype=torch.float32, device=bank.device))
    ticks, scale = r
    return ticks.clone(), scale


@tick16.register_fake
def _(bank):
    E, T = bank.shape
    T16 = native.tick16_stride(T)
    return bank.new_empty(E, T16, dtype=torch.int16), bank.new_empty(E, dtype=torch.float32)


@custom_op(f"{NS}::init_normal_", mutates_args=("block",))
def init_normal_(block: torch.Tensor, rows: int, cols: int, std: float, key0: int, key1: int, stream: int) -> None:
    """``block[:rows, :cols] = std * N(0, 1)`` from counter-based Philox draws (csrc/series.hip init_normal):
    the engines' weight initialisation, reproducible from (key, stream, index) alone."""
    native.init_normal(block, int(rows), int(cols), float(std), int(key0), int(key1), int(stream))


@init_normal_.register_fake
def _(block, rows, cols, std, key0, key1, stream):
    return None


OPS = ("gemm_nt", "qnet_select", "random_walk", "tick16_quantize_", "tick16", "init_normal_")
