"""Batched SelectionAction inference: the ``csrc/qserve.hip`` launch and its fp32 PyTorch oracle.

Reference: ``QDecisionPolicyActor.scala:56-62`` answers one ``SelectionAction(state [1,203], step)``
per TF session run (forward, host argmax, ``scala.util.Random`` epsilon-greedy with exploit
probability ``min(0.9, step/1000)``).  Here a batch of request rows in the reference's state layout
(``TrainerChildActor.scala:90-91``: 201 prices, budget, shares) is answered by one persistent HIP
launch over the flagship 2x128 bf16 Q-net (``csrc/qserve.hip``).  :func:`reference_select` is the
same computation in PyTorch (bf16 rounding emulated where the kernel rounds, fp32 elsewhere) and the
same Philox draws: the numerics oracle of ``tests/test_gpu_serve.py`` and the CPU backend of
:class:`~sharetrade.serve.server.PolicyServer`.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..env import trading as tr
from ..models import qnet as qn
from ..ops import native
from ..utils import rng

SERVE_STREAM = 2          # Philox counter word 3 of the serving draws: (row, seq_lo, seq_hi, 2)
PADDED_DIMS = (224, 128, 128)


class ServeParams(C.Structure):
    _fields_ = [
        ("states", C.c_void_p), ("steps", C.c_void_p), ("wq", C.c_void_p), ("wf", C.c_void_p),
        ("q_out", C.c_void_p), ("actions", C.c_void_p),
        ("B", C.c_int), ("ld", C.c_int), ("H", C.c_int),
        ("off_w0", C.c_int), ("off_w1", C.c_int), ("off_b1", C.c_int), ("off_w2", C.c_int), ("off_b2", C.c_int),
        ("feat_mode", C.c_int), ("output_relu", C.c_int),
        ("inv_b0", C.c_float), ("eps", C.c_float), ("inv_ramp", C.c_float),
        ("key0", C.c_uint32), ("key1", C.c_uint32),
        ("seq", C.c_ulonglong),
    ]


_bound = False


def _lib() -> C.CDLL:
    global _bound
    L = native.lib()
    if not _bound:
        L.st_qserve_launch.argtypes = [C.POINTER(ServeParams), C.c_int, C.c_void_p]
        L.st_qserve_launch.restype = C.c_int
        L.st_qserve_lds_bytes.restype = C.c_int
        _bound = True
    return L


def supported(layout: qn.QNetLayout) -> bool:
    """The serving kernel is built for the flagship padded dims (224 -> 128 -> 128 -> 16)."""
    return tuple(layout.pdims) == PADDED_DIMS + (qn.OUT_PAD,) and layout.n_layers == 3


class ServeKernel:
    """One reusable parameter block for ``st_qserve_launch`` (weights by pointer: the caller keeps
    ``params`` / ``params_bf`` alive and may update them in place between launches)."""

    def __init__(self, layout: qn.QNetLayout, params: torch.Tensor, params_bf: torch.Tensor, *,
                 history: int, feat_mode: int, output_relu: bool, budget0: float, epsilon: float,
                 ramp: float, key: Tuple[int, int]):
        if not supported(layout):
            raise NotImplementedError(f"serving kernel needs padded dims {PADDED_DIMS}, got {layout.pdims}")
        if history + 3 > PADDED_DIMS[0] or layout.input_dim != history + 2:
            raise ValueError(f"history {history} does not fit the {PADDED_DIMS[0]}-wide input")
        seg = layout.segments
        p = ServeParams()
        p.wq, p.wf = native.ptr(params_bf), native.ptr(params)
        p.H = int(history)
        p.off_w0, p.off_w1, p.off_b1 = seg["W0"].offset, seg["W1"].offset, seg["b1"].offset
        p.off_w2, p.off_b2 = seg["W2"].offset, seg["b2"].offset
        p.feat_mode, p.output_relu = int(feat_mode), int(bool(output_relu))
        p.inv_b0 = float(np.float32(1.0 / budget0))
        p.eps, p.inv_ramp = float(epsilon), float(np.float32(1.0 / ramp))
        p.key0, p.key1 = int(key[0]), int(key[1])
        self.p = p
        self._keep = (params, params_bf)

    def launch(self, states: torch.Tensor, actions: torch.Tensor, q_out: Optional[torch.Tensor] = None,
               steps: Optional[torch.Tensor] = None, seq: int = 0, grid: int = 0) -> None:
        """``states`` [B, >= H+2] fp32 (row stride = ``states.stride(0)``), ``actions`` [B] int32,
        ``q_out`` [B, 3] fp32 or None, ``steps`` [B] fp32 or None (greedy).  Current stream."""
        B = int(states.shape[0])
        if states.dtype != torch.float32 or states.stride(1) != 1 or states.shape[1] < self.p.H + 2:
            raise ValueError("states must be fp32 rows of >= H + 2 values, unit column stride")
        if actions.dtype != torch.int32 or actions.numel() < B or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous int32 buffer of >= B entries")
        if q_out is not None and (q_out.dtype != torch.float32 or q_out.numel() < 3 * B or not q_out.is_contiguous()):
            raise ValueError("q_out must be a contiguous fp32 buffer of >= 3 B entries")
        if steps is not None and (steps.dtype != torch.float32 or steps.numel() < B or not steps.is_contiguous()):
            raise ValueError("steps must be a contiguous fp32 buffer of >= B entries")
        p = self.p
        p.states, p.ld, p.B = native.ptr(states), int(states.stride(0)), B
        p.actions, p.q_out, p.steps = native.ptr(actions), native.ptr(q_out), native.ptr(steps)
        p.seq = int(seq) & 0xFFFFFFFFFFFFFFFF
        native.check(_lib().st_qserve_launch(C.byref(p), int(grid), native.stream_handle()), "st_qserve_launch")


def reference_select(params: torch.Tensor, layout: qn.QNetLayout, states: torch.Tensor, *, history: int,
                     feat_mode: str, output_relu: bool, budget0: float, epsilon: float, ramp: float,
                     key_seed: int, seq: int = 0, steps: Optional[Union[Sequence[float], torch.Tensor]] = None,
                     emulate_bf16: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """(actions int32 [B], q fp32 [B, 3]) for raw request rows [B, H+2] (CPU or GPU tensors)."""
    x = states[:, : history + 2].float()
    H = history
    feats = tr.features(x[:, :H], x[:, H], x[:, H + 1], feat_mode, budget0)
    q, _, _ = qn.forward(params.float().to(x.device), layout, feats, output_relu, emulate_bf16=emulate_bf16)
    q = q[:, : layout.n_actions]
    greedy = torch.argmax(q, dim=1).to(torch.int32)   # first max on ties (TF ArgMax)
    if steps is None:
        return greedy, q
    B = x.shape[0]
    u1, u2 = rng.uniforms(key_seed, 0, np.arange(B, dtype=np.uint32), seq, stream=SERVE_STREAM)
    st = torch.as_tensor(steps, dtype=torch.float32).cpu().numpy()
    thr = np.minimum(np.float32(epsilon), st.astype(np.float32) * np.float32(1.0 / ramp))
    exploit = torch.from_numpy(u1 < thr).to(x.device)
    rnd = torch.from_numpy(np.minimum((u2 * np.float32(3)).astype(np.int64), 2)).to(x.device)
    return torch.where(exploit, greedy.long(), rnd).to(torch.int32), q
