"""GRU(256) recurrent Q-network (BASELINE config 5): the plain-PyTorch reference.

Gate order and equations are exactly ``torch.nn.GRUCell`` (r, z, n)::

    r = sigma(W_ir x + b_ir + W_hr h + b_hr)
    z = sigma(W_iz x + b_iz + W_hz h + b_hz)
    n = tanh(W_in x + b_in + r * (W_hn h + b_hn))
    h' = (1 - z) * n + z * h          Q = W_q h' + b_q   (3 actions: Buy, Sell, Hold)

The HIP path (``csrc/gru.hip`` + bf16 GEMMs) keeps the same parameter tensors
(``w_ih [768, 64]`` -- the learner's x is zero-padded to a 64-wide GEMM K, the actor
reads the first 32 columns --, ``w_hh [768, 256]``, ``b_ih``, ``b_hh``, ``w_q [3, 256]``,
``b_q``), so this module is both the CPU implementation and the numerics oracle.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch

HID, GATES, X_ACT, X_PAD, N_ACT = 256, 768, 32, 64, 3


def init_params(seed: int = 0, hidden: int = HID, x_real: int = 12, device=None) -> Dict[str, torch.Tensor]:
    """torch.nn.GRUCell-style U(-1/sqrt(H), 1/sqrt(H)) init; small Q head."""
    g = torch.Generator().manual_seed(int(seed))
    k = 1.0 / math.sqrt(hidden)
    p = {
        "w_ih": torch.zeros(3 * hidden, X_PAD),
        "w_hh": (torch.rand(3 * hidden, hidden, generator=g) * 2 - 1) * k,
        "b_ih": (torch.rand(3 * hidden, generator=g) * 2 - 1) * k,
        "b_hh": (torch.rand(3 * hidden, generator=g) * 2 - 1) * k,
        "w_q": torch.randn(N_ACT, hidden, generator=g) * 0.01,
        "b_q": torch.zeros(N_ACT),
    }
    p["w_ih"][:, :x_real] = (torch.rand(3 * hidden, x_real, generator=g) * 2 - 1) * k
    return {n: t.to(device) if device is not None else t for n, t in p.items()}


def gru_cell(x: torch.Tensor, h: torch.Tensor, p: Dict[str, torch.Tensor]) -> torch.Tensor:
    H = h.shape[-1]
    gx = x @ p["w_ih"][:, : x.shape[-1]].t() + p["b_ih"]
    gh = h @ p["w_hh"].t() + p["b_hh"]
    r = torch.sigmoid(gx[..., :H] + gh[..., :H])
    z = torch.sigmoid(gx[..., H:2 * H] + gh[..., H:2 * H])
    n = torch.tanh(gx[..., 2 * H:] + r * gh[..., 2 * H:])
    return (1 - z) * n + z * h


def unroll(X: torch.Tensor, h0: torch.Tensor, p: Dict[str, torch.Tensor],
           done: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """X [T, B, F], h0 [B, H] -> (Q [T, B, 3], h_T).  ``done[t]`` resets h after step t."""
    h = h0
    qs = []
    for t in range(X.shape[0]):
        h = gru_cell(X[t], h, p)
        qs.append(h @ p["w_q"].t() + p["b_q"])
        if done is not None and t < done.shape[0]:
            h = h * (1 - done[t])[:, None]
    return torch.stack(qs), h


def sequence_td_loss(p: Dict[str, torch.Tensor], pt: Dict[str, torch.Tensor], X: torch.Tensor, h0: torch.Tensor,
                     A: torch.Tensor, R: torch.Tensor, D: torch.Tensor, gamma: float, burn: int) -> torch.Tensor:
    """Double-DQN loss over a segment (the learner's objective; csrc/gru.hip gru_td_kernel).

    X [S+1, B, F] (obs 0..S), A/R/D [S, B]; online and target nets both unroll from the
    stored segment-start state h0; loss = mean over t in [burn, S) of (Q(s_t, a_t) - y_t)^2,
    y_t = r_t + gamma (1 - d_t) Q_target(s_{t+1}, argmax_a Q_online(s_{t+1}, a)).
    """
    S = A.shape[0]
    q, _ = unroll(X, h0, p, D)
    with torch.no_grad():
        qt, _ = unroll(X, h0, pt, D)
        a_star = q[1:].argmax(-1, keepdim=True)
        y = R + gamma * (1 - D) * qt[1:].gather(-1, a_star)[..., 0]
    qa = q[:S].gather(-1, A.long()[..., None])[..., 0]
    return ((qa - y)[burn:] ** 2).mean()
