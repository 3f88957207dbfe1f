"""Host bindings of the GRU(256) recurrent Q-net kernels (``csrc/gru.hip``) plus the
plain-PyTorch references of the MX-fp8 block quantization the actor uses.

MX-fp8 (OCP microscaling): a block of 32 values shares one E8M0 scale ``2^e``; each
value is stored as OCP ``e4m3fn`` of ``x / 2^e``.  The kernel picks the smallest ``e``
with ``amax / 2^e <= 448`` (``mx_exp``), so nothing saturates.  The references here
follow the same rule bit for bit on the host (``torch.float8_e4m3fn`` does the
rounding), which is what the GPU numerics tests compare against.

Operand layout of ``v_mfma_scale_f32_16x16x128_f8f6f4`` (measured on gfx950 with
``tools/mx_layout_probe.py``): lane ``l = i + 16q`` holds row (A) / column (B) ``i``;
its bytes 0..15 are K ``16q + [0,16)`` and bytes 16..31 are K ``64 + 16q + [0,16)``; the
E8M0 scale of (row i, K-block ``s`` = ``[32s, 32s+32)``) is taken from lane ``i + 16s``.

Fragment layout of the packed actor weights (``gru_pack_kernel``): for wave ``w``
(units 32w..32w+31), gate ``g`` (r, z, n), 16-row tile ``m``, K-step ``ks`` and lane
``l``: row ``g*256 + 32w + 16m + (l & 15)``, K columns ``128ks + {16q.., 64+16q..}``
as above, and ``whhs`` holds the exponent of K-block ``q`` of that row.
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import numpy as np
import torch

from . import native

HID, GATES, XA, XL, NMF = 256, 768, 32, 64, 8
RW, RN, LB, NSV = 8, 32, 32, 5


class MinuteBarsArgs(C.Structure):
    _fields_ = [("close", C.c_void_p), ("feat", C.c_void_p), ("E", C.c_int), ("T", C.c_int), ("day", C.c_int),
                ("sigma", C.c_float), ("phi", C.c_float), ("alpha", C.c_float), ("beta", C.c_float),
                ("p0", C.c_float), ("key0", C.c_uint32), ("key1", C.c_uint32)]


class PackArgs(C.Structure):
    _fields_ = [("w_hh", C.c_void_p), ("w_ih", C.c_void_p), ("b_ih", C.c_void_p), ("b_hh", C.c_void_p),
                ("w_q", C.c_void_p), ("b_q", C.c_void_p), ("whh8", C.c_void_p), ("whhs", C.c_void_p),
                ("wih", C.c_void_p), ("bias4", C.c_void_p), ("wq", C.c_void_p), ("whhT8", C.c_void_p),
                ("whhTs", C.c_void_p)]


class ActArgs(C.Structure):
    _fields_ = [("whh8", C.c_void_p), ("whhs", C.c_void_p), ("wih", C.c_void_p), ("bias4", C.c_void_p),
                ("wq", C.c_void_p), ("feat", C.c_void_p), ("close", C.c_void_p), ("ret", C.c_void_p),
                ("E", C.c_int), ("T", C.c_int), ("S", C.c_int), ("ep_len", C.c_int),
                ("eps", C.c_float), ("inv_ramp", C.c_float), ("cost", C.c_float), ("inv_ep_len", C.c_float),
                ("h", C.c_void_p), ("pos", C.c_void_p), ("ep_start", C.c_void_p), ("position", C.c_void_p),
                ("entry", C.c_void_p), ("ep_ret", C.c_void_p), ("episodes", C.c_void_p), ("last_ret", C.c_void_p),
                ("rx", C.c_void_p), ("ra", C.c_void_p), ("rr", C.c_void_p), ("rd", C.c_void_p), ("rh0", C.c_void_p),
                ("rctrl", C.c_void_p), ("cap", C.c_int), ("key0", C.c_uint32), ("key1", C.c_uint32),
                ("ctrl", C.c_void_p), ("stats", C.c_void_p), ("q_out", C.c_void_p), ("stamps", C.c_void_p),
                ("done_ctr", C.c_void_p)]


class GatherArgs(C.Structure):
    _fields_ = [("rx", C.c_void_p), ("ra", C.c_void_p), ("rr", C.c_void_p), ("rd", C.c_void_p), ("rh0", C.c_void_p),
                ("rctrl", C.c_void_p), ("cap", C.c_int), ("S", C.c_int), ("B", C.c_int), ("key0", C.c_uint32),
                ("key1", C.c_uint32), ("step", C.c_void_p), ("X", C.c_void_p), ("H0", C.c_void_p),
                ("A", C.c_void_p), ("R", C.c_void_p), ("D", C.c_void_p)]


class NetW(C.Structure):
    _fields_ = [("whh8", C.c_void_p), ("whhs", C.c_void_p), ("wih", C.c_void_p), ("bias4", C.c_void_p),
                ("wq", C.c_void_p)]


class SeqFwdArgs(C.Structure):
    _fields_ = [("on", NetW), ("tg", NetW), ("X", C.c_void_p), ("H0", C.c_void_p), ("D", C.c_void_p),
                ("Q", C.c_void_p), ("Qt", C.c_void_p), ("HT", C.c_void_p), ("ldht", C.c_int), ("sv", C.c_void_p),
                ("B", C.c_int), ("S", C.c_int)]


class TDArgs(C.Structure):
    _fields_ = [("Q", C.c_void_p), ("Qt", C.c_void_p), ("A", C.c_void_p), ("R", C.c_void_p), ("D", C.c_void_p),
                ("dQ", C.c_void_p), ("loss", C.c_void_p), ("B", C.c_int), ("S", C.c_int), ("burn", C.c_int),
                ("gamma", C.c_float), ("coef", C.c_float)]


class SeqBwdArgs(C.Structure):
    _fields_ = [("sv", C.c_void_p), ("dQ", C.c_void_p), ("D", C.c_void_p), ("whhT8", C.c_void_p),
                ("whhTs", C.c_void_p), ("wq", C.c_void_p), ("dGxT", C.c_void_p), ("dGhT", C.c_void_p),
                ("gwq", C.c_void_p), ("gbq", C.c_void_p), ("B", C.c_int), ("S", C.c_int)]


def lib():
    L = native.lib()
    if not getattr(L, "_gru_bound", False):
        vp, i = C.c_void_p, C.c_int
        for fn, args in (("st_minute_bars", [C.POINTER(MinuteBarsArgs), vp]),
                         ("st_gru_pack", [C.POINTER(PackArgs), vp]),
                         ("st_gru_act", [C.POINTER(ActArgs), i, vp]),
                         ("st_gru_act_pair", [C.POINTER(ActArgs), i, vp]),
                         ("st_gru_gather", [C.POINTER(GatherArgs), vp]),
                         ("st_gru_seq_fwd", [C.POINTER(SeqFwdArgs), vp]),
                         ("st_gru_td", [C.POINTER(TDArgs), vp]),
                         ("st_gru_seq_bwd", [C.POINTER(SeqBwdArgs), vp]),
                         ("st_gru_grad_fixup", [vp, i, vp, vp, vp, vp, vp]),
                         ("st_mx_probe", [vp, vp, vp, vp, vp, vp])):
            f = getattr(L, fn)
            f.argtypes = args
            f.restype = C.c_int
        L.st_gru_act_lds_bytes.restype = C.c_int
        L.st_gru_act_pair_smax.restype = C.c_int
        L._gru_bound = True
    return L


# ---------------------------------------------------------------------------- MX-fp8 references
def mx_exp(amax: torch.Tensor) -> torch.Tensor:
    """Per-block E8M0 exponent: smallest e with amax / 2^e <= 448 (bit-exact with csrc/gru.hip)."""
    a = amax.float()
    m, e = torch.frexp(a * torch.tensor(1.0 / 448.0, dtype=torch.float32))
    e = e.to(torch.int32) - (m == 0.5).to(torch.int32)
    e = e + (torch.ldexp(a, -e.float()) > 448.0).to(torch.int32)
    e = torch.where(a > 0, e, torch.full_like(e, -127))
    return e.clamp(-127, 127)


def mx_quantize(x: torch.Tensor, block: int = 32) -> Tuple[torch.Tensor, torch.Tensor]:
    """x[..., K] fp32 -> (fp8 e4m3fn [..., K], int32 exponents [..., K/block])."""
    xb = x.float().reshape(*x.shape[:-1], x.shape[-1] // block, block)
    e = mx_exp(xb.abs().amax(-1))
    q = torch.ldexp(xb, -e.float()[..., None]).to(torch.float8_e4m3fn)
    return q.reshape(x.shape), e


def mx_dequantize(q: torch.Tensor, e: torch.Tensor, block: int = 32) -> torch.Tensor:
    qb = q.float().reshape(*q.shape[:-1], q.shape[-1] // block, block)
    return torch.ldexp(qb, e.float()[..., None]).reshape(q.shape)


def mx_roundtrip(x: torch.Tensor, block: int = 32) -> torch.Tensor:
    q, e = mx_quantize(x, block)
    return mx_dequantize(q, e, block)


# gate pre-scales folded into the packed weights and biases (csrc/gru_common.h GS_RZ / GS_N): the kernels
# evaluate sigmoid / tanh as exp2 + add + rcp on the pre-scaled pre-activations
GS_RZ = float(np.float32(-1.44269504))
GS_N = float(np.float32(-2.88539008))


def gate_prescale() -> torch.Tensor:
    """Per gate row (r, z, n blocks of 256) scale the packed W_hh / W_ih rows and biases carry, fp32 [768]."""
    return torch.cat([torch.full((2 * HID,), GS_RZ), torch.full((HID,), GS_N)]).float()


def unpack_whh(whh8: torch.Tensor, whhs: torch.Tensor, unscale: bool = True) -> torch.Tensor:
    """Packed actor fragments -> the dequantized W_hh [768, 256] the actor multiplies with; ``unscale``
    divides out the gate pre-scale (:func:`gate_prescale`), else the raw pre-scaled values."""
    b = whh8.detach().cpu().contiguous().view(torch.uint8).view(RW, 3, 2, 2, 64, 32)
    e = whhs.detach().cpu().view(RW, 3, 2, 2, 64).to(torch.int32) - 127
    vals = b.view(torch.float8_e4m3fn).float()
    W = torch.zeros(GATES, HID)
    for w in range(RW):
        for g in range(3):
            for m in range(2):
                for ks in range(2):
                    for l in range(64):
                        i, q = l & 15, l >> 4
                        r = g * HID + 32 * w + 16 * m + i
                        for half, k0 in ((0, 16 * q), (1, 64 + 16 * q)):
                            blk = k0 // 32
                            sc = 2.0 ** float(e[w, g, m, ks, i + 16 * blk])
                            W[r, 128 * ks + k0:128 * ks + k0 + 16] = vals[w, g, m, ks, l, 16 * half:16 * half + 16] * sc
    if unscale:
        W = (W.double() / gate_prescale().double()[:, None]).float()
    return W


def unpack_whhT(whhT8: torch.Tensor, whhTs: torch.Tensor) -> torch.Tensor:
    """Backward-pack fragments (W_hh^T rows = units, K = gate rows) -> the dequantized W_hh [768, 256]
    the learner's dh GEMM multiplies with (32-gate blocks per unit, so it differs from unpack_whh)."""
    b = whhT8.detach().cpu().contiguous().view(torch.uint8).view(RW, 2, 6, 64, 32)
    e = whhTs.detach().cpu().view(RW, 2, 6, 64).to(torch.int32) - 127
    vals = b.view(torch.float8_e4m3fn).float()
    WT = torch.zeros(HID, GATES)
    for w in range(RW):
        for m in range(2):
            for ks in range(6):
                for l in range(64):
                    i, q = l & 15, l >> 4
                    u = 32 * w + 16 * m + i
                    for half, k0 in ((0, 16 * q), (1, 64 + 16 * q)):
                        sc = 2.0 ** float(e[w, m, ks, i + 16 * (k0 // 32)])
                        WT[u, 128 * ks + k0:128 * ks + k0 + 16] = vals[w, m, ks, l, 16 * half:16 * half + 16] * sc
    return WT.t().contiguous()


def mx_probe(a: torch.Tensor, b: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor) -> torch.Tensor:
    """One v_mfma_scale_f32_16x16x128_f8f6f4 on raw fragments: a, b uint8 [64, 32]; sa, sb int32 [64] (E8M0).
    Returns the fp32 16x16 D tile (row = 4*(lane>>4) + reg, col = lane & 15)."""
    d = torch.zeros(64, 4, dtype=torch.float32, device=a.device)
    native.check(lib().st_mx_probe(a.data_ptr(), b.data_ptr(), sa.data_ptr(), sb.data_ptr(), d.data_ptr(),
                                   native.stream_handle()), "st_mx_probe")
    D = torch.zeros(16, 16, dtype=torch.float32, device=a.device)
    lane = torch.arange(64, device=a.device)
    for r in range(4):
        D[4 * (lane >> 4) + r, lane & 15] = d[:, r]
    return D
