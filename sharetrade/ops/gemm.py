"""Host wrapper of the bf16 MFMA GEMM (`csrc/gemm_bf16.hip`): ``C = A . B^T`` with
fused epilogues.  Shapes are validated on the host before any launch (the kernel
assumes whole tiles)."""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import native

EPI_BF16, EPI_RELU_GRAD, EPI_F32 = 0, 1, 2
# (BM, BN) or (BM, BN, LDS stages) -> st_gemm_nt tile id (csrc/gemm_bf16.hip)
TILES = {(128, 128): 0, (64, 64): 1, (128, 64): 2, (256, 128): 3, (128, 128, 3): 4, (128, 128, 4): 5,
         (256, 256): 6, (256, 256, "pp"): 7, (256, 256, "ppp"): 8, (256, 256, "w4"): 9}
# 7: 8-wave ping-pong, 8: the same with s_setprio on the MFMA segments, 9: 4 waves of 128x128 with
# fragment double buffering; 7-9 are gemm_nt only (no batch / C^T / split-K)


class GemmArgs(C.Structure):
    _fields_ = [
        ("A", C.c_void_p), ("B", C.c_void_p), ("out", C.c_void_p), ("outT", C.c_void_p), ("bias", C.c_void_p),
        ("auxT", C.c_void_p), ("M", C.c_int), ("N", C.c_int), ("K", C.c_int), ("lda", C.c_int), ("ldb", C.c_int),
        ("ldo", C.c_int), ("ldoT", C.c_int), ("ldaux", C.c_int), ("relu", C.c_int), ("accumulate", C.c_int),
        ("alpha", C.c_float), ("splitk", C.c_int), ("colpart", C.c_void_p), ("ldcp", C.c_int),
        ("qw", C.c_void_p), ("qpart", C.c_void_p), ("ldqw", C.c_int), ("nq", C.c_int), ("nqp", C.c_int),
    ]


def _bind():
    L = native.lib()
    if not getattr(L, "_gemm_bound", False):
        L.st_gemm_nt.argtypes = [C.POINTER(GemmArgs), C.c_int, C.c_int, C.c_void_p]
        L.st_gemm_nt.restype = C.c_int
        L.st_gemm_nt_batched.argtypes = [C.POINTER(GemmArgs), C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.st_gemm_nt_batched.restype = C.c_int
        L.st_gemm_dual.argtypes = [C.POINTER(GemmArgs), C.c_int, C.POINTER(GemmArgs), C.c_int, C.c_void_p]
        L.st_gemm_dual.restype = C.c_int
        L._gemm_bound = True
    return L


def pick_tile(M: int, N: int) -> tuple:
    """128x128 when that still gives >= ~256 workgroups, else smaller tiles."""
    if M % 128 == 0 and N % 128 == 0 and (M // 128) * (N // 128) >= 200:
        return (128, 128)
    if M % 128 == 0 and N % 64 == 0 and (M // 128) * (N // 64) >= 200:
        return (128, 64)
    return (64, 64)


def make_args(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, epi: int, outT: Optional[torch.Tensor] = None,
              bias: Optional[torch.Tensor] = None, auxT: Optional[torch.Tensor] = None, relu: bool = False,
              accumulate: bool = False, alpha: float = 1.0, splitk: int = 1,
              colpart: Optional[torch.Tensor] = None, qhead=None) -> GemmArgs:
    """``colpart`` (EPI_RELU_GRAD, 128-row 2-stage tiles): fp32 [M / 64, >= N] -- column sums of the bf16 output
    over each 64-row wave block (the bias gradient's partials).  ``qhead = (W, qpart)`` (EPI_BF16, 2-stage tiles):
    the next layer's head rows W bf16 [nq <= 4, >= N] folded into the epilogue -- qpart fp32 [N / WN, M, 4] gets
    per row the sums of output x W[a] over each wave's WN = BN / 2 columns (csrc/gemm_bf16.hip GemmArgs::qpart)."""
    M, K = A.shape
    N, K2 = B.shape
    if K != K2:
        raise ValueError(f"gemm_nt: K mismatch {A.shape} x {B.shape}^T")
    if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16:
        raise TypeError("gemm_nt operands must be bf16")
    if A.stride(1) != 1 or B.stride(1) != 1 or out.stride(1) != 1:
        raise ValueError("gemm_nt needs row-major (K-contiguous) operands")
    if tuple(out.shape) != (M, N):
        raise ValueError(f"gemm_nt: out {tuple(out.shape)} != {(M, N)}")
    if epi == EPI_F32 and out.dtype != torch.float32:
        raise TypeError("EPI_F32 writes fp32")
    if epi != EPI_F32 and out.dtype != torch.bfloat16:
        raise TypeError("bf16 epilogues write bf16")
    if outT is not None and tuple(outT.shape) != (N, M):
        raise ValueError("outT must be [N, M]")
    if auxT is not None and tuple(auxT.shape) != (N, M):
        raise ValueError("auxT must be [N, M]")
    if bias is not None and bias.numel() < N:
        raise ValueError("bias too short")
    g = GemmArgs()
    g.A, g.B, g.out = A.data_ptr(), B.data_ptr(), out.data_ptr()
    g.outT = outT.data_ptr() if outT is not None else None
    g.bias = bias.data_ptr() if bias is not None else None
    g.auxT = auxT.data_ptr() if auxT is not None else None
    g.M, g.N, g.K = M, N, K
    g.lda, g.ldb, g.ldo = A.stride(0), B.stride(0), out.stride(0)
    g.ldoT = outT.stride(0) if outT is not None else 0
    g.ldaux = auxT.stride(0) if auxT is not None else 0
    g.relu, g.accumulate, g.alpha = int(relu), int(accumulate), float(alpha)
    if splitk > 1:
        if epi != EPI_F32:
            raise ValueError("split-K needs the fp32 epilogue (atomic accumulation)")
        if (K // 64) % splitk:
            raise ValueError(f"split-K {splitk} does not divide the {K // 64} K-tiles")
    g.splitk = int(splitk)
    if colpart is not None:
        if epi != EPI_RELU_GRAD or colpart.dtype != torch.float32 or colpart.stride(1) != 1 or colpart.shape[1] < N:
            raise ValueError("colpart: EPI_RELU_GRAD, fp32 [M / 64, >= N] row-major")
        g.colpart, g.ldcp = colpart.data_ptr(), colpart.stride(0)
    if qhead is not None:
        qw, qp = qhead
        if (epi != EPI_BF16 or qw.dtype != torch.bfloat16 or qw.stride(1) != 1 or not 1 <= qw.shape[0] <= 4 or
                qw.shape[1] < N or qp.dtype != torch.float32 or not qp.is_contiguous() or qp.dim() != 3 or
                qp.shape[1] != M or qp.shape[2] != 4 or splitk > 1):
            raise ValueError("qhead: EPI_BF16, W bf16 [<= 4, >= N], qpart fp32 contiguous [N / WN, M, 4], no split-K")
        g.qw, g.qpart, g.ldqw, g.nq, g.nqp = qw.data_ptr(), qp.data_ptr(), qw.stride(0), qw.shape[0], qp.shape[0]
    return g


def pick_splitk(M: int, N: int, K: int, tile) -> int:
    """Split K until the launch has >= ~256 workgroups (one per CU) or the K-tiles run out."""
    wg = (M // tile[0]) * (N // tile[1])
    s = 1
    while wg * s < 256 and (K // 64) % (2 * s) == 0 and K // 64 // (2 * s) >= 4:
        s *= 2
    return s


PINGPONG = True   # auto_tile may pick the ping-pong kernel (benchmarks/bench_deep.py --no-pingpong turns it off)


def auto_tile(M: int, N: int, epi: int, kw: dict) -> tuple:
    """The 256x256 ping-pong kernel where it applies (bf16 / fp32 epilogue without C^T or split-K) and
    its tiles fill every CU (measured faster from 256 tiles up: profiles/r2_gemm_pingpong.md), else
    pick_tile."""
    if (PINGPONG and epi != EPI_RELU_GRAD and kw.get("outT") is None and kw.get("splitk", 1) in (1, "auto") and
            M % 256 == 0 and N % 256 == 0 and (M // 256) * (N // 256) >= 256):
        return (256, 256, "pp")
    return pick_tile(M, N)


def gemm_nt(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, epi: int = EPI_BF16, tile=None, **kw) -> torch.Tensor:
    """``out = A . B^T`` (+ epilogue).  ``splitk="auto"`` (fp32 epilogue only) splits long-K,
    few-tile products (weight gradients) over extra workgroups with atomic accumulation."""
    t = tile or auto_tile(A.shape[0], B.shape[0], epi, kw)
    if len(t) == 3 and t[2] in ("pp", "ppp", "w4") and kw.get("splitk", 1) == "auto":
        kw = dict(kw, splitk=1)
    sk = kw.pop("splitk", 1)
    prezeroed = kw.pop("prezeroed", False)   # split-K output already zeroed by an earlier kernel
    if sk == "auto":
        sk = pick_splitk(A.shape[0], B.shape[0], A.shape[1], t) if epi == EPI_F32 else 1
    if sk > 1 and not kw.get("accumulate", False) and not prezeroed:
        out.zero_()
    g = make_args(A, B, out, epi, splitk=sk, **kw)
    if g.M % t[0] or g.N % t[1] or g.K % 64:
        raise ValueError(f"gemm_nt: shape {g.M}x{g.N}x{g.K} not a multiple of tile {t} / BK 64")
    native.check(_bind().st_gemm_nt(g, epi, TILES[t], native.stream_handle()), "st_gemm_nt")
    return out


GEMM_MAXB = 4


def gemm_nt_batched(problems, epi: int = EPI_BF16, tile=None) -> None:
    """Up to 4 products ``out_i = A_i . B_i^T`` (one epilogue and tile; shapes and K splits may
    differ: a grouped GEMM) in ONE launch: ``problems`` is a list of ``(A, B, out, kwargs)``.
    Replaces a fork / join of concurrent streams (e.g. the online and target forward of one layer)
    by one grid that holds the tiles of all of them."""
    if not 1 <= len(problems) <= GEMM_MAXB:
        raise ValueError(f"gemm_nt_batched: 1..{GEMM_MAXB} problems")
    A0, B0 = problems[0][0], problems[0][1]
    t = tile or pick_tile(A0.shape[0], B0.shape[0])
    arr = (GemmArgs * len(problems))()
    for i, (A, B, out, kw) in enumerate(problems):
        kw = dict(kw)
        sk = kw.pop("splitk", 1)
        prezeroed = kw.pop("prezeroed", False)
        if sk > 1 and not kw.get("accumulate", False) and not prezeroed:
            out.zero_()
        g = make_args(A, B, out, epi, splitk=sk, **kw)
        if g.M % t[0] or g.N % t[1] or g.K % 64:
            raise ValueError(f"gemm_nt_batched: shape {g.M}x{g.N}x{g.K} not a multiple of tile {t} / BK 64")
        arr[i] = g
    native.check(_bind().st_gemm_nt_batched(arr, len(problems), epi, TILES[t], native.stream_handle()),
                 "st_gemm_nt_batched")


def gemm_dual(first, epi0: int, second, epi1: int) -> None:
    """Two products of any shapes / epilogues on 128x128 tiles in ONE launch (``first`` / ``second``
    = ``(A, B, out, kwargs)``; epilogue pairs relu-grad + f32, f32 + f32, bf16 + f32): e.g. a layer's
    data gradient beside the next layer's split-K weight gradient, with no stream fork / join."""
    args = []
    for (A, B, out, kw), epi in ((first, epi0), (second, epi1)):
        kw = dict(kw)
        sk = kw.pop("splitk", 1)
        prezeroed = kw.pop("prezeroed", False)
        if sk == "auto":
            sk = pick_splitk(A.shape[0], B.shape[0], A.shape[1], (128, 128)) if epi == EPI_F32 else 1
        if sk > 1 and not kw.get("accumulate", False) and not prezeroed:
            out.zero_()
        g = make_args(A, B, out, epi, splitk=sk, **kw)
        if g.M % 128 or g.N % 128 or g.K % 64:
            raise ValueError(f"gemm_dual: shape {g.M}x{g.N}x{g.K} not a multiple of 128x128 / BK 64")
        args.append(g)
    native.check(_bind().st_gemm_dual(args[0], epi0, args[1], epi1, native.stream_handle()), "st_gemm_dual")
