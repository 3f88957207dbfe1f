"""ctypes bindings to the in-tree HIP kernel library (``libsharetrade_hip.so``).

The kernels are plain C-ABI entry points (``csrc/*.hip``); tensors are
allocated by PyTorch's caching allocator and passed by device pointer, and
every launch goes onto PyTorch's *current* HIP stream, so the calls compose
with ``torch.cuda.graph`` capture and with RCCL collectives on the same stream.

If the library is missing while a GPU is present, :func:`lib` raises — the
engine never silently falls back to a non-native path on a GPU box.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "_native")
HIP_LIB_PATH = os.path.join(LIB_DIR, "libsharetrade_hip.so")

_lib: Optional[C.CDLL] = None


class NativeUnavailable(RuntimeError):
    pass


class QStepParams(C.Structure):
    _fields_ = [
        ("prices", C.c_void_p), ("prices4", C.c_void_p), ("env", C.c_void_p),
        ("wq", C.c_void_p), ("wf", C.c_void_p), ("slab", C.c_void_p), ("stats", C.c_void_p), ("ctrl", C.c_void_p),
        ("T", C.c_int), ("E", C.c_int), ("H", C.c_int), ("P", C.c_int), ("T4", C.c_int),
        ("off_w0", C.c_int), ("off_w1", C.c_int), ("off_b1", C.c_int), ("off_w2", C.c_int), ("off_b2", C.c_int),
        ("eps", C.c_float), ("inv_ramp", C.c_float), ("gamma", C.c_float), ("loss_coef", C.c_float),
        ("b0", C.c_float), ("inv_b0", C.c_float),
        ("s0", C.c_int), ("compat_env", C.c_int), ("target_compat", C.c_int), ("output_relu", C.c_int),
        ("feat_mode", C.c_int),
        ("key0", C.c_uint32), ("key1", C.c_uint32),
        ("env_offset", C.c_int),
        ("stamps", C.c_void_p),
        ("slab_bf16", C.c_int), ("slab_rows", C.c_int),
        ("chunk_heads", C.c_void_p),
        ("reward_mode", C.c_int), ("td_clip", C.c_float),
        ("err", C.c_void_p),
        ("reward_scale", C.c_float), ("ramp_global", C.c_int), ("qt", C.c_void_p), ("double_dqn", C.c_int),
        ("wimg", C.c_void_p),
        ("ticks", C.c_void_p), ("tscale", C.c_void_p), ("T16", C.c_int),
    ]


# csrc/qtarget.hip launch variants: (16-env tiles per wave, waves per workgroup)
QTARGET_VARIANTS = {0: (4, 4), 1: (2, 8), 2: (1, 8), 3: (1, 16)}


class QTargetParams(C.Structure):
    """csrc/qtarget.hip: target-net values of the three candidate next states of every env."""
    _fields_ = [
        ("prices4", C.c_void_p), ("env", C.c_void_p), ("wt", C.c_void_p), ("qt", C.c_void_p),
        ("T", C.c_int), ("E", C.c_int), ("T4", C.c_int),
        ("off_w0", C.c_int), ("off_w1", C.c_int), ("off_b1", C.c_int), ("off_w2", C.c_int), ("off_b2", C.c_int),
        ("b0", C.c_float), ("inv_b0", C.c_float),
        ("s0", C.c_int), ("compat_env", C.c_int), ("output_relu", C.c_int), ("feat_mode", C.c_int),
        ("wimg", C.c_void_p),
        ("ticks", C.c_void_p), ("tscale", C.c_void_p), ("T16", C.c_int),
    ]


class OptimParams(C.Structure):
    _fields_ = [
        ("params", C.c_void_p), ("params_bf", C.c_void_p), ("mask", C.c_void_p), ("s1", C.c_void_p),
        ("s2", C.c_void_p), ("slab", C.c_void_p), ("grad", C.c_void_p), ("ctrl", C.c_void_p),
        ("stats", C.c_void_p), ("stat_acc", C.c_void_p),
        ("G", C.c_int), ("P", C.c_int), ("kind", C.c_int), ("mode", C.c_int), ("nstat", C.c_int),
        ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float), ("scale", C.c_float),
        ("tdelay", C.c_int), ("slab_bf16", C.c_int),
        ("chunk_heads", C.c_void_p),
        ("ema", C.c_void_p), ("ema_decay", C.c_float),
        ("img_map", C.c_void_p), ("img", C.c_void_p),
    ]


# rows of QStepParams::env (csrc/qstep_fused.hip EnvRow): int32 / fp32 words
ENV_ROWS = ("pos", "budget", "shares", "value", "ret_sum", "episodes", "last_final", "actions_out", "rewards_out")


# Timing / debug builds of the flagship step kernel (csrc/ab/*.hip: per-phase stamps, phases skipped or
# run twice to price them).  They are NOT in the production library: `python build.py --ab` (or
# SHARETRADE_AB_BUILDS=1) builds them into their own libsharetrade_ab.so, and nothing loads it unless
# SHARETRADE_AB_BUILDS=1 is set.  Builds in WRONG_RESULT_VARIANTS compute wrong results by design.
AB_LIB_PATH = os.path.join(LIB_DIR, "libsharetrade_ab.so")
WRONG_RESULT_VARIANTS = frozenset({"gskip", "gskipst", "l1x2", "l2x2", "nopf", "nowb", "nophil"})
_ab_lib: Optional[C.CDLL] = None


def ab_builds_enabled() -> bool:
    return os.environ.get("SHARETRADE_AB_BUILDS", "") not in ("", "0")


def ab_lib() -> C.CDLL:
    global _ab_lib
    if not ab_builds_enabled():
        raise RuntimeError("timing / debug kernel builds are opt-in: set SHARETRADE_AB_BUILDS=1 and run "
                           "`python build.py --ab` (csrc/ab/*.hip -> libsharetrade_ab.so)")
    if _ab_lib is None:
        if not os.path.exists(AB_LIB_PATH):
            raise NativeUnavailable(f"{AB_LIB_PATH} not built: run `SHARETRADE_AB_BUILDS=1 python build.py`")
        lib()   # the production library first (HIP runtime, shared entry points)
        _ab_lib = C.CDLL(AB_LIB_PATH)
    return _ab_lib


def variant_launch(suffix: str, prefix: str = "st_qstep_ws_launch_"):
    """``<prefix><suffix>`` of a timing / debug build of a step kernel (same params), from the opt-in
    A/B library.  Refused unless SHARETRADE_AB_BUILDS=1: several of these builds compute wrong results
    on purpose (WRONG_RESULT_VARIANTS) and must never be selected by a production config."""
    if not ab_builds_enabled():
        bad = " (computes WRONG results by design)" if suffix in WRONG_RESULT_VARIANTS else ""
        raise RuntimeError(f"engine.step_variant={suffix!r}{bad} needs SHARETRADE_AB_BUILDS=1")
    fn = getattr(ab_lib(), prefix + suffix)
    fn.argtypes = [C.POINTER(QStepParams), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    fn.restype = C.c_int
    return fn


def available() -> bool:
    return os.path.exists(HIP_LIB_PATH)


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(HIP_LIB_PATH):
        raise NativeUnavailable(
            f"{HIP_LIB_PATH} not built: run `python build.py` (hipcc --offload-arch=gfx950)")
    L = C.CDLL(HIP_LIB_PATH)
    L.st_qstep_launch.argtypes = [C.POINTER(QStepParams), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.st_qstep_launch.restype = C.c_int
    L.st_qstep_lds_bytes.argtypes = [C.c_int, C.c_int, C.c_int]
    L.st_qstep_lds_bytes.restype = C.c_int
    L.st_qstep_wide_launch.argtypes = [C.POINTER(QStepParams), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.st_qstep_wide_launch.restype = C.c_int
    L.st_qstep_wide_lds_bytes.argtypes = [C.c_int, C.c_int, C.c_int]
    L.st_qstep_wide_lds_bytes.restype = C.c_int
    L.st_qstep_wide_launch_w8.argtypes = [C.POINTER(QStepParams), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.st_qstep_wide_launch_w8.restype = C.c_int
    L.st_qstep_ws_launch.argtypes = [C.POINTER(QStepParams), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.st_qstep_ws_launch.restype = C.c_int
    L.st_qstep_ws_lds_bytes.argtypes = [C.c_int, C.c_int, C.c_int]
    L.st_qstep_ws_lds_bytes.restype = C.c_int
    L.st_qtarget_launch.argtypes = [C.POINTER(QTargetParams), C.c_int, C.c_void_p]
    L.st_qtarget_launch.restype = C.c_int
    L.st_qtarget_launch_v.argtypes = [C.POINTER(QTargetParams), C.c_int, C.c_int, C.c_void_p]
    L.st_qtarget_launch_v.restype = C.c_int
    L.st_qtarget_img_bytes.argtypes = []
    L.st_qtarget_img_bytes.restype = C.c_int
    L.st_qtarget_img_map.argtypes = [C.c_void_p] + [C.c_int] * 4 + [C.c_void_p]
    L.st_qtarget_img_map.restype = C.c_int
    L.st_f32b_target_sync.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_void_p, C.c_longlong, C.c_void_p]
    L.st_f32b_target_sync.restype = C.c_int
    L.st_reduce_optim.argtypes = [C.POINTER(OptimParams), C.c_void_p]
    L.st_reduce_optim.restype = C.c_int
    L.st_advance.argtypes = [C.c_void_p, C.c_void_p]
    L.st_advance.restype = C.c_int
    L.st_commit_step.argtypes = [C.c_void_p, C.c_void_p]
    L.st_commit_step.restype = C.c_int
    L.st_to_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.st_to_bf16.restype = C.c_int
    L.st_img_pack.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.st_img_pack.restype = C.c_int
    L.st_qstep_ws_img_bytes.argtypes = []
    L.st_qstep_ws_img_bytes.restype = C.c_int
    L.st_qstep_ws_img_map.argtypes = [C.c_void_p] + [C.c_int] * 5 + [C.c_void_p]
    L.st_qstep_ws_img_map.restype = C.c_int
    L.st_random_walk.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_uint32,
                                 C.c_uint32, C.c_void_p]
    L.st_random_walk.restype = C.c_int
    L.st_replicate4.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.st_replicate4.restype = C.c_int
    L.st_tick16.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                            C.c_void_p]
    L.st_tick16.restype = C.c_int
    L.st_init_normal.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_float, C.c_uint32, C.c_uint32,
                                 C.c_uint32, C.c_void_p]
    L.st_init_normal.restype = C.c_int
    _bind_optional(L)
    _lib = L
    return L


def _bind_optional(L: C.CDLL) -> None:
    """Entry points of the fp32 small-batch path (csrc/mlp_f32.hip)."""
    if hasattr(L, "st_occupy"):   # csrc/diag.hip
        L.st_occupy.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.st_occupy.restype = C.c_int
    if hasattr(L, "st_mlp_fwd_f32"):
        L.st_mlp_fwd_f32.restype = C.c_int
        L.st_td_update_f32.restype = C.c_int


def clear_last_error() -> int:
    """Read and reset the HIP runtime's sticky last error (e.g. the hipErrorStreamCaptureInvalidated
    a failed graph capture leaves behind, which the next launcher's hipGetLastError would report)."""
    return int(C.CDLL("libamdhip64.so").hipGetLastError())


def check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"HIP error {err} in {what}")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


def qstep_supported(inp: int, h1p: int, h2p: int) -> bool:
    if not available():
        return False
    return lib().st_qstep_lds_bytes(inp, h1p, h2p) > 0


def qstep_wide_supported(inp: int, h1p: int, h2p: int) -> bool:
    """64-env-chunk variant (csrc/qstep_wide.hip: layer-1 weights in VGPRs)."""
    if not available():
        return False
    return lib().st_qstep_wide_lds_bytes(inp, h1p, h2p) > 0


def qstep_ws_supported(inp: int, h1p: int, h2p: int) -> bool:
    """Wave-specialised variant (csrc/qstep_ws.hip: data waves run whole 16-env tiles, gradient waves
    consume them through an LDS ring)."""
    if not available():
        return False
    return lib().st_qstep_ws_lds_bytes(inp, h1p, h2p) > 0


def qstep_pipe_supported(inp: int, h1p: int, h2p: int) -> bool:
    """Unit-sliced pipelined variant (csrc/ab/qstep_pipe.hip: weight slices in VGPRs, activations through
    LDS, five tiles' stages between two barriers).  Measured 2.6x slower than ws (profiles/r5_pipe_kernel.md),
    so it lives in the opt-in A/B library: needs SHARETRADE_AB_BUILDS=1."""
    if not available():
        return False
    fn = ab_lib().st_qstep_pipe_lds_bytes
    fn.argtypes = [C.c_int, C.c_int, C.c_int]
    fn.restype = C.c_int
    return fn(inp, h1p, h2p) > 0


def random_walk(out: torch.Tensor, start_price: float, vol: float, drift: float, key0: int, key1: int) -> None:
    E, T = out.shape
    check(lib().st_random_walk(ptr(out), E, T, start_price, vol, drift, key0 & 0xFFFFFFFF, key1 & 0xFFFFFFFF,
                               stream_handle()), "st_random_walk")


def replica_stride(T: int) -> int:
    """Row stride of the shifted price replicas (multiple of 4, >= T + 64: every lane of a wave reads
    one float4 of the window, 256 floats from its start)."""
    return (T + 64 + 3) // 4 * 4


def replicate4(src: torch.Tensor, reps: int = 4) -> torch.Tensor:
    """[E, T] -> [reps, E, T4] shifted replicas (csrc/series.hip: replicate4); reps=1 is a padded copy."""
    E, T = src.shape
    T4 = replica_stride(T)
    flat = torch.zeros(reps * E * T4 + 64, dtype=torch.float32, device=src.device)   # +64: last row's over-read
    out = flat[: reps * E * T4].view(reps, E, T4)
    check(lib().st_replicate4(ptr(src), ptr(out), E, T, T4, int(reps), stream_handle()), "st_replicate4")
    return out


def tick16_stride(T: int) -> int:
    """Row stride (u16 elements) of the tick bank: >= T + 8 (the window loads reach 2 ticks past the series'
    end), a multiple of 8 (16-byte rows)."""
    return (T + 8 + 7) // 8 * 8


def tick16(bank: torch.Tensor, quantize: bool):
    """The 16-bit tick copy of an [E, T] fp32 bank (csrc/series.hip tick16): ``(ticks [E, T16] int16 holding
    u16, scale [E] fp32)``, or ``None`` when ``quantize`` is off and some value is not on its row's tick grid.
    ``quantize=True`` first moves every value onto the grid IN PLACE (synthetic banks)."""
    E, T = bank.shape
    if not bank.is_contiguous():
        raise ValueError("tick16: contiguous [E, T] bank expected")
    T16 = tick16_stride(T)
    flat = torch.zeros(E * T16 + 64, dtype=torch.int16, device=bank.device)   # +64: the last row's loads
    ticks = flat[: E * T16].view(E, T16)
    scale = torch.empty(E, dtype=torch.float32, device=bank.device)
    bad = torch.zeros(1, dtype=torch.int32, device=bank.device)
    check(lib().st_tick16(ptr(bank), E, T, ptr(ticks), T16, ptr(scale), 0 if quantize else 1, ptr(bad),
                          stream_handle()), "st_tick16")
    if not quantize and int(bad.item()) != 0:
        return None
    return ticks, scale


def tick16_quantize_(bank: torch.Tensor) -> torch.Tensor:
    """Move every value of an [E, T] fp32 device bank onto its row's 16-bit tick grid, in place (csrc/series.hip
    tick16 mode 0; host mirror: data.prices.tick16_quantize)."""
    E, T = bank.shape
    if not bank.is_contiguous():
        raise ValueError("tick16: contiguous [E, T] bank expected")
    check(lib().st_tick16(ptr(bank), E, T, None, 0, None, 0, None, stream_handle()), "st_tick16")
    return bank


def init_normal(block: torch.Tensor, rows: int, cols: int, std: float, key0: int, key1: int, stream: int) -> None:
    """``block[:rows, :cols] = std * N(0, 1)`` on the device (csrc/series.hip init_normal_kernel);
    ``block`` is a row-major [R, ld] fp32 view (e.g. one weight of the flat parameter buffer)."""
    if not block.is_cuda or block.dtype != torch.float32 or block.dim() != 2 or block.stride(1) != 1:
        raise ValueError("init_normal: a 2-D row-major fp32 CUDA view is required")
    if rows > block.shape[0] or cols > block.shape[1]:
        raise ValueError("init_normal: block too small")
    check(lib().st_init_normal(ptr(block), rows, cols, block.stride(0), std, key0 & 0xFFFFFFFF, key1 & 0xFFFFFFFF,
                               stream, stream_handle()), "st_init_normal")


def ws_weight_image(params: torch.Tensor, seg) -> tuple:
    """The ws step kernel's weight images in LDS byte order (``QStepParams::wimg``) and the parameter ->
    image map the optimizer pass keeps it current with (``OptimParams::img`` / ``img_map``)."""
    L = lib()
    img = torch.zeros(L.st_qstep_ws_img_bytes(), dtype=torch.uint8, device=params.device)
    m = torch.full((params.numel(),), -1, dtype=torch.int32, device=params.device)
    check(L.st_qstep_ws_img_map(ptr(m), seg["W0"].offset, seg["W1"].offset, seg["W2"].offset, seg["b1"].offset,
                                seg["b2"].offset, stream_handle()), "st_qstep_ws_img_map")
    img_pack(params, m, img)
    return img, m


def qtarget_weight_image(target: torch.Tensor, seg) -> tuple:
    """The target pass's weight images in LDS byte order (``QTargetParams::wimg``) and its parameter map."""
    L = lib()
    img = torch.zeros(L.st_qtarget_img_bytes(), dtype=torch.uint8, device=target.device)
    m = torch.full((target.numel(),), -1, dtype=torch.int32, device=target.device)
    check(L.st_qtarget_img_map(ptr(m), seg["W0"].offset, seg["W1"].offset, seg["W2"].offset, seg["b1"].offset,
                               stream_handle()), "st_qtarget_img_map")
    img_pack(target, m, img)
    return img, m


def img_pack(params: torch.Tensor, m: torch.Tensor, img: torch.Tensor) -> None:
    check(lib().st_img_pack(ptr(params), ptr(m), ptr(img), params.numel(), stream_handle()), "st_img_pack")


def to_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    check(lib().st_to_bf16(ptr(src), ptr(dst), src.numel(), stream_handle()), "st_to_bf16")
