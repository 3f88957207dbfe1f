"""Host side of the exact-fp32 kernels (`csrc/mlp_f32.hip`).

* :class:`F32Learner` — the GPU backend of :class:`~sharetrade.policy.learner.QLearner`
  (the ``QDecisionPolicyActor`` path): ``forward`` = 1 launch,
  ``td_update`` = 2 launches (rows kernel + grad/optimizer kernel).
* :class:`F32EngineStep` — the fp32 step of :class:`~sharetrade.trainer.engine.VectorEngine`
  for networks the fused bf16 kernel does not cover (the reference's
  203->200->3 compat net): env step + TD + backward in the rows kernel, then the
  grad/optimizer kernel, then a counter advance — graph-capturable.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np
import torch

from ..models import qnet as qn
from . import native

F_MAXL = 6
OPT_KIND = {"sgd": 0, "adagrad": 1, "adam": 2}


# agent.reward_mode -> the kernels' code (csrc/mlp_f32*.hip, csrc/qstep_*.hip)
REWARD_MODES = {"absolute": 0, "relative": 1, "growth": 2}

class F32Net(C.Structure):
    _fields_ = [
        ("L", C.c_int), ("pd", C.c_int * (F_MAXL + 1)), ("dims", C.c_int * (F_MAXL + 1)),
        ("off_w", C.c_int * F_MAXL), ("off_b", C.c_int * F_MAXL), ("act_off", C.c_int * F_MAXL),
        ("dz_off", C.c_int * F_MAXL), ("act_stride", C.c_int), ("dz_stride", C.c_int),
        ("bias_col", C.c_int), ("input_dim", C.c_int), ("output_relu", C.c_int), ("P", C.c_int),
        ("gemv_legacy", C.c_int),
    ]


class F32Rows(C.Structure):
    _fields_ = [
        ("params", C.c_void_p), ("x", C.c_void_p), ("xn", C.c_void_p), ("reward", C.c_void_p),
        ("action", C.c_void_p), ("q_out", C.c_void_p), ("qn_out", C.c_void_p), ("acts", C.c_void_p),
        ("dz", C.c_void_p), ("loss", C.c_void_p), ("B", C.c_int), ("mode", C.c_int),
        ("gamma", C.c_float), ("coef", C.c_float),
        ("prices", C.c_void_p), ("budget", C.c_void_p), ("shares", C.c_void_p), ("value", C.c_void_p),
        ("pos", C.c_void_p), ("episodes", C.c_void_p), ("last_final", C.c_void_p), ("ret_sum", C.c_void_p),
        ("actions_out", C.c_void_p), ("rewards_out", C.c_void_p), ("ctrl", C.c_void_p),
        ("T", C.c_int), ("H", C.c_int), ("compat_env", C.c_int), ("target_compat", C.c_int),
        ("feat_mode", C.c_int), ("s0", C.c_int), ("env_offset", C.c_int),
        ("eps", C.c_float), ("inv_ramp", C.c_float), ("b0", C.c_float), ("inv_b0", C.c_float),
        ("key0", C.c_uint32), ("key1", C.c_uint32),
        ("reward_mode", C.c_int), ("td_clip", C.c_float),
    ]


class F32Optim(C.Structure):
    _fields_ = [
        ("params", C.c_void_p), ("mask", C.c_void_p), ("s1", C.c_void_p), ("s2", C.c_void_p),
        ("acts", C.c_void_p), ("dz", C.c_void_p), ("ctrl", C.c_void_p), ("grad", C.c_void_p), ("B", C.c_int),
        ("kind", C.c_int), ("t", C.c_int), ("mode", C.c_int), ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
        ("scale", C.c_float),
    ]


def _bind():
    L = native.lib()
    if not getattr(L, "_f32_bound", False):
        L.st_f32_rows.argtypes = [C.POINTER(F32Net), C.POINTER(F32Rows), C.c_void_p]
        L.st_f32_rows.restype = C.c_int
        L.st_f32_grad_optim.argtypes = [C.POINTER(F32Net), C.POINTER(F32Optim), C.c_void_p]
        L.st_f32_grad_optim.restype = C.c_int
        L.st_f32_advance.argtypes = [C.c_void_p, C.c_void_p]
        L.st_f32_advance.restype = C.c_int
        L.st_f32_lds_bytes.argtypes = [C.POINTER(F32Net)]
        L.st_f32_lds_bytes.restype = C.c_int
        L._f32_bound = True
    return L


def make_net(layout: qn.QNetLayout, output_relu: bool) -> F32Net:
    if layout.n_layers > F_MAXL:
        raise NotImplementedError(f"fp32 kernels support up to {F_MAXL} layers")
    if max(layout.pdims) > 1024:
        raise NotImplementedError("fp32 kernels support padded widths up to 1024")
    n = F32Net()
    n.L = layout.n_layers
    for l, d in enumerate(layout.pdims):
        n.pd[l] = d
        n.dims[l] = layout.dims[l]
    ao = dz = 0
    for l in range(layout.n_layers):
        n.off_w[l] = layout.segments[f"W{l}"].offset
        n.off_b[l] = layout.segments[f"b{l}"].offset if l > 0 else -1
        n.act_off[l] = ao
        ao += layout.pdims[l]
        n.dz_off[l] = dz
        dz += layout.pdims[l + 1]
    n.act_stride, n.dz_stride = ao, dz
    n.bias_col, n.input_dim, n.output_relu, n.P = layout.bias_col, layout.input_dim, int(output_relu), layout.numel
    # A/B switch for csrc/mlp_f32.hip gemv_layer: "legacy" = the wave-per-neuron form everywhere
    n.gemv_legacy = int(os.environ.get("SHARETRADE_F32_GEMV", "") == "legacy")
    return n


class _Scratch:
    """Per-batch-size work buffers (activations, dz, q, loss)."""

    def __init__(self, net: F32Net, B: int, device):
        f = dict(dtype=torch.float32, device=device)
        self.B = B
        self.acts = torch.zeros(B, net.act_stride, **f)
        self.dz = torch.zeros(B, net.dz_stride, **f)
        self.q = torch.zeros(B, 16, **f)
        self.qn = torch.zeros(B, 16, **f)
        self.loss = torch.zeros(B, **f)


class _Staging:
    """Pinned host images of one call's inputs -- padded rows of x (and x'), rewards, actions -- and
    their device twins: host-side inputs (the actor path's [1, 203] states) reach the GPU in ONE
    asynchronous copy instead of a copy + three pad kernels per tensor.  The bias column and the
    zero padding are written once.  Two images alternate (``_StagingPair``): an image is rewritten two
    calls later, after its copy's event, so the host runs up to two calls ahead of the GPU."""

    def __init__(self, layout: qn.QNetLayout, B: int, device):
        self.B, self.in_p = B, layout.in_p
        self.n_x = 2 * B * self.in_p
        n = self.n_x + 2 * B
        self.h = torch.zeros(n, dtype=torch.float32, pin_memory=True)
        rows = self.h[:self.n_x].view(2 * B, self.in_p)
        rows[:, layout.bias_col] = 1.0
        self.hn = self.h.numpy()
        self.rows = self.hn[:self.n_x].reshape(2 * B, self.in_p)
        self.rew = self.hn[self.n_x:self.n_x + B]
        self.act = self.hn[self.n_x + B:].view(np.int32)
        self.d = torch.empty(n, dtype=torch.float32, device=device)
        self.ev = None
        self.input_dim = layout.input_dim

    def put(self, x: torch.Tensor, xn=None, r=None, act=None) -> None:
        if self.ev is not None:
            self.ev.synchronize()      # the previous call's copy has read the host image
        B, D = self.B, self.input_dim
        self.rows[:B, :D] = x.numpy()
        if xn is not None:
            self.rows[B:, :D] = xn.numpy()
        if r is not None:
            self.rew[:] = r.numpy()
        if act is not None:
            self.act[:] = act.numpy()
        self.d.copy_(self.h, non_blocking=True)
        if self.ev is None:
            self.ev = torch.cuda.Event()
        self.ev.record()

    def ptr(self, what: str) -> int:
        off = {"x": 0, "xn": self.B * self.in_p, "r": self.n_x, "act": self.n_x + self.B}[what]
        return self.d.data_ptr() + 4 * off


class _StagingPair:
    """Two :class:`_Staging` images used in turn (the device copies stay in stream order)."""

    def __init__(self, layout: qn.QNetLayout, B: int, device):
        self.imgs = (_Staging(layout, B, device), _Staging(layout, B, device))
        self.i = 1

    def next(self) -> _Staging:
        self.i ^= 1
        return self.imgs[self.i]


class F32Learner:
    def __init__(self, learner):
        self.l = learner
        self.layout: qn.QNetLayout = learner.layout
        self.net = make_net(self.layout, learner.cfg.model.output_relu)
        self.L = _bind()
        self._scratch = {}
        self._staging = {}
        self._td_cache = {}
        self._fwd_cache = {}

    def _stage(self, B: int) -> _Staging:
        st = self._staging.get(B)
        if st is None:
            st = self._staging[B] = _StagingPair(self.layout, B, self.l.device)
        return st.next()

    def _s(self, B: int) -> _Scratch:
        s = self._scratch.get(B)
        if s is None:
            s = self._scratch[B] = _Scratch(self.net, B, self.l.device)
        return s

    def sync_from_learner(self) -> None:
        pass  # the learner's tensors are used in place

    def _pad(self, x: torch.Tensor) -> torch.Tensor:
        return qn.pad_input(self.layout, x.to(self.l.device, torch.float32)).contiguous()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B = x.shape[0]
        s = self._s(B)
        r = self._fwd_cache.get(B)
        if r is None:
            r = self._fwd_cache[B] = F32Rows()
            r.q_out, r.B, r.mode = s.q.data_ptr(), B, 0
        if x.device.type == "cpu":
            st = self._stage(B)
            st.put(x.float())
            xptr = st.ptr("x")
        else:
            xp = self._pad(x)
            xptr = xp.data_ptr()
        r.params, r.x = self.l.params.data_ptr(), xptr
        native.check(self.L.st_f32_rows(self.net, r, native.stream_handle()), "st_f32_rows(fwd)")
        return s.q.clone()

    def td_update(self, x, r_, xn, act: Optional[torch.Tensor], coef: float, want_loss: bool = True):
        """One fused TD update; returns the loss as a float, or (``want_loss=False``) the device
        tensor of per-row losses without waiting for the GPU."""
        B = x.shape[0]
        s = self._s(B)
        a = self.l.cfg.agent
        r, o = self._td_structs(B, s, coef)
        if x.device.type == "cpu" and xn.device.type == "cpu" and r_.device.type == "cpu" and \
                (act is None or act.device.type == "cpu"):
            st = self._stage(B)
            st.put(x.float(), xn.float(), r_.float(), act.to(torch.int32) if act is not None else None)
            r.params, r.x, r.xn, r.reward = self.l.params.data_ptr(), st.ptr("x"), st.ptr("xn"), st.ptr("r")
            r.action = st.ptr("act") if act is not None else None
        else:
            xp, xnp = self._pad(x), self._pad(xn)
            rew = r_.to(self.l.device, torch.float32).contiguous()
            acti = act.to(self.l.device, torch.int32).contiguous() if act is not None else None
            r.params, r.x, r.xn, r.reward = self.l.params.data_ptr(), xp.data_ptr(), xnp.data_ptr(), rew.data_ptr()
            r.action = acti.data_ptr() if acti is not None else None
        sh = native.stream_handle()
        native.check(self.L.st_f32_rows(self.net, r, sh), "st_f32_rows(td)")
        opt = self.l.opt
        opt.t += 1
        o.params = self.l.params.data_ptr()
        o.t = opt.t
        native.check(self.L.st_f32_grad_optim(self.net, o, sh), "st_f32_grad_optim")
        return float(s.loss.sum()) if want_loss else s.loss

    def _td_structs(self, B: int, s: "_Scratch", coef: float):
        """The launch structs of a TD update of batch B, built once (the actor path calls this per
        ``UpdateQ``: constructing and filling two ctypes structs per call cost more than the launches).
        Per call only the input pointers, the parameter pointer and the step counter change."""
        key = (B, float(coef))
        c = self._td_cache.get(key)
        a, opt = self.l.cfg.agent, self.l.opt
        if c is None:
            r = F32Rows()
            r.q_out, r.qn_out, r.acts, r.dz, r.loss = (s.q.data_ptr(), s.qn.data_ptr(), s.acts.data_ptr(),
                                                       s.dz.data_ptr(), s.loss.data_ptr())
            r.B, r.mode, r.gamma, r.coef = B, 1, float(a.gamma), float(coef)
            r.td_clip = float(a.td_clip)
            o = F32Optim()
            o.mask = self.l.mask.data_ptr()
            o.s1 = opt.s1.data_ptr() if opt.s1.numel() else None
            o.s2 = opt.s2.data_ptr() if opt.s2.numel() else None
            o.acts, o.dz, o.ctrl, o.B, o.kind = s.acts.data_ptr(), s.dz.data_ptr(), None, B, OPT_KIND[opt.kind]
            o.mode, o.grad = 0, None
            o.lr, o.beta1, o.beta2, o.eps, o.scale = a.lr, a.adam_betas[0], a.adam_betas[1], a.adam_eps, 1.0
            c = self._td_cache[key] = (r, o)
        r, o = c
        if o.mask != self.l.mask.data_ptr() or (opt.s1.numel() and o.s1 != opt.s1.data_ptr()) or \
                (opt.s2.numel() and o.s2 != opt.s2.data_ptr()):
            del self._td_cache[key]            # optimizer state re-allocated (load_state_dict): rebuild
            return self._td_structs(B, s, coef)
        return r, o


class F32EngineStep:
    """fp32 engine step for :class:`VectorEngine` (see module docstring)."""

    def __init__(self, eng):
        self.eng = eng
        cfg = eng.cfg
        self.layout = eng.layout
        self.net = make_net(self.layout, cfg.model.output_relu)
        self.L = _bind()
        E = eng.E
        self.s = _Scratch(self.net, E, eng.device)
        st = eng.state
        r = F32Rows()
        r.params = eng.params.data_ptr()
        r.q_out, r.qn_out, r.acts, r.dz, r.loss = (self.s.q.data_ptr(), None, self.s.acts.data_ptr(),
                                                   self.s.dz.data_ptr(), self.s.loss.data_ptr())
        r.B, r.mode, r.gamma, r.coef = E, 2, float(cfg.agent.gamma), float(eng.loss_coef)
        r.reward_mode = REWARD_MODES[cfg.agent.reward_mode]
        r.td_clip = float(cfg.agent.td_clip)
        r.prices = eng.prices.data_ptr()
        r.budget, r.shares, r.value, r.pos = (st.budget.data_ptr(), st.shares.data_ptr(), st.value.data_ptr(),
                                              st.pos.data_ptr())
        r.episodes, r.last_final, r.ret_sum = st.episodes.data_ptr(), st.last_final.data_ptr(), st.ret_sum.data_ptr()
        r.actions_out, r.rewards_out, r.ctrl = (eng.actions_out.data_ptr(), eng.rewards_out.data_ptr(),
                                                eng.ctrl.data_ptr())
        r.T, r.H = eng.T, eng.H
        r.compat_env = int(cfg.env.compat_decisions)
        r.target_compat = int(cfg.agent.target_slot == "compat")
        from ..env.trading import FEATURES

        r.feat_mode = FEATURES[cfg.env.features]
        r.s0, r.env_offset = int(cfg.env.shares), int(eng.env_offset)
        r.eps = float(cfg.agent.epsilon)
        r.inv_ramp = float(np.float32(1.0 / cfg.agent.ramp))
        r.b0 = float(cfg.env.budget)
        r.inv_b0 = float(np.float32(1.0 / cfg.env.budget))
        r.key0, r.key1 = int(eng.key0), int(eng.key1)
        self.rows = r
        a = cfg.agent
        o = F32Optim()
        opt = eng.opt
        o.params, o.mask = eng.params.data_ptr(), eng.mask.data_ptr()
        o.s1 = opt.s1.data_ptr() if opt.s1.numel() else None
        o.s2 = opt.s2.data_ptr() if opt.s2.numel() else None
        o.acts, o.dz, o.ctrl, o.B, o.kind = self.s.acts.data_ptr(), self.s.dz.data_ptr(), eng.ctrl.data_ptr(), E, \
            OPT_KIND[opt.kind]
        o.lr, o.beta1, o.beta2, o.eps, o.scale = a.lr, a.adam_betas[0], a.adam_betas[1], a.adam_eps, 1.0
        self.optim = o

    def grad_only(self) -> None:
        sh = native.stream_handle()
        native.check(self.L.st_f32_rows(self.net, self.rows, sh), "st_f32_rows(engine)")

    def grad(self, out: torch.Tensor) -> torch.Tensor:
        """Rows kernel + local gradient into ``out`` (no update)."""
        sh = native.stream_handle()
        native.check(self.L.st_f32_rows(self.net, self.rows, sh), "st_f32_rows(engine)")
        self.optim.mode, self.optim.grad = 1, out.data_ptr()
        native.check(self.L.st_f32_grad_optim(self.net, self.optim, sh), "st_f32_grad(engine)")
        return out

    def step(self, grad_buf: Optional[torch.Tensor] = None, allreduce=None) -> None:
        """One engine step.  With ``allreduce`` (DP): local grad -> allreduce(grad_buf) -> update."""
        sh = native.stream_handle()
        if allreduce is None:
            native.check(self.L.st_f32_rows(self.net, self.rows, sh), "st_f32_rows(engine)")
            self.optim.mode, self.optim.grad = 0, None
            native.check(self.L.st_f32_grad_optim(self.net, self.optim, sh), "st_f32_grad_optim")
        else:
            self.grad(grad_buf)
            allreduce(grad_buf)
            self.optim.mode, self.optim.grad = 2, grad_buf.data_ptr()
            native.check(self.L.st_f32_grad_optim(self.net, self.optim, sh), "st_f32_update(engine)")
        native.check(self.L.st_f32_advance(self.eng.ctrl.data_ptr(), sh), "st_f32_advance")


# ---------------------------------------------------------------------------------- batched (MFMA) fp32 step
class GemmF32(C.Structure):
    _fields_ = [
        ("A", C.c_void_p), ("B", C.c_void_p), ("C", C.c_void_p), ("bias", C.c_void_p), ("aux", C.c_void_p),
        ("M", C.c_int), ("N", C.c_int), ("K", C.c_int),
        ("am", C.c_longlong), ("ak", C.c_longlong), ("bk", C.c_longlong), ("bn", C.c_longlong),
        ("ldc", C.c_longlong), ("ldaux", C.c_longlong),
        ("epi", C.c_int), ("relu", C.c_int), ("kchunk", C.c_int),
        ("zstride", C.c_longlong),
    ]


class F32Batch(C.Structure):
    _fields_ = [
        ("E", C.c_int), ("in_p", C.c_int), ("H", C.c_int), ("T", C.c_int), ("bias_col", C.c_int),
        ("feat_mode", C.c_int),
        ("X", C.c_void_p), ("XN", C.c_void_p), ("Q", C.c_void_p), ("QN", C.c_void_p), ("DQ", C.c_void_p),
        ("loss", C.c_void_p),
        ("s_b2", C.c_void_p), ("s_s2", C.c_void_p), ("s_rew", C.c_void_p), ("s_act", C.c_void_p),
        ("prices", C.c_void_p), ("budget", C.c_void_p), ("shares", C.c_void_p), ("value", C.c_void_p),
        ("pos", C.c_void_p), ("episodes", C.c_void_p), ("last_final", C.c_void_p), ("ret_sum", C.c_void_p),
        ("actions_out", C.c_void_p), ("rewards_out", C.c_void_p), ("ctrl", C.c_void_p),
        ("compat_env", C.c_int), ("target_compat", C.c_int), ("output_relu", C.c_int), ("s0", C.c_int),
        ("env_offset", C.c_int), ("reward_mode", C.c_int),
        ("eps", C.c_float), ("inv_ramp", C.c_float), ("b0", C.c_float), ("inv_b0", C.c_float),
        ("gamma", C.c_float), ("coef", C.c_float), ("td_clip", C.c_float),
        ("key0", C.c_uint32), ("key1", C.c_uint32),
        ("stat", C.c_void_p),
        ("QT", C.c_void_p), ("reward_scale", C.c_float), ("double_dqn", C.c_int), ("ramp_global", C.c_int),
    ]


class Fwd2F32(C.Structure):
    _fields_ = [
        ("A", C.c_void_p), ("W1", C.c_void_p), ("b1", C.c_void_p), ("W2", C.c_void_p), ("b2", C.c_void_p),
        ("H", C.c_void_p), ("Q", C.c_void_p),
        ("M", C.c_int), ("K", C.c_int), ("N1", C.c_int), ("nout", C.c_int), ("relu_out", C.c_int),
        ("lda", C.c_longlong),
    ]


F32B_STORE, F32B_MASK, F32B_ATOMIC, F32B_PARTIAL = 0, 1, 2, 3


def _bind_batched():
    L = _bind()
    if not getattr(L, "_f32b_bound", False):
        L.st_f32b_gemm.argtypes = [C.POINTER(GemmF32), C.c_int, C.c_void_p]
        L.st_f32b_gemm.restype = C.c_int
        L.st_f32b_fwd2.argtypes = [C.POINTER(Fwd2F32), C.c_void_p]
        L.st_f32b_fwd2.restype = C.c_int
        L.st_f32b_splitsum.argtypes = [C.c_void_p, C.c_int, C.c_longlong, C.c_void_p, C.c_longlong, C.c_void_p]
        L.st_f32b_splitsum.restype = C.c_int
        L.st_f32b_target_sync.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_void_p, C.c_longlong, C.c_void_p]
        L.st_f32b_target_sync.restype = C.c_int
        for n in ("st_f32b_gather", "st_f32b_env", "st_f32b_td"):
            getattr(L, n).argtypes = [C.POINTER(F32Batch), C.c_void_p]
            getattr(L, n).restype = C.c_int
        L.st_f32b_colsum.argtypes = [C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.st_f32b_colsum.restype = C.c_int
        L.st_f32b_colsum_det.argtypes = [C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p]
        L.st_f32b_colsum_det.restype = C.c_int
        L._f32b_bound = True
    return L


class _Fwd2Op:
    """A fused two-layer forward launch (st_f32b_fwd2) in a batched step's launch list."""

    def __init__(self, args: Fwd2F32):
        self.args = args


class _BatchedScratch:
    def __init__(self, layout: qn.QNetLayout, E: int, device):
        f = dict(dtype=torch.float32, device=device)
        pd = layout.pdims
        self.X = torch.zeros(E, pd[0], **f)
        self.XN = torch.zeros(E, pd[0], **f)
        # activations of x (inputs of layers 1 .. L-1) and of x' (one buffer per layer, reused)
        self.A = [self.X] + [torch.zeros(E, pd[l], **f) for l in range(1, layout.n_layers)]
        self.AN = [self.XN] + [torch.zeros(E, pd[l], **f) for l in range(1, layout.n_layers)]
        self.q = torch.zeros(E, 16, **f)
        self.qn = torch.zeros(E, 16, **f)
        # dL/dz of every layer's output: dz[l] is [E][pd[l + 1]] (dz[L - 1] = dQ)
        self.dz = [torch.zeros(E, pd[l + 1], **f) for l in range(layout.n_layers)]
        self.loss = torch.zeros(E, **f)
        self.b2 = torch.zeros(E, **f)
        self.s2 = torch.zeros(E, dtype=torch.int32, device=device)
        self.rew = torch.zeros(E, **f)
        self.act = torch.zeros(E, dtype=torch.int32, device=device)


def f32_deterministic(cfg, world_size: int) -> bool:
    """engine.f32_deterministic: "on" / "off", or "auto" = on for DP ranks (world_size > 1) and for the
    reference's decision semantics (env.compat_decisions: the reference_compat preset), where replays must be
    bit-exact; SHARETRADE_F32_SPLIT_PARTIAL=0/1 overrides."""
    env = os.environ.get("SHARETRADE_F32_SPLIT_PARTIAL")
    if env in ("0", "1"):
        return env == "1"
    mode = cfg.engine.f32_deterministic
    if mode not in ("auto", "on", "off"):
        raise ValueError(f"engine.f32_deterministic: {mode!r}")
    if mode == "auto":
        return world_size > 1 or bool(cfg.env.compat_decisions)
    return mode == "on"


class F32BatchedStep:
    """Batched fp32 step of :class:`~sharetrade.trainer.engine.VectorEngine` on the matrix cores
    (csrc/mlp_f32_mfma.hip): the reference network's 203->200->3 geometry -- and any fp32 MLP of the
    flat layout -- over many envs.  Same interface as :class:`F32EngineStep` (``step``, ``grad``,
    ``s.loss``, ``rows`` / ``optim`` for ``policy_overrides``); the optimizer is csrc/mlp_f32.hip's
    ``f32_grad_optim`` applied to the reduced gradient (mode 2), so AdaGrad / Adam / SGD are unchanged."""

    def __init__(self, eng, splits: int = 0):
        self.eng = eng
        cfg = eng.cfg
        self.layout = lay = eng.layout
        self.net = make_net(lay, cfg.model.output_relu)
        self.L = _bind_batched()
        E = eng.E
        self.s = _BatchedScratch(lay, E, eng.device)
        self.grad_local = torch.zeros(lay.numel, dtype=torch.float32, device=eng.device)
        # split-K of the weight-gradient products (K = envs): ~1,024 workgroups per product (tiles x splits),
        # at least 256 envs per split.  One split per 256 envs on every product (the first form) put 4,096
        # workgroups and 16.7 M fp32 atomics on the 208 x 208 product: 164 us of a 750 us step at 65,536 envs
        self.splits = splits
        # deterministic mode (engine.f32_deterministic): split-K partial tiles of the weight-gradient products
        # (EPI_PARTIAL) and per-block bias column sums, each added in a fixed order by st_f32b_splitsum -- no
        # fp32 atomics, so the step is bit-reproducible (DP ranks replaying a dead rank's steps agree bit for
        # bit).  Otherwise fp32 atomics into the gradient.  SHARETRADE_F32_SPLIT_PARTIAL=0/1 overrides.
        self.deterministic = f32_deterministic(cfg, eng.world_size)
        need = max(self._splits(lay.pdims[l + 1], lay.pdims[l], E) * lay.pdims[l + 1] * lay.pdims[l]
                   for l in range(lay.n_layers))
        self.partials = torch.empty(need, dtype=torch.float32, device=eng.device) if self.deterministic else None
        # per-block bias column sums: 32 x 256 floats for the float4 form (widths <= 256), else one row of
        # partial sums per 256 envs at the widest biased layer (csrc/mlp_f32_mfma.hip st_f32b_colsum_det)
        cs = max([32 * 256] + [-(-E // 256) * lay.pdims[l + 1] for l in range(lay.n_layers)])
        self.colsum_part = (torch.empty(cs + 64, dtype=torch.float32, device=eng.device)
                            if self.deterministic else None)
        st, s = eng.state, self.s
        r = F32Batch()
        r.E, r.in_p, r.H, r.T, r.bias_col = E, lay.in_p, eng.H, eng.T, lay.bias_col
        from ..env.trading import FEATURES

        r.feat_mode = FEATURES[cfg.env.features]
        r.X, r.XN, r.Q, r.QN, r.DQ = (s.X.data_ptr(), s.XN.data_ptr(), s.q.data_ptr(), s.qn.data_ptr(),
                                      s.dz[-1].data_ptr())
        r.loss = s.loss.data_ptr()
        r.s_b2, r.s_s2, r.s_rew, r.s_act = s.b2.data_ptr(), s.s2.data_ptr(), s.rew.data_ptr(), s.act.data_ptr()
        r.prices = eng.prices.data_ptr()
        r.budget, r.shares, r.value, r.pos = (st.budget.data_ptr(), st.shares.data_ptr(), st.value.data_ptr(),
                                              st.pos.data_ptr())
        r.episodes, r.last_final, r.ret_sum = st.episodes.data_ptr(), st.last_final.data_ptr(), st.ret_sum.data_ptr()
        r.actions_out, r.rewards_out, r.ctrl = (eng.actions_out.data_ptr(), eng.rewards_out.data_ptr(),
                                                eng.ctrl.data_ptr())
        r.compat_env = int(cfg.env.compat_decisions)
        r.target_compat = int(cfg.agent.target_slot == "compat")
        r.output_relu = int(cfg.model.output_relu)
        r.s0, r.env_offset = int(cfg.env.shares), int(eng.env_offset)
        r.reward_mode = REWARD_MODES[cfg.agent.reward_mode]
        r.eps = float(cfg.agent.epsilon)
        r.inv_ramp = float(np.float32(1.0 / cfg.agent.ramp))
        r.b0 = float(cfg.env.budget)
        r.inv_b0 = float(np.float32(1.0 / cfg.env.budget))
        r.gamma, r.coef, r.td_clip = float(cfg.agent.gamma), float(eng.loss_coef), float(cfg.agent.td_clip)
        r.key0, r.key1 = int(eng.key0), int(eng.key1)
        # step statistics (reward sum, TD loss sum) accumulated by the TD kernel into stat_acc[0:2]
        r.stat = eng.stat_acc.data_ptr() if eng.stat_acc.dtype == torch.float64 and eng.stat_acc.is_cuda else None
        self.stats_in_kernel = r.stat is not None
        # learning experiments (agent.target_every / double_dqn / reward_scale / ramp_mode; the torch oracle's
        # engine_step_ref semantics): Q(x') of a target copy refreshed on the device every target_every steps
        a = cfg.agent
        r.reward_scale, r.double_dqn, r.ramp_global = float(a.reward_scale), int(a.double_dqn), int(a.ramp_mode == "global")
        self.target_every = int(a.target_every)
        self._fwd_t = None
        if self.target_every:
            eng.params_target = eng.params.detach().clone()
            s.qt = torch.zeros(E, 16, dtype=torch.float32, device=eng.device)
            r.QT = s.qt.data_ptr()
        else:
            r.QT = None
        self.rows = r          # (policy_overrides edits eps / inv_ramp here)
        a = cfg.agent
        o = F32Optim()
        opt = eng.opt
        o.params, o.mask = eng.params.data_ptr(), eng.mask.data_ptr()
        o.s1 = opt.s1.data_ptr() if opt.s1.numel() else None
        o.s2 = opt.s2.data_ptr() if opt.s2.numel() else None
        o.acts, o.dz, o.ctrl, o.B, o.kind = None, None, eng.ctrl.data_ptr(), E, OPT_KIND[opt.kind]
        o.lr, o.beta1, o.beta2, o.eps, o.scale = a.lr, a.adam_betas[0], a.adam_betas[1], a.adam_eps, 1.0
        o.mode = 2
        self.optim = o
        self._fwd = [self._fwd_structs(s.A, s.q), self._fwd_structs(s.AN, s.qn)]
        if self.target_every:   # target net on x' (its hidden activations reuse AN: the backward reads A only)
            self._fwd_t = self._fwd_structs(s.AN, s.qt, params=eng.params_target)

    def _gemm(self, A, B, Cp, M, N, K, am, ak, bk, bn, ldc, epi, bias=None, relu=False, aux=None, ldaux=0, splits=1):
        g = GemmF32()
        g.A, g.B, g.C, g.bias, g.aux = A, B, Cp, bias, aux
        g.M, g.N, g.K = M, N, K
        g.am, g.ak, g.bk, g.bn, g.ldc, g.ldaux = am, ak, bk, bn, ldc, ldaux
        g.epi, g.relu, g.kchunk = epi, int(relu), 0
        return (g, splits)

    def _fwd2_ok(self) -> bool:
        """The fused two-layer forward (csrc/mlp_f32_mfma.hip f32b_fwd2_kernel): 2 layers, <= 256 hidden,
        <= 3 actions on a 16-wide output, from 8,192 envs (one workgroup per 64 envs: at 1,024 envs its 16
        workgroups ran 14 % slower than the two GEMMs; ``SHARETRADE_F32_FWD2=0``: always two GEMM launches)."""
        lay = self.layout
        return (os.environ.get("SHARETRADE_F32_FWD2", "1") != "0" and self.eng.E >= 8192 and lay.n_layers == 2
                and lay.pdims[1] <= 256
                and lay.pdims[2] == 16 and lay.n_actions <= 3 and lay.pdims[0] % 4 == 0
                and self.net.off_w[0] % 4 == 0)

    def _fwd_structs(self, acts, q, params=None):
        lay, net, E = self.layout, self.net, self.eng.E
        P = self.eng.params if params is None else params
        if self._fwd2_ok():
            f = Fwd2F32()
            f.A, f.W1, f.W2 = acts[0].data_ptr(), P.data_ptr() + 4 * net.off_w[0], P.data_ptr() + 4 * net.off_w[1]
            f.b1 = P.data_ptr() + 4 * net.off_b[0] if net.off_b[0] >= 0 else None
            f.b2 = P.data_ptr() + 4 * net.off_b[1] if net.off_b[1] >= 0 else None
            f.H, f.Q = acts[1].data_ptr(), q.data_ptr()
            f.M, f.K, f.N1, f.nout = E, lay.pdims[0], lay.pdims[1], lay.n_actions
            f.relu_out, f.lda = int(bool(net.output_relu)), lay.pdims[0]
            return [_Fwd2Op(f)]
        out = []
        for l in range(lay.n_layers):
            K, N = lay.pdims[l], lay.pdims[l + 1]
            last = l == lay.n_layers - 1
            dst = q if last else acts[l + 1]
            bias = P.data_ptr() + 4 * net.off_b[l] if net.off_b[l] >= 0 else None
            relu = (not last) or bool(net.output_relu)
            # Z = A_l . W_l^T: A(m = env, k = in) row-major, B(k = in, n = out) = W^T[out][in]
            out.append(self._gemm(acts[l].data_ptr(), P.data_ptr() + 4 * net.off_w[l], dst.data_ptr(), E, N, K,
                                  K, 1, 1, K, N, F32B_STORE, bias=bias, relu=relu))
        return out

    def _splits(self, M: int, N: int, K: int) -> int:
        if self.splits:
            return int(self.splits)
        tiles = -(-M // 64) * -(-N // 64)
        return max(1, min(-(-1024 // tiles), K // 256))

    def _run(self, ops, sh):
        for op in ops:
            if isinstance(op, _Fwd2Op):
                native.check(self.L.st_f32b_fwd2(C.byref(op.args), sh), "st_f32b_fwd2")
            else:
                g, splits = op
                native.check(self.L.st_f32b_gemm(C.byref(g), splits, sh), "st_f32b_gemm")

    def grad(self, out: torch.Tensor) -> torch.Tensor:
        """One env step of every env and the local gradient into ``out`` (no update)."""
        sh = native.stream_handle()
        L, r, s, lay, net = self.L, self.rows, self.s, self.layout, self.net
        E = self.eng.E
        P = self.eng.params
        out.zero_()
        native.check(L.st_f32b_gather(C.byref(r), sh), "st_f32b_gather")
        self._run(self._fwd[0], sh)
        native.check(L.st_f32b_env(C.byref(r), sh), "st_f32b_env")
        self._run(self._fwd[1], sh)
        if self._fwd_t is not None:
            self._run(self._fwd_t, sh)
        native.check(L.st_f32b_td(C.byref(r), sh), "st_f32b_td")
        for l in reversed(range(lay.n_layers)):
            Kin, Nout = lay.pdims[l], lay.pdims[l + 1]
            dz = s.dz[l]
            # dW_l^T[out][in] += sum_e dZ_l[e][out] A_l[e][in]  (K = envs, split over workgroups)
            sp = self._splits(Nout, Kin, E)
            dst = out.data_ptr() + 4 * net.off_w[l]
            if sp > 1 and self.partials is not None:
                # (widths not a multiple of 4 / unaligned offsets: st_f32b_splitsum's one-element-per-thread
                # form, the same fixed order)
                # split-K partials into scratch, then one deterministic sum (the fp32 atomics of every
                # split's tile were the cost of the 224 x 224 product at 65,536 envs)
                zs = Nout * Kin
                g = self._gemm(dz.data_ptr(), s.A[l].data_ptr(), self.partials.data_ptr(), Nout, Kin, E,
                               1, Nout, Kin, 1, Kin, F32B_PARTIAL, splits=sp)
                g[0].zstride = zs
                self._run([g], sh)
                # (the launcher's actual split count: K rounded to whole 32-wide k-tiles per split)
                kchunk = -(-(-(-E // sp)) // 32) * 32
                native.check(L.st_f32b_splitsum(self.partials.data_ptr(), -(-E // kchunk), zs, dst, zs, sh),
                             "st_f32b_splitsum")
            else:
                g = self._gemm(dz.data_ptr(), s.A[l].data_ptr(), dst, Nout, Kin, E,
                               1, Nout, Kin, 1, Kin, F32B_ATOMIC, splits=sp)
                self._run([g], sh)
            if net.off_b[l] >= 0 and self.colsum_part is not None:
                native.check(L.st_f32b_colsum_det(dz.data_ptr(), Nout, E, Nout, out.data_ptr() + 4 * net.off_b[l],
                                                  self.colsum_part.data_ptr(), None, sh), "st_f32b_colsum_det")
            elif net.off_b[l] >= 0:
                native.check(L.st_f32b_colsum(dz.data_ptr(), Nout, E, Nout, out.data_ptr() + 4 * net.off_b[l], sh),
                             "st_f32b_colsum")
            if l > 0:
                # dZ_{l-1} = (dZ_l . W_l) * [A_l > 0]: B(k = out, n = in) = W^T[out][in]
                g = self._gemm(dz.data_ptr(), P.data_ptr() + 4 * net.off_w[l], s.dz[l - 1].data_ptr(), E, Kin, Nout,
                               Nout, 1, Kin, 1, Kin, F32B_MASK, aux=s.A[l].data_ptr(), ldaux=Kin)
                self._run([g], sh)
        return out

    def step(self, grad_buf: Optional[torch.Tensor] = None, allreduce=None) -> None:
        """One engine step: batched step + local gradient -> (DP: all-reduce) -> optimizer -> counter."""
        sh = native.stream_handle()
        g = grad_buf if grad_buf is not None else self.grad_local
        self.grad(g)
        if allreduce is not None:
            allreduce(g)
        self.optim.grad = g.data_ptr()
        native.check(self.L.st_f32_grad_optim(self.net, self.optim, sh), "st_f32_update(batched)")
        native.check(self.L.st_f32_advance(self.eng.ctrl.data_ptr(), sh), "st_f32_advance")
        if self.target_every:
            e = self.eng
            native.check(self.L.st_f32b_target_sync(e.params.data_ptr(), e.params_target.data_ptr(), e.params.numel(),
                                                    e.ctrl.data_ptr(), self.target_every, sh), "st_f32b_target_sync")
