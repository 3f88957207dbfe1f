"""VectorEngine — the data plane: E vectorised trading envs + the Q-learner on one GPU.

This replaces the reference's hot path — 10 ``TrainerChildActor`` rollout
workers each doing two blocking asks per step (``SelectionAction``,
``UpdateQ``) against ONE ``QDecisionPolicyActor`` mailbox
(`TrainerChildActor.scala:82-103`, `QDecisionPolicyActor.scala:54-77`) — with
two kernel launches per step for every env on the GPU:

1. ``qstep_fused`` (csrc/qstep_fused.hip): select + env step + TD target +
   backward for all envs, per-workgroup gradient slabs;
2. ``reduce_optim`` (csrc/optim.hip): slab reduction + optimizer + bf16 refresh.

With ``world_size > 1`` (one process per GPU, RCCL over xGMI) the reduction
is split: reduce -> ``all_reduce(SUM)`` of ONE flat fp32 gradient bucket ->
update; the loss is pre-scaled by ``1/(E*world)`` so SUM is the global mean.
This is the synchronous-DP analogue of the reference's Hogwild-style shared
learner.

``backend="torch"`` runs the same step through the plain-PyTorch oracle
(`sharetrade.env.trading.engine_step_ref`) — used on CPU (tests, gloo DP
rehearsal) and as the numerics reference; it is never chosen silently on a GPU.
"""
from __future__ import annotations

import contextlib

import math
import os
import time
from typing import Dict, Optional

import numpy as np
import torch

from ..config import Config
from ..env import trading as tr
from ..models import qnet as qn
from ..ops import native
from ..utils import rng

NSTAT = 8
STAT_NAMES = ("reward_sum", "loss_sum", "explore", "episodes_done", "final_sum", "final_sq", "qslot_sum", "_")
OPT_KIND = {"sgd": 0, "adagrad": 1, "adam": 2}


# HIP-graph capture mode: "thread_local" -- with an RCCL process group alive, its watchdog thread
# polls collective events during our captures; in the default global mode that poll invalidates the
# capture (hipErrorStreamCaptureInvalidated) and kills the watchdog.  Our own thread stays checked.
_CAPTURE_MODE = "thread_local"


def resolve_device(spec: str) -> torch.device:
    if spec == "auto":
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(spec)


BANK_TAIL = 64  # floats of zero padding after the bank: the fused kernel reads aligned 16-B slices


def padded_bank(E: int, T: int, device: torch.device) -> torch.Tensor:
    """Uninitialised [E, T] fp32 view on an allocation with BANK_TAIL zero floats behind it."""
    flat = torch.empty(E * T + BANK_TAIL, dtype=torch.float32, device=device)
    flat[E * T:].zero_()
    return flat[:E * T].view(E, T)


def make_price_bank(cfg: Config, E: int, device: torch.device, seed: int = 0) -> torch.Tensor:
    """[E, T] fp32 price bank resident on ``device`` (tail-padded, see BANK_TAIL).  Synthetic sources are put on
    a 16-bit tick grid per series when ``data.tick16`` (the flagship kernel's u16 window path)."""
    bank = _make_price_bank(cfg, E, device, seed)
    if cfg.data.tick16 and cfg.data.source in ("random_walk", "ar1", "trend"):
        if bank.device.type == "cuda":
            native.tick16_quantize_(bank)
        else:
            from ..data.prices import tick16_quantize

            bank.copy_(torch.from_numpy(tick16_quantize(bank.numpy())))
    return bank


def _make_price_bank(cfg: Config, E: int, device: torch.device, seed: int = 0) -> torch.Tensor:
    d = cfg.data
    if d.source == "random_walk":
        if device.type == "cuda":
            out = padded_bank(E, d.length, device)
            k0, k1 = rng.key_for(d.seed + 7919 * seed)
            native.random_walk(out, d.start_price, d.volatility, 0.0, int(k0), int(k1))
            return out
        arr = tr_random_walk(E, d.length, d.start_price, d.volatility, d.seed + 7919 * seed)
        return torch.from_numpy(arr).to(device)
    if d.source == "ar1":
        # momentum walk, generated on the device: one [E] recurrence step per day
        g = torch.Generator(device=device)
        g.manual_seed(d.seed + 7919 * seed)
        out = padded_bank(E, d.length, device)
        eps = torch.empty(E, device=device)
        r = torch.zeros(E, device=device)
        logp = torch.zeros(E, device=device)
        out[:, 0] = d.start_price
        for t in range(1, d.length):
            eps.normal_(0.0, d.volatility, generator=g)
            r.mul_(d.ar_phi).add_(eps)
            logp.add_(r)
            out[:, t] = d.start_price * torch.exp(logp)
        return out
    if d.source == "trend":
        # persistent zero-mean drift regimes (AR(1) on the drift, not on the returns), on the device
        g = torch.Generator(device=device)
        g.manual_seed(d.seed + 7919 * seed)
        out = padded_bank(E, d.length, device)
        eps = torch.empty(E, device=device)
        mu = torch.empty(E, device=device).normal_(0.0, d.trend_sd, generator=g)   # stationary start
        logp = torch.zeros(E, device=device)
        out[:, 0] = d.start_price
        k = float(d.trend_sd * math.sqrt(max(0.0, 1.0 - d.trend_rho ** 2)))
        for t in range(1, d.length):
            eps.normal_(0.0, 1.0, generator=g)
            mu.mul_(d.trend_rho).add_(eps, alpha=k)
            eps.normal_(0.0, d.volatility, generator=g)
            logp.add_(mu).add_(eps)
            out[:, t] = d.start_price * torch.exp(logp)
        return out
    from ..data import prices as pr

    src = pr.make_source(d)
    q = src.query(d.ticker, pr.to_date(d.start), pr.to_date(d.end))
    _, series = pr.sorted_series(q)
    row = torch.tensor(series, dtype=torch.float32)
    return row[None, :].expand(E, -1).contiguous().to(device)


def tr_random_walk(E: int, T: int, start: float, vol: float, seed: int) -> np.ndarray:
    from ..data.prices import random_walk

    return random_walk(T, start, vol, seed, n_series=E).astype(np.float32)


class _SplitStepGraph:
    """One synchronous-DP step as two captured graphs around an eager host-side all-reduce (gloo)."""

    def __init__(self, pre, post, all_reduce, grad):
        self.pre, self.post, self.all_reduce, self.grad = pre, post, all_reduce, grad

    def replay(self) -> None:
        self.pre.replay()
        self.all_reduce(self.grad)
        self.post.replay()


class VectorEngine:
    """E envs + learner on one device; optionally one rank of a DP group."""

    def __init__(self, cfg: Config, prices: Optional[torch.Tensor] = None, device: Optional[torch.device] = None,
                 rank: int = 0, world_size: int = 1, group=None, envs: Optional[int] = None,
                 backend: Optional[str] = None, params: Optional[torch.Tensor] = None):
        self.cfg = cfg
        self.device = device if device is not None else resolve_device(cfg.engine.device)
        self.rank, self.world_size, self.group = rank, world_size, group
        self.E = int(envs if envs is not None else cfg.engine.envs_per_rank)
        self.layout = qn.QNetLayout.from_config(cfg.model)
        self.H = cfg.model.history
        be = backend or cfg.engine.backend
        if be == "auto":
            be = "native" if self.device.type == "cuda" else "torch"
        self.backend = be
        a = cfg.agent
        self._learn_knobs = bool(a.target_every or a.double_dqn or a.reward_scale != 1.0 or a.ramp_mode != "position")
        if a.ramp_mode not in ("position", "global"):
            raise ValueError(f"agent.ramp_mode: {a.ramp_mode!r}")
        if a.double_dqn and not a.target_every:
            raise ValueError("agent.double_dqn needs agent.target_every > 0")
        self.params_target = None
        L = self.layout
        self.kernel = None
        if be == "native":
            if self.device.type != "cuda":
                raise ValueError("native backend needs a GPU device")
            fused_ok = (cfg.engine.dtype == "bf16" and L.n_layers == 3 and self.E % 32 == 0
                        and self.H + 3 <= L.in_p - 16
                        and native.qstep_supported(L.pdims[0], L.pdims[1], L.pdims[2]))
            if cfg.engine.dtype == "bf16" and not fused_ok:
                raise NotImplementedError(
                    f"no fused bf16 step kernel for padded dims {L.pdims} / E={self.E} (use engine.dtype=fp32)")
            # bf16: the fused MFMA step kernel (csrc/qstep_fused.hip);
            # fp32: the exact-fp32 row kernels (csrc/mlp_f32.hip) — any MLP up to 6 layers x 1024
            self.kernel = "bf16_fused" if fused_ok else "fp32_rows"
        # envs per chunk of the fused kernel: 64 -> csrc/qstep_wide.hip / csrc/qstep_ws.hip, 32 ->
        # csrc/qstep_fused.hip
        self.chunk = 32
        self.step_kernel = "narrow"
        sk = cfg.engine.step_kernel
        if sk not in ("auto", "wide", "narrow", "ws", "pipe"):
            raise ValueError(f"engine.step_kernel: {sk!r}")
        if cfg.engine.step_variant:
            # timing / debug builds of the ws kernel only; refused unless SHARETRADE_AB_BUILDS=1
            if sk not in ("auto", "ws", "pipe"):
                raise ValueError("engine.step_variant selects a build of the ws or pipe kernel")
            native.variant_launch(cfg.engine.step_variant,
                                  "st_qstep_pipe_launch_" if sk == "pipe" else "st_qstep_ws_launch_")
        if self.kernel == "bf16_fused" and sk == "pipe":
            if not native.ab_builds_enabled():
                raise RuntimeError("engine.step_kernel='pipe' (csrc/ab/qstep_pipe.hip: 2.6x slower than ws, kept "
                                   "as a measured record) is in the opt-in A/B library: set SHARETRADE_AB_BUILDS=1")
            if not (self.ws_ok(cfg, L) and native.qstep_pipe_supported(L.pdims[0], L.pdims[1], L.pdims[2])):
                raise NotImplementedError(f"engine.step_kernel='pipe' needs E % 64 == 0, history 201 and padded dims "
                                          f"(224, 128, 128); got E={self.E}, H={self.H}, dims {L.pdims}")
            self.chunk, self.step_kernel = 64, "pipe"
        elif self.kernel == "bf16_fused" and (sk == "ws" or (sk == "auto" and int(cfg.engine.chunk) == 0
                                                            and cfg.engine.step_waves == 8 and self.ws_ok(cfg, L))):
            if not self.ws_ok(cfg, L):
                raise NotImplementedError(f"engine.step_kernel='ws' needs E % 64 == 0, history 201, padded dims "
                                          f"(224, 128, 128) and the static chunk schedule; got E={self.E}, "
                                          f"H={self.H}, dims {L.pdims}")
            self.chunk, self.step_kernel = 64, "ws"
        elif self.kernel == "bf16_fused":
            want = int(cfg.engine.chunk)
            wide_ok = self.E % 64 == 0 and native.qstep_wide_supported(L.pdims[0], L.pdims[1], L.pdims[2])
            if want == 64 and not wide_ok:
                raise NotImplementedError(f"engine.chunk=64 needs E % 64 == 0 and padded dims (224, 128, 128); "
                                          f"got E={self.E}, dims {L.pdims}")
            if cfg.engine.step_waves not in (4, 8):
                raise ValueError(f"engine.step_waves must be 4 or 8, got {cfg.engine.step_waves}")
            if want not in (0, 32, 64):
                raise ValueError(f"engine.chunk must be 0 (auto), 32 or 64, got {want}")
            if sk == "wide":
                want = 64
            elif sk == "narrow":
                want = 32
            if want == 64 and not wide_ok:
                raise NotImplementedError(f"the 64-env-chunk kernel needs E % 64 == 0 and padded dims "
                                          f"(224, 128, 128); got E={self.E}, dims {L.pdims}")
            self.chunk = 64 if (want in (0, 64) and wide_ok) else 32
            self.step_kernel = "wide" if self.chunk == 64 else "narrow"
        if self._learn_knobs and self.kernel == "bf16_fused" and self.step_kernel != "ws":
            # bf16: the ws kernel's knob build (csrc/qstep_ws.hip KN) + the target pass (csrc/qtarget.hip)
            raise NotImplementedError("agent.target_every / double_dqn / reward_scale / ramp_mode on the bf16 "
                                      "native step need the ws kernel (engine.step_kernel='ws' or 'auto'; "
                                      f"this config selected {self.step_kernel!r})")
        # ------------------------------------------------------------ data
        if prices is not None:
            bank = padded_bank(prices.shape[0], prices.shape[1], self.device)
            bank.copy_(prices)
            self.prices = bank
        else:
            self.prices = make_price_bank(cfg, self.E, self.device, seed=rank)
        if self.prices.shape[0] != self.E:
            raise ValueError(f"price bank has {self.prices.shape[0]} rows, expected {self.E}")
        self.T = int(self.prices.shape[1])
        if self.T <= self.H + 1:
            # TrainerChildActor.scala:69-70
            raise ValueError("Stock price count should be more than Tensorflow input nodes")
        # ------------------------------------------------------------ params / optimizer
        m, a = cfg.model, cfg.agent
        p0 = params.clone().float() if params is not None else qn.init_params(L, m, seed=a.seed, device=self.device)
        self.params = p0.to(self.device)
        # padding entries of the flat layout are exactly zero (csrc/qstep_wide.hip relies on the layer-1
        # padding columns: the gathered rows carry finite non-zero values there)
        self._real = L.trainable_mask(True).to(self.device)
        self.params.mul_(self._real)
        self.mask = L.trainable_mask(m.train_bias).to(self.device)
        # Polyak average of the parameters (engine.ema_decay > 0): the weights to serve
        self.ema_decay = float(cfg.engine.ema_decay)
        if not 0.0 <= self.ema_decay < 1.0:
            raise ValueError(f"engine.ema_decay must be in [0, 1), got {self.ema_decay}")
        self.params_ema = self.params.clone() if self.ema_decay > 0 else None
        self.opt = qn.OptimState(a.optimizer, L.numel, a.adagrad_init_acc, device=self.device)
        self.state = tr.EnvState.create(self.E, cfg.env.budget, cfg.env.shares, device=self.device)
        self.env_offset = rank * self.E
        self.step_count = 0
        # one key for the whole job: draws are indexed by the GLOBAL env id (env_offset + e), so a
        # DP run draws exactly what a single process holding all envs would
        self.key0, self.key1 = rng.key_for(a.seed, 0)
        total = self.E * world_size
        self.loss_coef = 2.0 / total if a.loss_reduction == "mean" else 2.0
        self.stats = torch.zeros(NSTAT, dtype=torch.float64)
        self._sync = None
        if world_size > 1:
            from ..parallel.dist import DistContext, GradSync

            ctx = DistContext(rank, world_size, 0, "dist", self.device, group)
            self._sync = GradSync(ctx, L.numel, bucket_mb=cfg.engine.bucket_mb,
                                  compress=cfg.engine.grad_compress or None)
        self._graph = None
        self._last_actions: Optional[torch.Tensor] = None
        if be == "native":
            self._init_native()

    def ws_ok(self, cfg: Config, L) -> bool:
        """Geometry of csrc/qstep_ws.hip (wave-specialised step kernel; static or dynamic chunk schedule)."""
        return (self.E % 64 == 0 and self.H == 201 and tuple(L.pdims[:3]) == (224, 128, 128)
                and native.qstep_ws_supported(L.pdims[0], L.pdims[1], L.pdims[2]))

    # ---------------------------------------------------------------- native buffers
    def _init_native(self):
        dev = self.device
        L = self.layout
        self.ctrl = torch.zeros(2, dtype=torch.int64, device=dev)
        # env state + step outputs live in one [rows][E] 4-byte buffer (the fused kernel takes ONE
        # base pointer); the EnvState tensors become row views of it, values carried over
        self.env_soa = torch.zeros(len(native.ENV_ROWS), self.E, dtype=torch.int32, device=dev)
        rows = {}
        for i, k in enumerate(native.ENV_ROWS):
            src = getattr(self.state, k, None)
            dt = torch.float32 if k in ("budget", "value", "ret_sum", "last_final", "rewards_out") else torch.int32
            rows[k] = self.env_soa[i].view(dt)
            if src is not None:
                rows[k].copy_(src)
        for k in self.state.as_dict():
            setattr(self.state, k, rows[k])
        self.actions_out, self.rewards_out = rows["actions_out"], rows["rewards_out"]
        self.grad = torch.zeros(L.numel, dtype=torch.float32, device=dev)
        self.stat_acc = torch.zeros(NSTAT, dtype=torch.float64, device=dev)
        if self.kernel == "fp32_rows":
            from ..ops.mlp_f32 import F32BatchedStep, F32EngineStep

            # many envs: the batched MFMA step (csrc/mlp_f32_mfma.hip); few: the per-env row kernels
            fb = self.cfg.engine.f32_batched
            if fb not in ("auto", "on", "off"):
                raise ValueError(f"engine.f32_batched: {fb!r}")
            self.f32_path = "batched" if (fb == "on" or (fb == "auto" and self.E >= 1024)) else "rows"
            if self._learn_knobs and self.f32_path != "batched":
                raise NotImplementedError("the learning-experiment knobs need the batched fp32 step "
                                          "(engine.f32_batched='on', or 'auto' with >= 1,024 envs)")
            self._f32 = F32BatchedStep(self) if self.f32_path == "batched" else F32EngineStep(self)
            return
        self.params_bf = torch.empty(L.numel, dtype=torch.bfloat16, device=dev)
        # ws + relative features: the windows as 16-bit ticks when every series is exactly on a tick grid (synthetic
        # banks are generated on one, data.tick16): half the bytes of the fp32 windows, bit-identical features
        # (csrc/series.hip tick16, profiles/r6_window_gather_ubench.md)
        self.ticks = self.tscale = None
        b16 = self.cfg.engine.bank16
        if b16 not in ("auto", "off"):
            raise ValueError(f"engine.bank16: {b16!r}")
        if (b16 == "auto" and self.step_kernel == "ws" and self.cfg.env.features == "relative"
                and self.prices.is_contiguous()):
            t16 = native.tick16(self.prices, quantize=False)
            if t16 is not None:
                self.ticks, self.tscale = t16
        # window-gather copies of the fp32 bank: 4 shifted replicas for the 16-B-aligned gathers of the wide
        # kernels; one padded copy for ws (4-B-aligned dwordx4 reads, as fast: profiles/r3_ws_ab.md) -- none when
        # the ws windows come from the tick bank
        self.prices4 = (None if self.ticks is not None else
                        native.replicate4(self.prices, 1 if self.step_kernel in ("ws", "pipe") else 4))
        # ws: the weight images in LDS byte order, kept current by the optimizer pass and copied by DMA in the
        # kernel's prologue (the per-launch gather of them cost ~10 us: profiles/r5_ws_prologue.md)
        self._wimg = self._wimg_map = None
        if self.step_kernel == "ws" and os.environ.get("SHARETRADE_WS_WIMG", "1") != "0":
            self._wimg, self._wimg_map = native.ws_weight_image(self.params, self.layout.segments)
        self._bf16_refresh()
        props = torch.cuda.get_device_properties(dev)
        self.grid = max(1, min(self.cfg.engine.grid or props.multi_processor_count, self.E // self.chunk))
        # per-workgroup gradient partials: bf16 rows for the 64-env-chunk kernel by default (the slab
        # pass of reduce_optim reads half the bytes; each partial is rounded once, summed in fp32)
        self.slab_bf16 = (self.chunk == 64 and self.cfg.engine.slab_dtype == "bf16" and L.numel % 32 == 0
                          and all(seg.offset % 32 == 0 for seg in L.segments.values()))
        # (bf16 slabs are column-blocked [P/32][grid][32])
        self.slab = (torch.zeros((L.numel + 127) // 128 * 128 * self.grid, dtype=torch.bfloat16, device=dev)
                     if self.slab_bf16 else torch.zeros(self.grid, L.numel, dtype=torch.float32, device=dev))
        self.stat_slab = torch.zeros(self.grid, NSTAT, dtype=torch.float32, device=dev)
        sched = self.cfg.engine.chunk_schedule
        if sched == "auto":
            # ws: static even under overlapped DP -- its dynamic build costs +14 % per step on one GPU (a
            # 256-VGPR data wave with 36 B of spills), the static one +0.0 % beside the overlapped
            # all-reduce (tools/bench_flagship_dp.py, profiles/r4_flagship_dp.md)
            sched = ("dynamic" if (self.world_size > 1 and self.cfg.engine.dp_overlap and self.step_kernel != "ws")
                     else "static")
        if sched not in ("static", "dynamic"):
            raise ValueError(f"engine.chunk_schedule: {sched!r}")
        if sched == "dynamic" and self.step_kernel == "ws" and self._learn_knobs:
            # the ws knob build (target net, double DQN, reward scale, global ramp) has the static schedule only
            # (csrc/qstep_ws.hip returns InvalidValue for it): refuse here, not at the first launch
            raise ValueError("engine.chunk_schedule='dynamic' is not available with the learning knobs "
                             "(agent.target_every / double_dqn / reward_scale / ramp_mode) on the ws kernel; "
                             "use 'static' or 'auto'")
        # dynamic: 8 per-XCD claim heads, one per 128-byte line (csrc/qstep_wide.hip, csrc/qstep_ws.hip);
        # needs grid % 8 == 0 (the wide kernel also (E / 64) % 8 == 0), else the static schedule is used
        dyn_ok = ((self.step_kernel == "wide" and self.grid % 8 == 0 and (self.E // 64) % 8 == 0)
                  or (self.step_kernel == "ws" and self.grid % 8 == 0))
        self.chunk_schedule = "dynamic" if (sched == "dynamic" and dyn_ok) else "static"
        self.chunk_heads = (torch.zeros(8 * 32, dtype=torch.int32, device=dev)
                            if self.chunk_schedule == "dynamic" else None)
        # target network (agent.target_every): an fp32 copy of the parameters refreshed every target_every
        # optimizer steps, and QT[e][a][0..3] = its Q values of the three candidate next states, written by
        # csrc/qtarget.hip before each step kernel
        self.qt_buf = None
        if self.cfg.agent.target_every:
            self.params_target = self.params.detach().clone()
            self.qt_buf = torch.zeros(self.E * 12, dtype=torch.float32, device=dev)
        self._build_structs()

    def _build_structs(self):
        cfg, L, st = self.cfg, self.layout, self.state
        seg = L.segments
        q = native.QStepParams()
        if self.prices4 is not None:
            q.prices4, q.T4 = native.ptr(self.prices4), int(self.prices4.shape[2])
        else:
            q.prices4, q.T4 = None, native.replica_stride(self.T)
        if self.ticks is not None:
            q.ticks, q.tscale, q.T16 = native.ptr(self.ticks), native.ptr(self.tscale), int(self.ticks.shape[1])
        q.prices, q.env = native.ptr(self.prices), native.ptr(self.env_soa)
        q.wq, q.wf = native.ptr(self.params_bf), native.ptr(self.params)
        q.wimg = native.ptr(self._wimg) if self._wimg is not None else None
        q.slab, q.stats = native.ptr(self.slab), native.ptr(self.stat_slab)
        q.slab_bf16, q.slab_rows = int(self.slab_bf16), self.grid
        q.ctrl = native.ptr(self.ctrl)
        q.T, q.E, q.H, q.P = self.T, self.E, self.H, L.numel
        q.off_w0, q.off_w1, q.off_b1 = seg["W0"].offset, seg["W1"].offset, seg["b1"].offset
        q.off_w2, q.off_b2 = seg["W2"].offset, seg["b2"].offset
        q.eps = cfg.agent.epsilon
        q.inv_ramp = float(np.float32(1.0 / cfg.agent.ramp))
        q.gamma = cfg.agent.gamma
        q.loss_coef = self.loss_coef
        q.b0 = cfg.env.budget
        q.inv_b0 = float(np.float32(1.0 / cfg.env.budget))
        q.s0 = cfg.env.shares
        q.compat_env = int(cfg.env.compat_decisions)
        q.target_compat = int(cfg.agent.target_slot == "compat")
        q.output_relu = int(cfg.model.output_relu)
        q.feat_mode = tr.FEATURES[cfg.env.features]
        q.key0, q.key1 = int(self.key0), int(self.key1)
        q.env_offset = self.env_offset
        q.chunk_heads = native.ptr(self.chunk_heads) if self.chunk_heads is not None else None
        q.reward_mode = {"absolute": 0, "relative": 1, "growth": 2}[cfg.agent.reward_mode]
        q.td_clip = float(cfg.agent.td_clip)
        self.kernel_err = torch.zeros(4, dtype=torch.int32, device=self.device)
        q.err = native.ptr(self.kernel_err)
        a = cfg.agent
        q.reward_scale = float(a.reward_scale)
        q.ramp_global = int(a.ramp_mode == "global")
        q.double_dqn = int(a.double_dqn)
        q.qt = native.ptr(self.qt_buf) if self.qt_buf is not None else None
        self._qp = q
        self._qtp = None
        if self.qt_buf is not None:
            t = native.QTargetParams()
            t.prices4, t.env, t.wt, t.qt = q.prices4, q.env, native.ptr(self.params_target), q.qt
            t.T, t.E, t.T4 = q.T, q.E, q.T4
            t.ticks, t.tscale, t.T16 = q.ticks, q.tscale, q.T16
            t.off_w0, t.off_w1, t.off_b1, t.off_w2, t.off_b2 = q.off_w0, q.off_w1, q.off_b1, q.off_w2, q.off_b2
            t.b0, t.inv_b0, t.s0 = q.b0, q.inv_b0, q.s0
            t.compat_env, t.output_relu, t.feat_mode = q.compat_env, q.output_relu, q.feat_mode
            # the target net's weight images in LDS byte order, refreshed with every target copy (the pass
            # DMA-copies them instead of gathering and converting per launch)
            if os.environ.get("SHARETRADE_WS_WIMG", "1") != "0":
                self._qt_img, self._qt_map = native.qtarget_weight_image(self.params_target, seg)
                t.wimg = native.ptr(self._qt_img)
            self._qtp = t
            # one workgroup per CU (the weight images take 87.5 KB of LDS), grid-stride over 16-env tiles
            # variant 3 (one 16-env tile per wave, 16 waves): 383 vs 393 us for variant 1 on the tick windows, 442
            # vs 447 on fp32 windows (tools/bench_qtarget.py, profiles/r6_window_u16.md)
            self._qt_variant = int(os.environ.get("SHARETRADE_QT_VARIANT", "3"))
            tpw, nw = native.QTARGET_VARIANTS[self._qt_variant]
            if self.E % (16 * tpw):
                raise NotImplementedError(f"target pass: E % {16 * tpw} != 0")
            self._qt_grid = max(1, min(torch.cuda.get_device_properties(self.device).multi_processor_count,
                                       self.E // (16 * tpw * nw)))
        a = cfg.agent
        o = native.OptimParams()
        o.params, o.params_bf, o.mask = native.ptr(self.params), native.ptr(self.params_bf), native.ptr(self.mask)
        if self._wimg is not None:
            o.img, o.img_map = native.ptr(self._wimg), native.ptr(self._wimg_map)
        o.s1 = native.ptr(self.opt.s1) if self.opt.s1.numel() else None
        o.s2 = native.ptr(self.opt.s2) if self.opt.s2.numel() else None
        o.slab, o.grad, o.ctrl = native.ptr(self.slab), native.ptr(self.grad), native.ptr(self.ctrl)
        o.slab_bf16 = int(self.slab_bf16)
        o.G, o.P, o.kind = self.grid, L.numel, OPT_KIND[a.optimizer]
        o.stats, o.stat_acc, o.nstat = native.ptr(self.stat_slab), native.ptr(self.stat_acc), NSTAT
        o.lr, o.beta1, o.beta2, o.eps, o.scale = a.lr, a.adam_betas[0], a.adam_betas[1], a.adam_eps, 1.0
        o.chunk_heads = q.chunk_heads   # re-zeroed by every slab pass (modes 0 / 1)
        if self.params_ema is not None:   # the optimizer pass also advances the Polyak average
            o.ema, o.ema_decay = native.ptr(self.params_ema), self.ema_decay
        self._op = o

    # ---------------------------------------------------------------- stepping
    def _native_step(self):
        if self.kernel == "fp32_rows":
            ar = None
            if self.world_size > 1:
                ar = self._sync.all_reduce
            self._f32.step(self.grad, ar)
            self._f32_stats()
            self._ema_update()
            return
        L = native.lib()
        sh = native.stream_handle()
        if self.world_size > 1 and self.cfg.engine.dp_overlap:
            self._launch_qstep(L, sh)
            self._overlap_step(L, sh)
            self._target_sync(L, sh)
        elif self.world_size > 1:
            self._dp_pre()
            self._sync.all_reduce(self.grad)
            self._dp_post()
        else:
            self._launch_qstep(L, sh)
            self._op.mode = 0
            native.check(L.st_reduce_optim(self._op, sh), "reduce_optim")
            self._target_sync(L, sh)

    def _dp_pre(self) -> None:
        """Synchronous DP, the part before the gradient all-reduce: step kernel + slab reduction."""
        L, sh = native.lib(), native.stream_handle()
        self._launch_qstep(L, sh)
        self._op.mode = 1
        native.check(L.st_reduce_optim(self._op, sh), "reduce")

    def _dp_post(self) -> None:
        """Synchronous DP, the part after the all-reduce: optimizer on the reduced gradient (+ target copy)."""
        L, sh = native.lib(), native.stream_handle()
        self._op.mode = 2
        native.check(L.st_reduce_optim(self._op, sh), "update")
        self._target_sync(L, sh)

    def _target_sync(self, L, sh) -> None:
        if self._qtp is not None:
            # after the counter advanced: copy when ctrl[0] % target_every == 0 (the torch engine's
            # (step + 1) % target_every); under overlapped DP the copy follows the delayed update
            native.check(L.st_f32b_target_sync(native.ptr(self.params), native.ptr(self.params_target),
                                               self.params.numel(), native.ptr(self.ctrl),
                                               int(self.cfg.agent.target_every), sh), "target_sync")

    def _target_img_refresh(self) -> None:
        """The target pass's weight images from the current target net (every step, right before the pass:
        the target may also be written directly, as the fp32 copy the pass used to gather from)."""
        if getattr(self, "_qt_img", None) is not None:
            native.img_pack(self.params_target, self._qt_map, self._qt_img)

    def _launch_qstep(self, L, sh) -> None:
        if self._qtp is not None:
            self._target_img_refresh()
            native.check(L.st_qtarget_launch_v(self._qtp, self._qt_grid, self._qt_variant, sh), "qtarget")
        if self.step_kernel == "pipe":
            # the measured-and-retired unit-sliced kernel (csrc/ab/qstep_pipe.hip, opt-in A/B library) and
            # its timing builds (csrc/ab/qstep_pipe_<v>.hip), same contract
            fn = native.variant_launch(self.cfg.engine.step_variant, "st_qstep_pipe_launch_") \
                if self.cfg.engine.step_variant else native.variant_launch("", "st_qstep_pipe_launch")
        elif self.step_kernel == "ws":
            fn = L.st_qstep_ws_launch
            if self._qp.stamps:   # tools/stamp_qstep.py: the debug stamps build (opt-in A/B library)
                fn = native.variant_launch(self.cfg.engine.step_variant or "stamps")
            elif self.cfg.engine.step_variant:   # timing builds (csrc/ab/qstep_ws_<v>.hip), same contract
                fn = native.variant_launch(self.cfg.engine.step_variant)
        elif self.chunk == 64:
            fn = L.st_qstep_wide_launch_w8 if self.cfg.engine.step_waves == 8 else L.st_qstep_wide_launch
        else:
            fn = L.st_qstep_launch
        d = self.layout.pdims
        native.check(fn(self._qp, d[0], d[1], d[2], self.grid, sh), f"qstep(chunk={self.chunk})")

    def _overlap_step(self, L, sh) -> None:
        """DP step with the all-reduce hidden behind the next fused kernel: reduce this step's slabs
        into one of two gradient buffers, enqueue its all-reduce, then apply the PREVIOUS step's
        reduced gradient (identical on every rank); the first step only commits the step counter."""
        if not hasattr(self, "_ov"):
            import ctypes as C

            bufs = [self.grad, torch.zeros_like(self.grad)]
            ops = []
            for b in bufs:
                o = native.OptimParams()
                C.pointer(o)[0] = self._op
                o.grad = native.ptr(b)
                o.tdelay = 1
                ops.append(o)
            self._ov = {"bufs": bufs, "ops": ops, "parity": 0, "pending": None}
        ov = self._ov
        i = ov["parity"]
        op = ov["ops"][i]
        op.mode = 1
        native.check(L.st_reduce_optim(op, sh), "reduce")
        wait_new = self._sync.start(ov["bufs"][i])
        if ov["pending"] is not None:
            wait_prev, j = ov["pending"]
            wait_prev()
            upd = ov["ops"][j]
            upd.mode = 2
            native.check(L.st_reduce_optim(upd, sh), "update")
        else:
            native.check(L.st_commit_step(native.ptr(self.ctrl), sh), "commit")
        ov["pending"] = (wait_new, i)
        ov["parity"] = i ^ 1

    def flush_pending(self) -> None:
        """Apply a gradient still in flight (overlapped DP) -- before checkpoints and at the end of training."""
        ov = getattr(self, "_ov", None)
        if ov is None or ov["pending"] is None:
            return
        wait_prev, j = ov["pending"]
        wait_prev()
        upd = ov["ops"][j]
        upd.mode, upd.tdelay = 2, 0          # the last step's own update count
        L, sh = native.lib(), native.stream_handle()
        native.check(L.st_reduce_optim(upd, sh), "update")
        upd.tdelay = 1
        ov["pending"] = None
        # the target copy of a boundary step (ctrl[0] % target_every == 0) followed the delayed update; with the
        # last update applied, copy again, so a checkpoint / evaluation taken here sees the target net that
        # synchronous training has at this step.  The counter does not move: continued overlapped
        # training then starts from synchronous state (its next step only commits the counter).
        self._target_sync(L, sh)

    def _f32_stats(self) -> None:
        if getattr(self._f32, "stats_in_kernel", False):   # the batched path's TD kernel accumulates them
            return
        r = self.rewards_out.double()
        self.stat_acc[0] += r.sum()
        self.stat_acc[1] += self._f32.s.loss.double().sum()

    def native_grad(self) -> torch.Tensor:
        """Test hook: run the fused step kernel + slab reduction only (no optimizer
        update); returns the reduced gradient.  Advances the env state."""
        if self.kernel == "fp32_rows":
            self._f32.grad(self.grad)
            self._f32_stats()
            self.step_count += 1
            return self.grad
        L = native.lib()
        sh = native.stream_handle()
        self._launch_qstep(L, sh)
        self._op.mode = 1
        native.check(L.st_reduce_optim(self._op, sh), "reduce")
        self.step_count += 1
        return self.grad

    def _torch_step(self):
        cfg = self.cfg
        ns, grad, info = tr.engine_step_ref(
            self.prices, self.state, self.params, self.layout, history=self.H, feature_mode=cfg.env.features,
            budget0=cfg.env.budget, shares0=cfg.env.shares, compat_env=cfg.env.compat_decisions,
            target_slot=cfg.agent.target_slot, gamma=cfg.agent.gamma, output_relu=cfg.model.output_relu,
            epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, seed=cfg.agent.seed, rank=0,
            step=self.step_count, loss_coef=self.loss_coef, env_offset=self.env_offset,
            emulate_bf16=(cfg.engine.dtype == "bf16"), reward_mode=cfg.agent.reward_mode,
            td_clip=cfg.agent.td_clip, target_params=self._target_params(), double_dqn=cfg.agent.double_dqn,
            reward_scale=cfg.agent.reward_scale,
            ramp_pos=(torch.full_like(self.state.pos, self.step_count) if cfg.agent.ramp_mode == "global" else None))
        if self.world_size > 1:
            self._sync.all_reduce(grad)
        qn.optimizer_step_ref(self.params, grad, self.opt, self.mask, cfg.agent.lr, cfg.agent.adam_betas,
                              cfg.agent.adam_eps)
        if cfg.agent.target_every and (self.step_count + 1) % int(cfg.agent.target_every) == 0:
            self.params_target.copy_(self.params)
        self._ema_update()
        done = ns.episodes > self.state.episodes
        fin = torch.where(done, ns.last_final, torch.zeros_like(ns.last_final)).double()
        self.stats += torch.tensor([
            float(info["reward"].double().sum()), float(info["loss"]), float((~info["exploit"]).sum()),
            float(done.sum()), float(fin.sum()), float((fin * fin).sum()),
            float(info["q"].gather(1, info["slot"][:, None]).double().sum()), 0.0], dtype=torch.float64)
        self.state = ns
        self._last_actions = info["actions"]
        self.grad_last = grad

    def _target_params(self) -> Optional[torch.Tensor]:
        if not self.cfg.agent.target_every:
            return None
        if self.params_target is None:
            self.params_target = self.params.detach().clone()
        return self.params_target

    def _ema_update(self) -> None:
        """ema <- ema + (1 - decay) (w - ema) in fp32, as csrc/optim.hip does it (host-side paths)."""
        if self.params_ema is not None:
            c = float(np.float32(1.0) - np.float32(self.ema_decay))
            self.params_ema.add_((self.params - self.params_ema) * c)

    @property
    def serving_params(self) -> torch.Tensor:
        """The weights to serve: the Polyak average when engine.ema_decay > 0, else the live ones."""
        return self.params_ema if self.params_ema is not None else self.params

    @contextlib.contextmanager
    def policy_overrides(self, epsilon: Optional[float] = None, lr: Optional[float] = None):
        """Temporarily change the behaviour policy / learning rate of the eager step (evaluation
        episodes).  ``epsilon = inf`` is the greedy policy: every kernel's exploit test is
        ``u < min(eps, pos * inv_ramp)``, and with eps = inv_ramp = +inf the threshold is +inf at every
        position (at pos 0, 0 * inf is NaN and min(inf, NaN) = inf).  ``epsilon = 0``: uniform random
        actions.  ``lr = 0``: the optimizer's update is exactly zero (frozen weights; its moment
        estimates still move -- restore them from a snapshot).  Captured graphs hold the original
        parameter structs, so they are set aside while the overrides are active: steps run eagerly."""
        saved_graphs = (self._graph, getattr(self, "_graph_k", None))
        self._graph, self._graph_k = None, None
        a = self.cfg.agent
        undo = []
        inv = None if epsilon is None else (math.inf if math.isinf(epsilon) else float(np.float32(1.0 / a.ramp)))
        if self.backend == "native" and self.kernel == "fp32_rows":
            r, o = self._f32.rows, self._f32.optim
            undo.append((r, "eps", r.eps)); undo.append((r, "inv_ramp", r.inv_ramp)); undo.append((o, "lr", o.lr))
            if epsilon is not None:
                r.eps, r.inv_ramp = float(epsilon), inv
            if lr is not None:
                o.lr = float(lr)
        elif self.backend == "native":
            q, o = self._qp, self._op
            # overlapped DP applies its updates through struct copies of self._op (``_ov['ops']``): a
            # gradient still in flight is a TRAINING gradient -- applied now, at the training lr -- and the
            # copies take the override too, so no evaluation step changes the weights
            self.flush_pending()
            ops = [o] + list(getattr(self, "_ov", {}).get("ops", []))
            undo.append((q, "eps", q.eps)); undo.append((q, "inv_ramp", q.inv_ramp))
            for oo in ops:
                undo.append((oo, "lr", oo.lr))
            if epsilon is not None:
                q.eps, q.inv_ramp = float(epsilon), inv
            if lr is not None:
                for oo in ops:
                    oo.lr = float(lr)
        undo.append((a, "epsilon", a.epsilon)); undo.append((a, "lr", a.lr))
        if epsilon is not None:
            a.epsilon = float(epsilon)
        if lr is not None:
            a.lr = float(lr)
        try:
            yield self
        finally:
            # the last overridden step's gradient (overlapped DP) is applied under the override
            self.flush_pending()
            for obj, k, v in reversed(undo):
                setattr(obj, k, v)
            self._graph, self._graph_k = saved_graphs

    def step(self) -> None:
        if self.backend == "native":
            if self._graph is not None:
                self._graph.replay()
            else:
                self._native_step()
        else:
            self._torch_step()
        self.step_count += 1

    def run(self, n: int) -> None:
        """``n`` steps; with captured graphs, whole multi-step graphs first (one replay per
        ``graph_steps`` steps: fewer graph-launch boundaries on the GPU), then single steps."""
        gk = getattr(self, "_graph_k", None)
        if gk is not None:
            g, k = gk
            for _ in range(n // k):
                g.replay()
                self.step_count += k
            n -= (n // k) * k
        for _ in range(n):
            self.step()

    def capture_graph(self, warmup: int = 2, graph_steps: Optional[int] = None, prime: bool = False,
                      prime_reps: int = 1) -> bool:
        """Capture one native step in a HIP graph, plus a ``graph_steps``-step graph for :meth:`run`
        (``engine.graph_steps``; the step index lives in device memory, so the captured steps replay
        correctly back to back).

        DP (world_size > 1): the synchronous step -- slab reduce, RCCL all-reduce of the flat
        gradient, optimizer -- is captured with its collective (every rank captures the same
        sequence).  On one MI355X that removes the per-step cross-stream event handshakes of the
        eager path: a 1-rank RCCL group measured 69.0 us/step eager, 61.1 us/step replayed, against
        58.8 us without DP (tools/dp_host_overhead.py).  The overlapped-DP path (``dp_overlap``)
        keeps Python-side pending state between steps and is not captured.

        ``prime``: replay each captured graph (real, counted steps; the multi-step graph at least
        ``prime_reps`` times and until its replay time has settled, :meth:`prime_graph`) so that the first timed replay does not pay the one-time graph upload
        to the device (~1.6 ms for the 16-step graph at 1M envs) and the clock has settled after the
        idle of the capture itself (a >= 10 ms idle costs the next ~40 steps up to 35 %,
        profiles/r2_dvfs_probe.md)."""
        if self.backend != "native" or (self.world_size > 1 and self.cfg.engine.dp_overlap):
            return False
        if self.world_size > 1:
            import torch.distributed as dist

            if dist.get_backend(self.group) != "nccl":
                # gloo collectives run on the host and cannot be captured: two graphs around the all-reduce
                return self._capture_split(warmup)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._native_step()
                self.step_count += 1
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
            self._native_step()
        self._graph = g
        k = int(self.cfg.engine.graph_steps if graph_steps is None else graph_steps)
        self._graph_k = None
        if k > 1:
            gk = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gk, capture_error_mode=_CAPTURE_MODE):
                for _ in range(k):
                    self._native_step()
            self._graph_k = (gk, k)
        if prime:
            g.replay()
            self.step_count += 1
            if self._graph_k is not None:
                self.prime_graph(prime_reps)
        return True

    def _capture_split(self, warmup: int) -> bool:
        """Synchronous DP over a host-side collective (gloo rehearsal groups): the step as two HIP graphs --
        step kernel + slab reduction, then optimizer (+ target copy) -- with the eager all-reduce of the flat
        gradient between the replays.  ``step`` replays the pair; no multi-step graph (every step holds a
        collective).  Every rank captures the same two graphs, so the collective sequence is unchanged."""
        if self.kernel != "bf16_fused":
            return False
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._native_step()
                self.step_count += 1
        torch.cuda.current_stream(self.device).wait_stream(s)
        pre, post = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(pre, capture_error_mode=_CAPTURE_MODE):
            self._dp_pre()
        with torch.cuda.graph(post, capture_error_mode=_CAPTURE_MODE):
            self._dp_post()
        self._graph = _SplitStepGraph(pre, post, self._sync.all_reduce, self.grad)
        self._graph_k = None
        return True

    def prime_graph(self, min_reps: int = 1, max_reps: int = 40, tol: float = 0.015) -> int:
        """Replay the multi-step graph at least ``min_reps`` times and until two consecutive replays
        take the same time within ``tol`` (the clock has settled; at most ``max_reps``).  Real,
        counted steps.  Returns the replays done.

        DP (world_size > 1): exactly ``min_reps`` replays on every rank -- each replay holds the
        gradient all-reduce, so a per-rank stopping decision could leave ranks with different
        collective counts (a hang)."""
        if getattr(self, "_graph_k", None) is None:
            return 0
        gk, k = self._graph_k
        if self.world_size > 1:
            for _ in range(max(1, int(min_reps))):
                gk.replay()
                self.step_count += k
            return max(1, int(min_reps))
        prev, n = None, 0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        while n < max_reps:
            ev[0].record()
            gk.replay()
            ev[1].record()
            self.step_count += k
            n += 1
            ev[1].synchronize()
            t = ev[0].elapsed_time(ev[1])
            if n >= min_reps and prev is not None and abs(t - prev) <= tol * prev:
                break
            prev = t
        return n

    # ---------------------------------------------------------------- metrics
    def stats_dict(self) -> Dict[str, float]:
        acc = self.stat_acc.cpu() if self.backend == "native" else self.stats
        out = {k: float(v) for k, v in zip(STAT_NAMES, acc.tolist()) if not k.startswith("_")}
        return out

    def actions(self) -> torch.Tensor:
        return self.actions_out if self.backend == "native" else self._last_actions

    def final_portfolios(self) -> torch.Tensor:
        """Final portfolio of the last completed episode per env (NaN if none)."""
        return self.state.last_final

    def current_portfolios(self) -> torch.Tensor:
        st = self.state
        return st.budget + st.shares.float() * st.value

    def portfolio_summary(self) -> Dict[str, float]:
        """Mean / population std over envs (TrainerRouterActor.scala:148-151)."""
        fin = self.final_portfolios()
        ok = ~torch.isnan(fin)
        vals = fin[ok].double() if bool(ok.any()) else self.current_portfolios().double()
        mean = float(vals.mean())
        std = float(((vals - mean) ** 2).mean().sqrt())
        return {"mean": mean, "std": std, "n": int(vals.numel()),
                "return_mean": mean - self.cfg.env.budget}

    # ---------------------------------------------------------------- state
    def state_dict(self) -> Dict[str, torch.Tensor]:
        self.flush_pending()
        d = {"params": self.params, "opt_s1": self.opt.s1, "opt_s2": self.opt.s2,
             "opt_t": torch.tensor([self._opt_count()], dtype=torch.int64),
             "step": torch.tensor([self.step_count], dtype=torch.int64)}
        for k, v in self.state.as_dict().items():
            d["env_" + k] = v
        if self.params_ema is not None:
            d["params_ema"] = self.params_ema
        if self.params_target is not None:
            d["params_target"] = self.params_target
        return {k: v.detach().cpu().clone() for k, v in d.items()}

    def _opt_count(self) -> int:
        """Optimizer update count (Adam bias correction).  The fused bf16 kernel keeps it on the
        device (``ctrl``: one update per step, flushed above), so it equals ``step_count``; the
        host-side ``opt.t`` is only advanced by the torch / fp32-row backends."""
        if self.backend == "native" and self.kernel == "bf16_fused":
            return self.step_count
        return self.opt.t

    def _bf16_refresh(self) -> None:
        """The bf16 image of the parameters (and the ws weight images) after they changed outside the
        optimizer pass."""
        native.to_bf16(self.params, self.params_bf)
        if getattr(self, "_wimg", None) is not None:
            native.img_pack(self.params, self._wimg_map, self._wimg)

    def set_params(self, params: torch.Tensor) -> None:
        """Overwrite the live parameters (fp32 master copy and, for the bf16 kernels, its bf16 image)."""
        self.params.copy_(params.to(self.device))
        self.params.mul_(self._real)
        if self.backend == "native" and self.kernel == "bf16_fused":
            self._bf16_refresh()

    def load_state_dict(self, d: Dict[str, torch.Tensor]) -> None:
        ov = getattr(self, "_ov", None)
        if ov is not None and ov["pending"] is not None:
            # a gradient in flight belongs to the replaced state: wait for its collective (every rank
            # started it), then drop it instead of applying it to the restored parameters
            ov["pending"][0]()
            ov["pending"] = None
        self.params.copy_(d["params"].to(self.device))
        self.params.mul_(self._real)
        if self.params_ema is not None:
            self.params_ema.copy_(d["params_ema"].to(self.device) if "params_ema" in d else self.params)
        if self.opt.s1.numel():
            self.opt.s1.copy_(d["opt_s1"].to(self.device))
        if self.opt.s2.numel():
            self.opt.s2.copy_(d["opt_s2"].to(self.device))
        if "params_target" in d:
            self._target_params()
            self.params_target.copy_(d["params_target"].to(self.device))
        elif self.params_target is not None:
            # a checkpoint without a target net: bootstrap from the loaded parameters (as the torch
            # backend's lazy first copy does), not from the construction-time weights
            self.params_target.copy_(self.params)
        self.opt.t = int(d["opt_t"][0])
        self.step_count = int(d["step"][0])
        for k in self.state.as_dict():
            getattr(self.state, k).copy_(d["env_" + k].to(self.device))
        if self.backend == "native":
            if self.kernel == "bf16_fused":
                self._bf16_refresh()
            self.ctrl.fill_(self.step_count)

    def sync_params_from(self, src_rank: int = 0) -> None:
        """Broadcast parameters + optimizer state (DP start / elastic re-join)."""
        if self.world_size <= 1:
            return
        import torch.distributed as dist

        # the target net too (agent.target_every): a re-joined rank must bootstrap from rank 0's target
        tgt = (self.params_target,) if self.params_target is not None else ()
        for t in (self.params, self.opt.s1, self.opt.s2) + tgt:
            if t.numel():
                dist.broadcast(t, src_rank, group=self.group)
        if self.backend == "native" and self.kernel == "bf16_fused":
            self._bf16_refresh()

    def synchronize(self, check: bool = True) -> None:
        """Wait for the device; then (``check``) raise if a step kernel reported a protocol error."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
            if check:
                self.check_kernel_err()

    def check_kernel_err(self) -> None:
        """The ws kernel's error word (csrc/qstep_ws.hip ``ws_fail``: a bounded ring wait gave up and the
        workgroup aborted -- that launch's gradients are garbage).  Reads 16 bytes from the device: call
        it where the host already synchronises (logging, checkpoints, end of a run).  The word is copied to
        the host and tested there: a device-side reduction would load torch's reduction kernels on first use
        and idle the GPU for >= 10 ms, which drops its clock for the next ~40 steps (bench.py calls this
        right before its timed window; profiles/r2_dvfs_probe.md, profiles/r4_bench_window.md)."""
        err = getattr(self, "kernel_err", None)
        if err is not None and err.device.type == "cuda":
            v = max(abs(int(x)) for x in err.cpu().tolist())
            if v:
                err.zero_()   # reported once: the next launch starts from a clean word
                raise RuntimeError(f"step kernel reported error word {v:#x} (ws ring protocol wait gave up; "
                                   f"gradients of the failing launch are invalid)")
