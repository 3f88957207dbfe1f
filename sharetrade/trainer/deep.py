"""DeepDQN — the 4x1024 MLP Q-net with an HBM replay buffer (BASELINE.json config 4).

Not in the reference (its learner is a 203->200->3 net trained online at batch 1,
`QDecisionPolicyActor.scala:38-77`); this is the north-star scale-up of the same
agent/env: E vectorised trading envs act with the current Q-net, every transition
goes into a 1M-entry replay ring resident in HBM, and each learner update samples
a batch of 4096 transitions, rebuilds their states from the price bank, and runs a
DQN update (target network, Adam) — all on MFMA GEMMs (`csrc/gemm_bf16.hip`) with
fused bias/ReLU/ReLU-grad epilogues, plus the gather / env / TD / Adam kernels of
`csrc/deep.hip`.  One rollout step and one learner update are each captured in a
HIP graph.

Every product is in ``C = A . B^T`` form (see gemm_bf16.hip): activations are kept
as ``A`` and ``A^T``, weights as bf16 ``W`` and ``W^T`` (written by the Adam kernel).
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import Config
from ..ops import gemm as gm
from ..ops import native
from ..utils import rng

ACT_PAD = 64  # output layer rows padded to a GEMM tile


# HIP-graph capture mode: "thread_local" -- with an RCCL process group alive, its watchdog thread
# polls collective events during our captures; in the default global mode that poll invalidates the
# capture (hipErrorStreamCaptureInvalidated) and kills the watchdog.  Our own thread stays checked.
_CAPTURE_MODE = "thread_local"


class _Replay(C.Structure):
    _fields_ = [("env", C.c_void_p), ("pos", C.c_void_p), ("budget", C.c_void_p), ("shares", C.c_void_p),
                ("action", C.c_void_p), ("reward", C.c_void_p), ("budget2", C.c_void_p), ("shares2", C.c_void_p),
                ("done", C.c_void_p), ("ctrl", C.c_void_p), ("cap", C.c_int)]


class _Gather(C.Structure):
    _fields_ = [("prices", C.c_void_p), ("T", C.c_int), ("H", C.c_int), ("in_p", C.c_int), ("feat_mode", C.c_int),
                ("inv_b0", C.c_float), ("mode", C.c_int), ("B", C.c_int), ("pos", C.c_void_p),
                ("budget", C.c_void_p), ("shares", C.c_void_p), ("rp", _Replay), ("key0", C.c_uint32),
                ("key1", C.c_uint32), ("step", C.c_void_p), ("X", C.c_void_p), ("Xn", C.c_void_p),
                ("r_out", C.c_void_p), ("a_out", C.c_void_p), ("done_out", C.c_void_p),
                ("zero0", C.c_void_p), ("zero0_n", C.c_int), ("zero1", C.c_void_p), ("zero1_n", C.c_int),
                ("XT", C.c_void_p), ("ldxt", C.c_int)]


class _Env(C.Structure):
    _fields_ = [("prices", C.c_void_p), ("T", C.c_int), ("H", C.c_int), ("E", C.c_int), ("compat_env", C.c_int),
                ("s0", C.c_int), ("n_actions", C.c_int), ("b0", C.c_float), ("eps", C.c_float),
                ("inv_ramp", C.c_float), ("budget", C.c_void_p), ("shares", C.c_void_p), ("value", C.c_void_p),
                ("pos", C.c_void_p), ("episodes", C.c_void_p), ("last_final", C.c_void_p), ("q", C.c_void_p),
                ("ldq", C.c_int), ("key0", C.c_uint32), ("key1", C.c_uint32), ("ctrl", C.c_void_p),
                ("rp", _Replay), ("stats", C.c_void_p)]


class _TD(C.Structure):
    _fields_ = [("q", C.c_void_p), ("qt", C.c_void_p), ("r", C.c_void_p), ("a", C.c_void_p), ("done", C.c_void_p),
                ("dq", C.c_void_p), ("dqT", C.c_void_p), ("loss", C.c_void_p), ("B", C.c_int), ("ldq", C.c_int),
                ("n_actions", C.c_int), ("gamma", C.c_float), ("coef", C.c_float), ("t", C.c_void_p)]


class _Head(C.Structure):
    _fields_ = [("td", _TD), ("A", C.c_void_p), ("W", C.c_void_p), ("G", C.c_void_p), ("GT", C.c_void_p),
                ("dW", C.c_void_p), ("H", C.c_int), ("gpart", C.c_void_p), ("ldgp", C.c_int), ("qp", C.c_void_p),
                ("qpt", C.c_void_p), ("nqp", C.c_int), ("bq", C.c_void_p), ("bqt", C.c_void_p)]


class _QHead(C.Structure):
    _fields_ = [("A", C.c_void_p), ("W", C.c_void_p), ("bias", C.c_void_p), ("Q", C.c_void_p), ("R", C.c_int),
                ("H", C.c_int), ("lda", C.c_int), ("ldw", C.c_int), ("ldq", C.c_int), ("nact", C.c_int)]


class _Adam(C.Structure):
    _fields_ = [("w", C.c_void_p), ("g", C.c_void_p), ("m", C.c_void_p), ("v", C.c_void_p), ("mask", C.c_void_p),
                ("wb", C.c_void_p), ("wbT", C.c_void_p), ("t", C.c_void_p), ("O", C.c_int), ("I", C.c_int),
                ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float)]


ADAM_MAX_SEG = 16


class _AdamSeg(C.Structure):
    _fields_ = [("w", C.c_void_p), ("g", C.c_void_p), ("m", C.c_void_p), ("v", C.c_void_p), ("mask", C.c_void_p),
                ("wb", C.c_void_p), ("wbT", C.c_void_p), ("gT", C.c_void_p), ("O", C.c_int), ("I", C.c_int),
                ("ldg", C.c_int), ("nb", C.c_int), ("bias", C.c_int), ("blocks", C.c_int), ("gP", C.c_void_p),
                ("np", C.c_int), ("ldp", C.c_int)]


class _AdamMulti(C.Structure):
    _fields_ = [("seg", _AdamSeg * ADAM_MAX_SEG), ("nseg", C.c_int), ("t", C.c_void_p), ("total", C.c_int), ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float),
                ("eps", C.c_float), ("grads_only", C.c_int)]


def _bind():
    L = native.lib()
    if not getattr(L, "_deep_bound", False):
        for fn, args in (("st_deep_gather", [C.POINTER(_Gather), C.c_void_p]),
                         ("st_deep_env_step", [C.POINTER(_Env), C.c_void_p]),
                         ("st_deep_td", [C.POINTER(_TD), C.c_void_p]),
                         ("st_deep_head", [C.POINTER(_Head), C.c_void_p]),
                         ("st_qhead", [C.POINTER(_QHead), C.c_void_p]),
                         ("st_row_sum_bf16", [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
                         ("st_transpose_bf16", [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                C.c_void_p]),
                         ("st_adam_tile", [C.POINTER(_Adam), C.c_void_p]),
                         ("st_adam_multi", [C.POINTER(_AdamMulti), C.c_void_p]),
                         ("st_counter_inc", [C.c_void_p, C.c_void_p])):
            f = getattr(L, fn)
            f.argtypes = args
            f.restype = C.c_int
        L._deep_bound = True
    return L


def _p(t: Optional[torch.Tensor]):
    return t.data_ptr() if t is not None else None


class DeepDQN:
    """E envs + replay ring + deep MLP learner on one GPU."""

    def __init__(self, cfg: Config, device: torch.device, envs: int = 16384, batch: int = 4096,
                 replay_capacity: int = 1 << 20, hidden: Optional[List[int]] = None, target_every: int = 1000,
                 prices: Optional[torch.Tensor] = None, seed: Optional[int] = None, dw_gemm: str = "auto",
                 concurrent: bool = True, fused_adam: bool = True, overlap_act: bool = False,
                 batched_fwd: bool = True, dual_bwd: bool = True, act_inline: bool = False,
                 fuse_act: bool = False, world_size: int = 1, grad_sync=None, bank_seed: int = 0,
                 fuse_xt: bool = True, act_after_fwd: bool = True, early_adam: bool = False,
                 act_gemm: str = "lib", fuse_head: bool = True, bias_part: bool = True, head_qfwd: bool = True,
                 act_qhead: bool = True):
        if device.type != "cuda":
            raise ValueError("DeepDQN runs on the GPU (MFMA GEMMs)")
        self.cfg, self.dev = cfg, device
        self.E, self.B, self.cap = int(envs), int(batch), int(replay_capacity)
        # weight-gradient GEMMs (plain bf16 -> fp32 products, no epilogue): csrc/gemm_bf16.hip, split-K for
        # the long-K / few-tile shapes ("auto" and "hip" are the same; there is no library GEMM path)
        if dw_gemm not in ("auto", "hip"):
            raise ValueError(f"dw_gemm: {dw_gemm!r}")
        self.dw_gemm = dw_gemm
        # concurrent: the independent GEMM chains of an update (online / target forward; weight
        # gradients / data backward) on two streams inside the captured graph -- each 4096-row GEMM
        # fills only one 128x128 tile per CU, two chains at once give every CU two.
        # fused_adam: one multi-tensor Adam launch that also reduces the bias gradients and advances
        # the update counter (was 2L Adam + L row-sum + 1 counter launches).
        self.concurrent, self.fused_adam = bool(concurrent), bool(fused_adam)
        # overlap_act: one captured graph per iteration in which the update first samples its batch,
        # then the act step (gather -> 5 GEMMs -> env step -> replay insert) runs on a third stream
        # beside the update's GEMM chains; Adam waits for both (the act step reads the pre-update
        # weights, as in the serial order).  Only difference from the serial order: the update samples
        # the ring as it was BEFORE this iteration's 16k inserts (one act step older).
        self.overlap_act = bool(overlap_act)
        # batched_fwd: the online and target forward of each layer as ONE launch of the batched GEMM
        # (both problems' tiles in one grid) instead of two GEMM chains on two streams
        self.batched_fwd = bool(batched_fwd)
        # dual_bwd: for the hidden layers, each layer's data gradient and the weight gradient of the
        # layer above run as ONE launch of the two-product GEMM (split-K weight gradient), instead of a
        # fork / join of two streams per layer (each join left a ~10-17 us gap in the graph)
        self.dual_bwd = bool(dual_bwd)
        # act_inline (with overlap_act): the act step in the same graph and order, but on the update's
        # stream (no fork / join; the two GEMM chains then run back to back instead of side by side)
        self.act_inline = bool(act_inline)
        # fuse_act (with overlap_act and batched_fwd): the act step's forward layers join the update's
        # grouped forward launches (online x, target x', act states: three products per launch), its
        # env step follows on the same stream -- one stream, no fork / join, every launch fuller
        self.fuse_act = bool(fuse_act)
        # fuse_xt: the replay gather also writes X transposed (the layer-0 weight gradient's operand)
        # instead of a separate transpose launch in the update
        self.fuse_xt = bool(fuse_xt)
        # act_after_fwd (with overlap_act): fork the act step after the update's forward instead of
        # right after the replay sample
        self.act_after_fwd = bool(act_after_fwd)
        if act_gemm not in ("own", "lib", "lib0"):
            raise ValueError(f"act_gemm must be 'own', 'lib' or 'lib0', not {act_gemm!r}")
        if act_gemm != "own" and not hasattr(torch, "_addmm_activation"):   # (a private PyTorch op)
            act_gemm = "own"
        self.act_gemm = act_gemm
        # early_adam (with overlap_act): Adam waits for the act step's forward only, not its env step
        self.early_adam = bool(early_adam)
        # data parallel (one process per GPU, trainer/runs.py): grad_sync(grad_flat) sums the weight and
        # bias gradients (one flat buffer) over the ranks before Adam; the TD coefficient carries
        # 1/world_size.  The bias gradients then come from row-sum launches (all-reduced with the rest)
        # and the fused Adam reads them instead of reducing the layer gradients itself.
        self.world_size = int(world_size)
        self.grad_sync = grad_sync
        # capture_sync: the backend's collectives can be captured (RCCL): the all-reduce stays inside the
        # update graph; with layer_sync (callable issuing an all-reduce of one tensor on the current
        # stream) each layer's dW / db is reduced on a comm stream as soon as the backward has produced
        # it, overlapped with the rest of the backward; Adam waits for the comm stream
        self.capture_sync = False
        self.layer_sync = None
        self._comm = torch.cuda.Stream(device=device)
        self._bias_from_db = self.world_size > 1 or grad_sync is not None
        self.H = cfg.model.history
        self.in_real = self.H + 2
        self.in_p = 256
        if self.in_real > self.in_p:
            raise ValueError("history too long for the 256-wide input tile")
        hid = list(hidden or cfg.model.hidden)
        if any(h % 128 for h in hid):
            raise ValueError("hidden widths must be multiples of 128 (GEMM tiles)")
        if self.E % 128 or self.B % 128:
            raise ValueError("envs and batch must be multiples of 128")
        self.n_act = cfg.model.n_actions
        self.dims = [self.in_real] + hid + [self.n_act]
        self.pdims = [self.in_p] + hid + [ACT_PAD]
        self.L = len(self.pdims) - 1
        self.target_every = int(target_every)
        self.seed = cfg.agent.seed if seed is None else seed
        self.k = _bind()
        f32, b16, i32 = torch.float32, torch.bfloat16, torch.int32
        dev = device
        # ------------------------------------------------------------ parameters (+ Adam, bf16 copies, target)
        g = torch.Generator().manual_seed(int(self.seed))
        self.W, self.b, self.Wm, self.Wv, self.bm, self.bv = [], [], [], [], [], []
        self.Wb, self.WbT, self.Wt, self.bt, self.Wmask, self.bmask, self.dW, self.db = [], [], [], [], [], [], [], []
        for l in range(self.L):
            o, i = self.pdims[l + 1], self.pdims[l]
            ro, ri = self.dims[l + 1], self.dims[l]
            w = torch.zeros(o, i)
            std = math.sqrt(2.0 / ri) if l < self.L - 1 else 0.01
            w[:ro, :ri] = torch.randn(ro, ri, generator=g) * std
            mask = torch.zeros(o, i)
            mask[:ro, :ri] = 1.0
            bm = torch.zeros(1, o)
            bm[0, :ro] = 1.0
            self.W.append(w.to(dev))
            self.b.append(torch.zeros(1, o, device=dev))
            self.Wmask.append(mask.to(dev))
            self.bmask.append(bm.to(dev))
            for lst, shape in ((self.Wm, (o, i)), (self.Wv, (o, i)), (self.bm, (1, o)), (self.bv, (1, o))):
                lst.append(torch.zeros(*shape, device=dev))
            self.Wb.append(self.W[l].to(b16).contiguous())
            self.WbT.append(self.W[l].t().contiguous().to(b16))
            self.Wt.append(self.Wb[l].clone())
            self.bt.append(self.b[l].clone())
        # weight + bias gradients: views of one flat fp32 buffer (dW first: the replay gather zeroes
        # the split-K span; the whole buffer is the data-parallel all-reduce bucket)
        sizes = [self.pdims[l + 1] * self.pdims[l] for l in range(self.L)]
        self.grad_flat = torch.zeros(sum(sizes) + sum(self.pdims[1:]), device=dev)
        self._dW_flat = self.grad_flat[:sum(sizes)]
        off = 0
        for l in range(self.L):
            self.dW.append(self._dW_flat[off:off + sizes[l]].view(self.pdims[l + 1], self.pdims[l]))
            off += sizes[l]
        self._db_flat = self.grad_flat[off:]
        for l in range(self.L):
            self.db.append(self.grad_flat[off:off + self.pdims[l + 1]].view(1, self.pdims[l + 1]))
            off += self.pdims[l + 1]
        self._dw_plan = []   # per layer: ("hip", (tile, splitk))
        for l in range(self.L):
            o, i = self.pdims[l + 1], self.pdims[l]
            # few output tiles, long K: 64x64 tiles split over K (1024x256: 10.6 us vs 16.3 with
            # 128x128 split 8; tools/bench_dw.py, profiles/r2_config4_dual_bwd.md)
            if o % 64 == 0 and i % 64 == 0 and (o // 64) * (i // 64) <= 256:
                wt = (64, 64)
            else:
                wt = (128, 128) if o % 128 == 0 and i % 128 == 0 else gm.pick_tile(o, i)
            self._dw_plan.append(("hip", (wt, gm.pick_splitk(o, self.pdims[l], self.B, wt))))
        # output layer of the batched forward: split K until both problems' tiles reach ~256 workgroups
        self._q_splitk = 1
        if self.batched_fwd:
            qt = gm.pick_tile(self.B, ACT_PAD)
            tiles = 2 * (self.B // qt[0]) * (ACT_PAD // qt[1])      # online + target problems
            ktiles = self.pdims[-2] // 64
            while tiles * self._q_splitk < 256 and ktiles % (2 * self._q_splitk) == 0 and \
                    ktiles // (2 * self._q_splitk) >= 4:
                self._q_splitk *= 2
        # fuse_head: TD + the output layer's backward (G_{L-2}, dW_{L-1}) in one launch (csrc/deep.hip
        # deep_head_kernel); dW_{L-1} is then accumulated atomically into the zeroed span
        self.fuse_head = bool(fuse_head) and self.L >= 2 and self.pdims[-2] % 256 == 0 and self.B % 64 == 0 \
            and 1 <= self.n_act <= 4
        # head_qfwd: the output layer's forward (online on x, target on x') folded into the last hidden layer's
        # batched launch (per-row partial head sums in its epilogue, GemmArgs::qpart) and summed by deep_head_kernel,
        # instead of a split-K output GEMM launch
        self.head_qfwd = bool(head_qfwd) and self.fuse_head and self.batched_fwd
        # act_qhead: the act step's output layer (E x H -> n_actions) on csrc/deep.hip qhead_kernel (16 lanes per
        # row, packed bf16 dot products) instead of the 64-wide padded EPI_F32 GEMM
        self.act_qhead = bool(act_qhead) and self.pdims[-2] <= 1024 and self.pdims[-2] % 8 == 0 and \
            self.E % 16 == 0 and 1 <= self.n_act <= 4
        self._qpart = None
        if self.head_qfwd:   # [online, target][N / WN parts][B][4], WN = the forward tile's per-wave width
            wn = gm.pick_tile(self.B, self.pdims[-2])[1] // 2
            self._qpart = torch.zeros(2, self.pdims[-2] // wn, self.B, 4, device=dev)
        self._dual = [False] * self.L   # layer l's weight gradient in a dual launch with G_{l-1}
        if self.dual_bwd:
            for l in range(1, self.L - 1):
                o, i = self.pdims[l + 1], self.pdims[l]
                if o % 128 == 0 and i % 128 == 0 and self.B % 128 == 0:
                    self._dw_plan[l] = ("hip", ((128, 128), gm.pick_splitk(o, i, self.B, (128, 128))))
                    self._dual[l] = True
        # bias_part: the hidden layers' bias gradients as fp32 column partials of G over 64-row blocks, written by
        # the backward launches themselves (the dual GEMMs' EPI_RELU_GRAD epilogue, deep_head_kernel) and summed by
        # the fused Adam -- instead of Adam re-reading every G^T (8 MB per 1024-wide layer at batch 4096)
        self._bpart = [None] * self.L
        if (bias_part and self.fused_adam and self.fuse_head and self.B % 128 == 0 and
                all(self._dual[l] for l in range(1, self.L - 1))):
            for l in range(self.L - 1):
                self._bpart[l] = torch.zeros(self.B // 64, self.pdims[l + 1], device=dev)
        sk_layers = [l for l, (k, a) in enumerate(self._dw_plan) if k == "hip" and (a[1] > 1 or
                                                                                    (self.fuse_head and l == self.L - 1))]
        self._zero_span = (0, 0)
        if sk_layers:
            lo = sum(sizes[:sk_layers[0]])
            hi = sum(sizes[:sk_layers[-1] + 1])
            self._zero_span = (lo, hi - lo)
        self._bT_scratch = torch.zeros(max(self.pdims), 1, dtype=b16, device=dev)
        self.t_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self._side = torch.cuda.Stream(device=dev) if self.concurrent else None
        self._act_stream = torch.cuda.Stream(device=dev) if self.overlap_act else None
        # ------------------------------------------------------------ data, envs, replay
        from .engine import make_price_bank, padded_bank

        if prices is not None:
            bank = padded_bank(prices.shape[0], prices.shape[1], dev)
            bank.copy_(prices)
            self.prices = bank
        else:
            self.prices = make_price_bank(cfg, self.E, dev, seed=int(bank_seed))
        if self.prices.shape[0] != self.E:
            raise ValueError("price bank rows != envs")
        self.T = int(self.prices.shape[1])
        e = cfg.env
        self.budget = torch.full((self.E,), float(e.budget), device=dev)
        self.shares = torch.full((self.E,), int(e.shares), dtype=i32, device=dev)
        self.value = torch.zeros(self.E, device=dev)
        self.pos = torch.zeros(self.E, dtype=i32, device=dev)
        self.episodes = torch.zeros(self.E, dtype=i32, device=dev)
        self.last_final = torch.full((self.E,), float("nan"), device=dev)
        self.env_ctrl = torch.zeros(2, dtype=torch.int64, device=dev)
        self.rp = {k: torch.zeros(self.cap, dtype=(f32 if k in ("budget", "reward", "budget2") else i32), device=dev)
                   for k in ("env", "pos", "budget", "shares", "action", "reward", "budget2", "shares2", "done")}
        self.rp_ctrl = torch.zeros(2, dtype=torch.int64, device=dev)
        self.stats = torch.zeros(4, device=dev)
        self.loss = torch.zeros(1, device=dev)
        # ------------------------------------------------------------ activations
        M = self.B
        self.X = torch.zeros(M, self.in_p, dtype=b16, device=dev)
        self.XT = torch.zeros(self.in_p, M, dtype=b16, device=dev)
        self.Xn = torch.zeros(M, self.in_p, dtype=b16, device=dev)
        self.Act = [None] + [torch.zeros(M, h, dtype=b16, device=dev) for h in hid]
        self.ActT = [None] + [torch.zeros(h, M, dtype=b16, device=dev) for h in hid]
        self.ActN = [None] + [torch.zeros(M, h, dtype=b16, device=dev) for h in hid]
        self.G = [torch.zeros(M, self.pdims[l + 1], dtype=b16, device=dev) for l in range(self.L)]
        self.GT = [torch.zeros(self.pdims[l + 1], M, dtype=b16, device=dev) for l in range(self.L)]
        self._Qpair = torch.zeros(2, M, ACT_PAD, device=dev)   # online / target Q: one zero range
        self.Q, self.Qt = self._Qpair[0], self._Qpair[1]
        self.r_b = torch.zeros(M, device=dev)
        self.a_b = torch.zeros(M, dtype=i32, device=dev)
        self.d_b = torch.zeros(M, device=dev)
        # acting buffers (M = E)
        self.Xe = torch.zeros(self.E, self.in_p, dtype=b16, device=dev)
        self.Acte = [None] + [torch.zeros(self.E, h, dtype=b16, device=dev) for h in hid]
        self.Qe = torch.zeros(self.E, ACT_PAD, device=dev)
        self.key0, self.key1 = (int(x) for x in rng.key_for(self.seed, 0))
        self.updates = 0
        self.env_steps = 0
        self._g_act = None
        self._g_upd = None
        self._build_structs()

    # ---------------------------------------------------------------- ctypes structs
    def _replay_struct(self) -> _Replay:
        r = _Replay()
        for k in ("env", "pos", "budget", "shares", "action", "reward", "budget2", "shares2", "done"):
            setattr(r, k, self.rp[k].data_ptr())
        r.ctrl, r.cap = self.rp_ctrl.data_ptr(), self.cap
        return r

    def _build_structs(self) -> None:
        cfg = self.cfg
        from ..env.trading import FEATURES

        fm = FEATURES[cfg.env.features]
        ib0 = float(np.float32(1.0 / cfg.env.budget))
        ge = _Gather()
        ge.prices, ge.T, ge.H, ge.in_p, ge.feat_mode, ge.inv_b0 = self.prices.data_ptr(), self.T, self.H, self.in_p, fm, ib0
        ge.mode, ge.B = 0, self.E
        ge.pos, ge.budget, ge.shares = self.pos.data_ptr(), self.budget.data_ptr(), self.shares.data_ptr()
        ge.rp = self._replay_struct()
        ge.key0, ge.key1, ge.step = self.key0, self.key1, self.t_ctr.data_ptr()
        ge.X = self.Xe.data_ptr()
        self._gather_env = ge
        gr = _Gather()
        C.pointer(gr)[0] = ge
        gr.mode, gr.B = 1, self.B
        gr.X, gr.Xn = self.X.data_ptr(), self.Xn.data_ptr()
        gr.r_out, gr.a_out, gr.done_out = self.r_b.data_ptr(), self.a_b.data_ptr(), self.d_b.data_ptr()
        z0, zn = self._zero_span
        gr.zero0 = self._dW_flat.data_ptr() + 4 * z0 if zn else None
        gr.zero0_n = zn
        # the batched output layer accumulates Q / Q_t over K splits: zeroed here as well
        # (not with head_qfwd: the head kernel writes Q / Q_t with plain stores)
        gr.zero1, gr.zero1_n = ((self._Qpair.data_ptr(), self._Qpair.numel()) if self._q_splitk > 1 and not self.head_qfwd
                                else (None, 0))
        gr.XT, gr.ldxt = (self.XT.data_ptr(), self.B) if self.fuse_xt else (None, 0)
        self._gather_rp = gr
        ev = _Env()
        ev.prices, ev.T, ev.H, ev.E = self.prices.data_ptr(), self.T, self.H, self.E
        ev.compat_env, ev.s0, ev.n_actions = int(cfg.env.compat_decisions), int(cfg.env.shares), self.n_act
        ev.b0, ev.eps, ev.inv_ramp = float(cfg.env.budget), float(cfg.agent.epsilon), float(np.float32(1 / cfg.agent.ramp))
        ev.budget, ev.shares, ev.value, ev.pos = (self.budget.data_ptr(), self.shares.data_ptr(), self.value.data_ptr(),
                                                  self.pos.data_ptr())
        ev.episodes, ev.last_final = self.episodes.data_ptr(), self.last_final.data_ptr()
        ev.q, ev.ldq, ev.key0, ev.key1 = self.Qe.data_ptr(), ACT_PAD, self.key0, self.key1
        ev.ctrl, ev.rp, ev.stats = self.env_ctrl.data_ptr(), self._replay_struct(), self.stats.data_ptr()
        self._env = ev
        td = _TD()
        td.q, td.qt, td.r, td.a, td.done = (self.Q.data_ptr(), self.Qt.data_ptr(), self.r_b.data_ptr(),
                                            self.a_b.data_ptr(), self.d_b.data_ptr())
        td.dq, td.dqT, td.loss = self.G[-1].data_ptr(), self.GT[-1].data_ptr(), self.loss.data_ptr()
        td.B, td.ldq, td.n_actions = self.B, ACT_PAD, self.n_act
        td.gamma, td.coef = float(cfg.agent.gamma), 2.0 / (self.B * self.world_size)
        td.t = self.t_ctr.data_ptr()   # the update counter advances in the TD kernel
        self._td = td
        hd = _Head()
        hd.td = td
        hd.A, hd.W = self.Act[self.L - 1].data_ptr(), self.Wb[self.L - 1].data_ptr()
        hd.G, hd.GT = self.G[self.L - 2].data_ptr(), self.GT[self.L - 2].data_ptr()
        hd.dW, hd.H = self.dW[self.L - 1].data_ptr(), self.pdims[self.L - 1]
        if self._bpart[self.L - 2] is not None:
            hd.gpart, hd.ldgp = self._bpart[self.L - 2].data_ptr(), self.pdims[self.L - 1]
        if self.head_qfwd:
            hd.qp, hd.qpt, hd.nqp = self._qpart[0].data_ptr(), self._qpart[1].data_ptr(), self._qpart.shape[1]
            hd.bq, hd.bqt = self.b[self.L - 1].data_ptr(), self.bt[self.L - 1].data_ptr()
        self._head = hd
        a = cfg.agent
        self._adam = []
        for l in range(self.L):
            for (w, g_, m, v, mk, wb, wbT, O, I) in (
                    (self.W[l], self.dW[l], self.Wm[l], self.Wv[l], self.Wmask[l], self.Wb[l], self.WbT[l],
                     self.pdims[l + 1], self.pdims[l]),
                    (self.b[l], self.db[l], self.bm[l], self.bv[l], self.bmask[l], None, None, 1, self.pdims[l + 1])):
                ad = _Adam()
                ad.w, ad.g, ad.m, ad.v, ad.mask = w.data_ptr(), g_.data_ptr(), m.data_ptr(), v.data_ptr(), mk.data_ptr()
                ad.wb = wb.data_ptr() if wb is not None else self._bscratch(l).data_ptr()
                ad.wbT = wbT.data_ptr() if wbT is not None else None
                ad.t, ad.O, ad.I = self.t_ctr.data_ptr(), O, I
                ad.lr, ad.beta1, ad.beta2, ad.eps = float(a.lr), float(a.adam_betas[0]), float(a.adam_betas[1]), \
                    float(a.adam_eps)
                self._adam.append(ad)
        am = _AdamMulti()
        segs = []
        for l in range(self.L):
            O, I = self.pdims[l + 1], self.pdims[l]
            w = _AdamSeg()
            # all-ones masks (hidden layers) are not read: 4 of the ~36 bytes per parameter
            w.w, w.g, w.m, w.v = (self.W[l].data_ptr(), self.dW[l].data_ptr(), self.Wm[l].data_ptr(),
                                  self.Wv[l].data_ptr())
            w.mask = None if bool(self.Wmask[l].bool().all()) else self.Wmask[l].data_ptr()
            w.wb, w.wbT, w.gT = self.Wb[l].data_ptr(), self.WbT[l].data_ptr(), None
            w.O, w.I, w.ldg, w.nb, w.bias = O, I, 0, 0, 0
            w.blocks = ((I + 63) // 64) * ((O + 63) // 64)
            b = self._bias_seg(l, reduce=not self._bias_from_db)
            segs += [w, b]
        # bias segments first: their blocks (4 rows x batch of gradient sums each) are the longest,
        # started first they do not form the tail
        segs = [sg for sg in segs if sg.bias] + [sg for sg in segs if not sg.bias]
        if len(segs) > ADAM_MAX_SEG:
            self.fused_adam = False
        else:
            for k, sg in enumerate(segs):
                am.seg[k] = sg
            am.nseg, am.t = len(segs), self.t_ctr.data_ptr()
            am.total = sum(sg.blocks for sg in segs)
            am.lr, am.beta1, am.beta2, am.eps = (float(a.lr), float(a.adam_betas[0]), float(a.adam_betas[1]),
                                                 float(a.adam_eps))
        self._adam_multi = am
        # data parallel + fused Adam: every layer's bias gradient in ONE launch after the backward (the
        # multi-tensor kernel's reduction, no update), all-reduced, then read by the fused Adam
        self._bias_multi = None
        if self._bias_from_db and self.fused_adam:
            bm = _AdamMulti()
            for l in range(self.L):
                bm.seg[l] = self._bias_seg(l, reduce=True)
            bm.nseg, bm.t, bm.grads_only = self.L, self.t_ctr.data_ptr(), 1
            bm.total = sum(bm.seg[l].blocks for l in range(self.L))
            bm.lr, bm.beta1, bm.beta2, bm.eps = am.lr, am.beta1, am.beta2, am.eps
            self._bias_multi = bm

    def _bias_seg(self, l: int, reduce: bool) -> _AdamSeg:
        """Multi-tensor Adam segment of bias l: ``reduce`` = its gradient is the row sums of GT[l] (reduced
        in the kernel), else it is read from db[l]."""
        O = self.pdims[l + 1]
        b = _AdamSeg()
        b.w, b.g, b.m, b.v = (self.b[l].data_ptr(), self.db[l].data_ptr(), self.bm[l].data_ptr(),
                              self.bv[l].data_ptr())
        b.mask = None if bool(self.bmask[l].bool().all()) else self.bmask[l].data_ptr()
        b.wb, b.wbT, b.gT = self._bscratch(l).data_ptr(), None, self.GT[l].data_ptr() if reduce else None
        b.O, b.I, b.ldg, b.nb, b.bias = 1, O, self.B, self.B, 1
        b.blocks = (O + 3) // 4 if reduce else (O + 31) // 32   # (4 rows of G^T / 32 entries per block)
        if reduce and self._bpart[l] is not None:   # the backward launch's column partials instead of G^T
            b.gT, b.gP, b.np, b.ldp = None, self._bpart[l].data_ptr(), self._bpart[l].shape[0], O
            b.blocks = (O + 31) // 32
        return b

    def _bscratch(self, l: int) -> torch.Tensor:
        """bf16 copy of bias l [1, n], rewritten by every Adam step (the operand of the library act-step
        epilogue, ``act_gemm="lib"``)."""
        if not hasattr(self, "_bias_bf"):
            self._bias_bf = [self.b[k].detach().to(torch.bfloat16).view(1, -1).clone() for k in range(self.L)]
        return self._bias_bf[l]

    def _refresh_bias_bf(self) -> None:
        for l in range(self.L):
            self._bscratch(l).copy_(self.b[l].view(1, -1).to(torch.bfloat16))

    # ---------------------------------------------------------------- forward
    def _forward(self, X, acts, actsT, Wb, bias, Q, lib: int = -1, qhead: bool = False) -> None:
        """acts[l+1] = relu(acts[l] . W_l^T + b_l); Q = acts[L-1] . W_{L-1}^T + b_{L-1} (fp32).  ``lib`` >= 0:
        the hidden layers from that one on through hipBLASLt's fused bias + ReLU epilogue (bf16 bias copies;
        the act step's 16,384 x 1024 -> 1024 layers, where the library's K loop is faster than our ping-pong
        kernel's, profiles/r6_gemm_ablation.md).  The act step passes 1 (``act_gemm="lib"``); 0 (``"lib0"``) also
        takes its 16,384 x 256 -> 1024 first layer, alone a tie with our ping-pong kernel (18.2-18.7 vs 18.6 us) and
        +0.5 % per iteration beside the update chain (profiles/r6_config4_act_lib.md)."""
        a = X
        for l in range(self.L):
            if l < self.L - 1:
                if 0 <= lib <= l:
                    torch._addmm_activation(self._bscratch(l)[0], a, Wb[l].t(), out=acts[l + 1])
                else:
                    gm.gemm_nt(a, Wb[l], acts[l + 1], gm.EPI_BF16, outT=actsT[l + 1] if actsT else None,
                               bias=bias[l], relu=True)
                a = acts[l + 1]
            elif qhead:   # (act_qhead)
                qh = _QHead()
                qh.A, qh.W, qh.bias, qh.Q = a.data_ptr(), Wb[l].data_ptr(), bias[l].data_ptr(), Q.data_ptr()
                qh.R, qh.H, qh.lda, qh.ldw, qh.ldq, qh.nact = a.shape[0], a.shape[1], a.stride(0), Wb[l].stride(0), \
                    Q.stride(0), self.n_act
                native.check(self.k.st_qhead(qh, native.stream_handle()), "qhead")
            else:
                gm.gemm_nt(a, Wb[l], Q, gm.EPI_F32, bias=bias[l])

    def _forward_pair(self, acts, actsT, actsN, actsE=None) -> None:
        """Online forward on x (+ transposed activations for the backward) and target forward on x',
        one grouped launch per layer; with ``actsE`` the act step's forward on the env states (online
        weights, no transposed copy) is a third product of the same launches."""
        for l in range(self.L):
            if l < self.L - 1:
                qh = self.head_qfwd and l == self.L - 2   # the output head folded into this launch's epilogue
                qa = (self.Wb[l + 1][: self.n_act], self._qpart[0]) if qh else None
                qb = (self.Wt[l + 1][: self.n_act], self._qpart[1]) if qh else None
                probs = [(acts[l], self.Wb[l], acts[l + 1], dict(outT=actsT[l + 1], bias=self.b[l], relu=True, qhead=qa)),
                         (actsN[l], self.Wt[l], actsN[l + 1], dict(bias=self.bt[l], relu=True, qhead=qb))]
                if actsE is not None:
                    probs.append((actsE[l], self.Wb[l], actsE[l + 1], dict(bias=self.b[l], relu=True)))
                gm.gemm_nt_batched(probs, gm.EPI_BF16, tile=gm.pick_tile(self.B, self.pdims[l + 1]))
            else:
                sk = self._q_splitk   # few output tiles, long K: split (outputs zeroed by the replay gather)
                probs = [] if self.head_qfwd else [   # (head_qfwd: Q, Qt come from deep_head_kernel)
                    (acts[l], self.Wb[l], self.Q, dict(bias=self.b[l], splitk=sk, prezeroed=True)),
                    (actsN[l], self.Wt[l], self.Qt, dict(bias=self.bt[l], splitk=sk, prezeroed=True))]
                if actsE is not None:
                    probs.append((actsE[l], self.Wb[l], self.Qe, dict(bias=self.b[l])))
                if probs:
                    gm.gemm_nt_batched(probs, gm.EPI_F32, tile=gm.pick_tile(self.B, ACT_PAD))

    def act_step(self, after_forward=None) -> None:
        """One env step of all E envs: gather -> Q forward -> select/transition/replay insert.
        ``after_forward()`` runs between the forward (the last reader of the weights) and the env step."""
        sh = native.stream_handle()
        native.check(self.k.st_deep_gather(self._gather_env, sh), "deep_gather(env)")
        self._forward(self.Xe, self.Acte, None, self.Wb, self.b, self.Qe,
                      lib={"own": -1, "lib": 1, "lib0": 0}[self.act_gemm], qhead=self.act_qhead)
        if after_forward is not None:
            after_forward()
        native.check(self.k.st_deep_env_step(self._env, sh), "deep_env_step")

    def _fork_act(self, main, act):
        """The act step on its own stream; returns an event recorded after its forward (Adam, which
        overwrites the weights, waits for that, not for the env step behind it)."""
        act.wait_stream(main)
        ev = torch.cuda.Event()
        with torch.cuda.stream(act):
            self.act_step(after_forward=lambda: ev.record(act))
        return ev

    def _dw(self, l: int, actsT) -> None:
        """Weight gradient of layer l: dW = G_l^T . A_l (long-K, few-tile product)."""
        _, (tile, sk) = self._dw_plan[l]
        gm.gemm_nt(self.GT[l], actsT[l], self.dW[l], gm.EPI_F32, tile=tile, splitk=sk,
                   prezeroed=sk > 1)   # zeroed by this update's replay gather

    def update_step(self, with_act: bool = False, split: bool = False) -> None:
        """One DQN update: sample B transitions, Q(x) online / Q(x') target, TD, backward, Adam.

        With ``concurrent``: the target-network forward runs beside the online forward, and each
        layer's weight gradient beside the next data-backward GEMM, on a second stream (fork / join
        with stream waits, so the whole update still captures into one HIP graph).  ``split``: stop
        before the gradient all-reduce and Adam (data-parallel capture, see capture())."""
        sh = native.stream_handle()
        k = self.k
        main = torch.cuda.current_stream(self.dev)
        side = self._side
        native.check(k.st_deep_gather(self._gather_rp, sh), "deep_gather(replay)")
        act = self._act_stream if with_act else None
        if with_act:
            if act is None:
                raise RuntimeError("update_step(with_act=True) needs overlap_act=True")
            if self.fuse_act and self.batched_fwd:
                native.check(k.st_deep_gather(self._gather_env, sh), "deep_gather(env)")
                act = None                     # forward grouped with the update's below
            elif self.act_inline:
                self.act_step()                # same order, same stream
                act = None
            elif not self.act_after_fwd:
                act_fwd_done = self._fork_act(main, act)   # the batch is sampled: the act step may insert now
        if not self.fuse_xt:
            native.check(k.st_transpose_bf16(self.X.data_ptr(), self.in_p, self.XT.data_ptr(), self.B, self.B,
                                             self.in_p, sh), "transpose X")
        acts = [self.X] + self.Act[1:]
        actsT = [self.XT] + self.ActT[1:]
        if self.batched_fwd and with_act and self.fuse_act:
            self._forward_pair(acts, actsT, [self.Xn] + self.ActN[1:], [self.Xe] + self.Acte[1:])
            native.check(k.st_deep_env_step(self._env, sh), "deep_env_step")
        elif self.batched_fwd:
            self._forward_pair(acts, actsT, [self.Xn] + self.ActN[1:])
        elif side is not None:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self._forward(self.Xn, [self.Xn] + self.ActN[1:], None, self.Wt, self.bt, self.Qt)
            self._forward(self.X, acts, actsT, self.Wb, self.b, self.Q)
            main.wait_stream(side)
        else:
            self._forward(self.X, acts, actsT, self.Wb, self.b, self.Q)
            self._forward(self.Xn, [self.Xn] + self.ActN[1:], None, self.Wt, self.bt, self.Qt)
        if act is not None and self.act_after_fwd:
            # the act step beside the backward chain (TD, small GEMMs, dual launches) rather than beside
            # the forward's GEMMs, which already fill the chip
            act_fwd_done = self._fork_act(main, act)
        if self.fuse_head:
            native.check(k.st_deep_head(self._head, sh), "deep_head")
        else:
            native.check(k.st_deep_td(self._td, sh), "deep_td")
        for l in reversed(range(self.L)):
            head = self.fuse_head and l == self.L - 1   # TD launch did G_{L-2} and dW_{L-1}
            if not head and self._dual[l]:
                # one launch: G_{l-1} = (G_l . W_l) * (A_l > 0)  and  dW_l = G_l^T . A_l (split-K)
                _, (_, sk) = self._dw_plan[l]
                kw0 = dict(outT=self.GT[l - 1], auxT=actsT[l])
                if self._bpart[l - 1] is not None:
                    kw0["colpart"] = self._bpart[l - 1]
                gm.gemm_dual((self.G[l], self.WbT[l], self.G[l - 1], kw0),
                             gm.EPI_RELU_GRAD,
                             (self.GT[l], actsT[l], self.dW[l], dict(splitk=sk, prezeroed=sk > 1)), gm.EPI_F32)
            elif not head:
                if side is not None and not self.dual_bwd:
                    side.wait_stream(main)        # G_l is ready
                    with torch.cuda.stream(side):
                        self._dw(l, actsT)
                else:   # dual_bwd: the two small leftover weight gradients stay on the main stream
                    self._dw(l, actsT)
            if not self.fused_adam:
                native.check(k.st_row_sum_bf16(self.GT[l].data_ptr(), self.B, self.pdims[l + 1], self.B,
                                               self.db[l].data_ptr(), sh), "bias grad")
            if self.layer_sync is not None and not split:
                comm = self._comm
                comm.wait_stream(main)
                if side is not None and not self.dual_bwd:
                    comm.wait_stream(side)        # dW_l came from the side stream
                with torch.cuda.stream(comm):
                    self.layer_sync(self.dW[l])
                    if self._bias_multi is None:
                        self.layer_sync(self.db[l])
            if l > 0 and not self._dual[l] and not head:
                # G_{l-1} = (G_l . W_l) * (A_l > 0)
                gm.gemm_nt(self.G[l], self.WbT[l], self.G[l - 1], gm.EPI_RELU_GRAD, outT=self.GT[l - 1],
                           auxT=actsT[l])
        if self._bias_multi is not None:
            # every bias gradient in one launch, ahead of the joins (the act step may still be running)
            native.check(k.st_adam_multi(self._bias_multi, sh), "bias grads")
            if self.layer_sync is not None and not split:
                self._comm.wait_stream(main)
                with torch.cuda.stream(self._comm):
                    self.layer_sync(self._db_flat)
        if side is not None and not self.dual_bwd:
            main.wait_stream(side)
        if not split and self.layer_sync is None and self.grad_sync is not None:
            self.grad_sync(self.grad_flat)     # one flat all-reduce, beside a still-running act step
        if split:
            if act is not None:
                main.wait_stream(act)
            return
        if act is not None:
            # the act step's GEMMs read the pre-update weights; with early_adam its env step / replay
            # insert may still run beside Adam
            if self.early_adam:
                main.wait_event(act_fwd_done)
            else:
                main.wait_stream(act)
        if self.layer_sync is not None:
            main.wait_stream(self._comm)
        self._adam_step()
        if act is not None and self.early_adam:
            main.wait_stream(act)

    def _adam_step(self) -> None:
        sh = native.stream_handle()
        k = self.k
        if self.fused_adam:
            native.check(k.st_adam_multi(self._adam_multi, sh), "adam_multi")
        else:
            for ad in self._adam:
                native.check(k.st_adam_tile(ad, sh), "adam")

    def sync_params(self, ctx) -> None:
        """Data-parallel start: every rank takes rank 0's parameters (online and target net)."""
        from ..parallel.dist import broadcast_tensors

        broadcast_tensors(ctx, list(self.W) + list(self.b))
        for l in range(self.L):
            self.Wb[l].copy_(self.W[l].to(torch.bfloat16))
            self.WbT[l].copy_(self.W[l].t().contiguous().to(torch.bfloat16))
        self._refresh_bias_bf()
        self.sync_target()

    def sync_target(self) -> None:
        for l in range(self.L):
            self.Wt[l].copy_(self.Wb[l])
            self.bt[l].copy_(self.b[l])

    # ---------------------------------------------------------------- driver
    def capture(self, iters_per_graph: int = 1) -> None:
        """Capture one act step and one update into HIP graphs (after a warm-up of each).  With
        ``iters_per_graph`` k > 1 (overlapped single-update iterations without a host all-reduce) also k whole
        iterations into one graph, which ``iterations(n)`` replays: one graph launch per k iterations instead
        of per iteration."""
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            if self.overlap_act:
                self.update_step(with_act=True)   # same op order as the captured iteration
            else:
                self.act_step()
                self.update_step()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        self.env_steps += 1
        self.updates += 1
        if self.target_every and self.updates % self.target_every == 0:   # as iteration()
            self.sync_target()
        self._g_act = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_act, capture_error_mode=_CAPTURE_MODE):
            self.act_step()
        self._g_upd = self._g_iter = self._g_pre = self._g_pre_act = self._g_post = None
        if self.grad_sync is None or self.capture_sync:
            self._g_upd = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_upd, capture_error_mode=_CAPTURE_MODE):
                self.update_step()
            if self.overlap_act:
                self._g_iter = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._g_iter, capture_error_mode=_CAPTURE_MODE):
                    self.update_step(with_act=True)
                if iters_per_graph > 1:
                    self._g_iter_k = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self._g_iter_k, capture_error_mode=_CAPTURE_MODE):
                        for _ in range(iters_per_graph):
                            self.update_step(with_act=True)
                    self._iter_k = int(iters_per_graph)
        else:
            # data parallel: the gradient all-reduce runs between two graphs (act + gradients | Adam);
            # the collective itself stays outside the capture
            self._g_pre = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_pre, capture_error_mode=_CAPTURE_MODE):
                self.update_step(split=True)
            if self.overlap_act:
                self._g_pre_act = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._g_pre_act, capture_error_mode=_CAPTURE_MODE):
                    self.update_step(with_act=True, split=True)
            self._g_post = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_post, capture_error_mode=_CAPTURE_MODE):
                self._adam_step()
        self._captured = True

    def _replay_dp(self, with_act: bool) -> None:
        (self._g_pre_act if with_act else self._g_pre).replay()
        self.grad_sync(self.grad_flat)
        self._g_post.replay()

    def iterations(self, n: int) -> None:
        """n single-update iterations: whole k-iteration graphs (``capture(iters_per_graph=k)``) where the
        target-net copy cannot fall inside one (it runs on the host between graphs), single ones otherwise."""
        k = getattr(self, "_iter_k", 1)
        g = getattr(self, "_g_iter_k", None)
        while n > 0:
            if (g is not None and n >= k and (not self.target_every or
                                              self.updates // self.target_every == (self.updates + k - 1) // self.target_every)):
                g.replay()
                self.env_steps += k
                self.updates += k
                if self.target_every and self.updates % self.target_every == 0:
                    self.sync_target()
                n -= k
            else:
                self.iteration()
                n -= 1

    def iteration(self, updates_per_step: int = 1) -> None:
        if self.overlap_act and updates_per_step >= 1:
            if getattr(self, "_g_pre_act", None) is not None:
                self._replay_dp(True)
            elif getattr(self, "_g_iter", None) is not None:
                self._g_iter.replay()
            else:
                self.update_step(with_act=True)
            self.env_steps += 1
            self.updates += 1
            if self.target_every and self.updates % self.target_every == 0:
                self.sync_target()
            updates_per_step -= 1
        else:
            if self._g_act is not None:
                self._g_act.replay()
            else:
                self.act_step()
            self.env_steps += 1
        for _ in range(updates_per_step):
            if getattr(self, "_g_pre", None) is not None:
                self._replay_dp(False)
            elif self._g_upd is not None:
                self._g_upd.replay()
            else:
                self.update_step()
            self.updates += 1
            if self.target_every and self.updates % self.target_every == 0:
                self.sync_target()

    # ---------------------------------------------------------------- checkpoint / resume
    _ENV_KEYS = ("budget", "shares", "value", "pos", "episodes", "last_final", "env_ctrl", "rp_ctrl", "t_ctr",
                 "stats", "loss")

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Everything a resumed run needs to continue exactly (host copies): fp32 masters, Adam moments,
        target net, update / env-step / sampling counters, env state and the whole replay ring.  The
        price bank is not saved: it is regenerated from the config seed (or passed in again)."""
        d: Dict[str, torch.Tensor] = {}
        for l in range(self.L):
            for name, lst in (("W", self.W), ("b", self.b), ("Wm", self.Wm), ("Wv", self.Wv), ("bm", self.bm),
                              ("bv", self.bv), ("Wt", self.Wt), ("bt", self.bt)):
                d[f"{name}{l}"] = lst[l].detach().cpu().clone()
        for k in self._ENV_KEYS:
            d[k] = getattr(self, k).detach().cpu().clone()
        for k, t in self.rp.items():
            d[f"rp_{k}"] = t.detach().cpu().clone()
        d["counters"] = torch.tensor([self.updates, self.env_steps], dtype=torch.int64)
        return d

    def load_state_dict(self, d: Dict[str, torch.Tensor]) -> None:
        for l in range(self.L):
            for name, lst in (("W", self.W), ("b", self.b), ("Wm", self.Wm), ("Wv", self.Wv), ("bm", self.bm),
                              ("bv", self.bv), ("Wt", self.Wt), ("bt", self.bt)):
                lst[l].copy_(d[f"{name}{l}"].to(lst[l].device))
            # the bf16 operand copies are a rounding of the masters (what the Adam kernel writes)
            self.Wb[l].copy_(self.W[l].to(torch.bfloat16))
            self.WbT[l].copy_(self.W[l].t().contiguous().to(torch.bfloat16))
        self._refresh_bias_bf()
        for k in self._ENV_KEYS:
            getattr(self, k).copy_(d[k].to(self.dev))
        for k, t in self.rp.items():
            t.copy_(d[f"rp_{k}"].to(self.dev))
        self.updates, self.env_steps = (int(x) for x in d["counters"].tolist())

    def stats_dict(self) -> Dict[str, float]:
        s = self.stats.cpu().tolist()
        return {"reward_sum": s[0], "explore": s[1], "episodes_done": s[2], "final_sum": s[3],
                "loss_sum": float(self.loss.item()), "replay_size": int(self.rp_ctrl[1].item()),
                "updates": self.updates, "env_steps": self.env_steps * self.E}
