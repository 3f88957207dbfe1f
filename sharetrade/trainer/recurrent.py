"""RecurrentDQN — GRU(256) recurrent Q-net on minute-bar sequences (BASELINE.json config 5).

Not in the reference (its learner is a 203->200->3 MLP trained online at batch 1,
`QDecisionPolicyActor.scala:38-77`, over daily closes, `TrainerChildActor.scala:64-103`).
This is the north-star recurrent variant of the same Buy/Sell/Hold agent, built
actor-learner style (R2D2-like stored-state sequence replay):

* **actor** (``act``): one launch of ``csrc/gru.hip::gru_act_kernel`` advances all E envs by
  S minute bars.  W_hh is block-scaled MX-fp8 resident in VGPRs and the gate products run
  on ``v_mfma_scale_f32_16x16x128_f8f6f4`` (the fp8 MFMA path); h stays fp32 on-chip for
  all S steps; every env writes one replay *segment* {x_0..x_S, a, r, done, h_0}.
* **learner** (``update``): samples B segments; ``csrc/gru_learn.hip`` unrolls online and target
  nets over S+1 steps in one persistent launch (the actor's MX-fp8 arithmetic), double-DQN TD
  over steps [burn_in, S), then backward through time in one persistent launch (W_hh^T
  resident as MX-fp8, the dGh operand as an fp8 hi/lo pair, the recurrent gradient in
  registers), split-K bf16 weight-gradient GEMMs, Adam, and re-packs the fp8 weights.
  Both halves are captured in HIP graphs.

Env (minute-bar trading, long-only single unit like the reference's share count):
Buy -> long, Sell -> flat, Hold -> keep; reward = position * ret_t - ``cost`` per position
change, with ``ret_t = (c_{t+1}/c_t - 1) * 100`` precomputed per bar (``minute_bars.bar_returns``); episodes are ``ep_len`` bars from a random start.
x_t = 8 market features ++ (position, unrealised pnl %, elapsed fraction, 1) zero-padded to 32.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from ..config import Config
from ..data import minute_bars as mb
from ..models import gru_qnet as gq
from ..ops import gemm as gm
from ..ops import gru as G
from ..ops import native
from ..utils import rng
from .deep import _bind as _bind_deep

HID, GATES, XA, XL = G.HID, G.GATES, G.XA, G.XL


# HIP-graph capture mode: "thread_local" -- with an RCCL process group alive, its watchdog thread
# polls collective events during our captures; in the default global mode that poll invalidates the
# capture (hipErrorStreamCaptureInvalidated) and kills the watchdog.  Our own thread stays checked.
_CAPTURE_MODE = "thread_local"


class RecurrentDQN:
    """E minute-bar envs + segment replay + GRU(256) learner on one GPU."""

    def __init__(self, cfg: Config, device: torch.device, envs: int = 65536, seq: int = 16, batch: int = 1024,
                 replay_segments: int = 1 << 17, bars: int = 4096, ep_len: int = 390, burn_in: int = 4,
                 target_every: int = 100, cost: float = 0.01, lr: float = 3e-4, seed: Optional[int] = None,
                 bar_params: Optional[mb.BarParams] = None, actor_grid: int = 0, grad_sync=None,
                 overlap_act: bool = False, actor_kernel: str = "auto", world_size: int = 1):
        if device.type != "cuda":
            raise ValueError("RecurrentDQN runs on the GPU (MX-fp8 / bf16 MFMA kernels)")
        if envs % G.RN:
            raise ValueError(f"envs must be a multiple of {G.RN}")
        if batch % 128 or batch <= 0:
            raise ValueError("batch must be a multiple of 128 (GEMM tiles)")
        if not (0 <= burn_in < seq <= 64):
            raise ValueError("need 0 <= burn_in < seq <= 64")
        if bars < ep_len + 3:
            raise ValueError("bars must exceed the episode length")
        self.cfg, self.dev = cfg, device
        self.E, self.S, self.B, self.cap = int(envs), int(seq), int(batch), int(replay_segments)
        self.T, self.ep_len, self.burn = int(bars), int(ep_len), int(burn_in)
        self.target_every, self.cost, self.lr = int(target_every), float(cost), float(lr)
        self.seed = cfg.agent.seed if seed is None else int(seed)
        self.gamma = float(cfg.agent.gamma)
        # actor_kernel: "single" = gru_act_kernel (one 32-env chunk per workgroup at a time), "pair" =
        # gru_act_pair_kernel (two chunks per workgroup, one chunk's env phase beside the other's MFMA
        # phase; needs seq <= 32), "auto" = pair when it fits.  Same results bit for bit.
        if actor_kernel not in ("auto", "single", "pair"):
            raise ValueError(f"actor_kernel must be auto/single/pair, got {actor_kernel!r}")
        smax = int(G.lib().st_gru_act_pair_smax())
        if actor_kernel == "pair" and self.S > smax:
            raise ValueError(f"the two-chunk actor needs seq <= {smax}")
        self.actor_kernel = ("pair" if self.S <= smax else "single") if actor_kernel == "auto" else actor_kernel
        # data parallel (one process per GPU, trainer/runs.py): grad_sync(gflat) sums the gradient over
        # the ranks between the weight-gradient GEMMs and Adam; the TD coefficient carries 1/world_size
        # so the sum is the mean over the global batch (B x world_size segments)
        self.grad_sync = grad_sync
        self.world_size = int(world_size)
        # capture_sync: the backend's collectives can be captured (RCCL): the all-reduce stays inside the
        # update graph, on the main stream while the overlapped actor still runs on its side stream
        self.capture_sync = False
        # overlap_act: one captured graph per iteration in which the update samples its segments first,
        # then the actor launch runs on a side stream beside the rest of the update (unroll, BPTT,
        # weight-gradient GEMMs, Adam); the MX-fp8 re-pack of the actor weights waits for it (the actor
        # reads the pre-update packed weights, as in the serial order).  Only difference from the
        # serial order: the update samples the ring as it was before this iteration's segments.
        self.overlap_act = bool(overlap_act)
        self._act_stream = torch.cuda.Stream(device=device) if self.overlap_act else None
        self.grid = int(actor_grid) if actor_grid > 0 else self._auto_grid(device)
        self.k = G.lib()
        self.kd = _bind_deep()
        dev, f32, b16, i32, u8 = device, torch.float32, torch.bfloat16, torch.int32, torch.uint8
        # ---------------------------------------------------------------- parameters (one flat buffer)
        p0 = gq.init_params(self.seed)
        self._names = ["w_ih", "w_hh", "b_ih", "b_hh", "w_q", "b_q"]
        sizes = [p0[n].numel() for n in self._names]
        self.n_params = sum(sizes)
        npad = (self.n_params + 3) // 4 * 4          # float4 columns of the flat Adam kernel; tail stays 0
        self.flat = torch.zeros(npad, device=dev)
        self.gflat = torch.zeros(npad, device=dev)
        self.mflat = torch.zeros(npad, device=dev)
        self.vflat = torch.zeros(npad, device=dev)
        self.ones = torch.ones(npad, device=dev)
        self.P, self.dP, self.M1, self.M2 = {}, {}, {}, {}
        o = 0
        for n, sz in zip(self._names, sizes):
            shp = p0[n].shape if p0[n].dim() == 2 else (1, p0[n].numel())
            self.P[n] = self.flat[o:o + sz].view(*shp)
            self.dP[n] = self.gflat[o:o + sz].view(*shp)
            self.M1[n] = self.mflat[o:o + sz].view(*shp)
            self.M2[n] = self.vflat[o:o + sz].view(*shp)
            self.P[n].copy_(p0[n].view(*shp))
            o += sz
        # optimizer control words (csrc/optim.hip): ctrl[0] = completed updates (also the replay
        # sampling counter), ctrl[1] = 1-based count of the update in flight
        self.opt_ctrl = torch.zeros(2, dtype=torch.int64, device=dev)
        self.t_ctr = self.opt_ctrl[:1]
        # target net: an fp32 copy of the flat parameters, packed like the actor's weights
        self.tflat = self.flat.clone()
        self.T_P = {}
        o = 0
        for n, sz in zip(self._names, sizes):
            self.T_P[n] = self.tflat[o:o + sz].view(*self.P[n].shape)
            o += sz
        # packed weights (gru_pack_kernel layout): online (actor + learner fwd) and target
        nfr = G.RW * 3 * 2 * 2 * 64
        self.pk = {}
        for net in ("on", "tg"):
            self.pk[net] = {"whh8": torch.zeros(nfr * 8, dtype=i32, device=dev),
                            "whhs": torch.zeros(nfr, dtype=i32, device=dev),
                            "wih": torch.zeros(G.RW * 6 * 64 * 8, dtype=torch.int16, device=dev),
                            "bias4": torch.zeros(4 * HID, device=dev), "wq": torch.zeros(4 * HID, device=dev)}
        # the learner's backward dh GEMM reads W_hh^T as resident MX-fp8 fragments too (online net only)
        self.pk["on"]["whhT8"] = torch.zeros(nfr * 8, dtype=i32, device=dev)
        self.pk["on"]["whhTs"] = torch.zeros(nfr, dtype=i32, device=dev)
        # a second online set: the overlapped iteration re-packs the updated weights into the other set
        # while the actor still reads this one, so the re-pack need not wait for the actor (the sets
        # alternate: ``_par`` is the set holding the current weights)
        self.pk["on1"] = {k: torch.zeros_like(v) for k, v in self.pk["on"].items()}
        self._par = 0
        # ---------------------------------------------------------------- data + envs
        self.bp = bar_params or mb.BarParams()
        self.close, self.feat = mb.generate_gpu(self.E, self.T, dev, self.bp, seed=self.seed)
        self.ret = mb.bar_returns(self.close)
        g = np.random.default_rng(self.seed)
        start = torch.from_numpy(g.integers(0, self.T - self.ep_len - 1, size=self.E).astype(np.int32)).to(dev)
        self.h = torch.zeros(self.E, HID, device=dev)
        self.pos = start.clone()
        self.ep_start = start.clone()
        self.position = torch.zeros(self.E, dtype=i32, device=dev)
        self.entry = torch.zeros(self.E, device=dev)
        self.ep_ret = torch.zeros(self.E, device=dev)
        self.episodes = torch.zeros(self.E, dtype=i32, device=dev)
        self.last_ret = torch.full((self.E,), float("nan"), device=dev)
        # replay segments
        S = self.S
        self.rx = torch.zeros(self.cap, S + 1, XA, dtype=b16, device=dev)
        self.ra = torch.zeros(self.cap, S, dtype=u8, device=dev)
        self.rr = torch.zeros(self.cap, S, device=dev)
        self.rd = torch.zeros(self.cap, S, dtype=u8, device=dev)
        self.rh0 = torch.zeros(self.cap, HID, dtype=b16, device=dev)
        self.rctrl = torch.zeros(2, dtype=torch.int64, device=dev)
        self.ctrl = torch.zeros(1, dtype=torch.int64, device=dev)
        # the pair actor's finished-workgroup count (its last workgroup advances rctrl / ctrl; always 0
        # between launches)
        self._act_done = torch.zeros(1, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(4, device=dev)
        self.loss = torch.zeros(1, device=dev)
        # ---------------------------------------------------------------- learner buffers (time-major rows t*B + b)
        B, R1, RS = self.B, (S + 1) * self.B, S * self.B
        if B % G.LB:
            raise ValueError(f"batch must be a multiple of {G.LB}")
        self.X = torch.zeros(R1, XL, dtype=b16, device=dev)
        self.XT = torch.zeros(XL, R1, dtype=b16, device=dev)
        self.H0 = torch.zeros(B, HID, device=dev)
        # h_{t-1}^T for the dW_hh GEMM, with a ones row at HID: column HID of that GEMM is then db_hh
        self.HT = torch.zeros(HID + 64, R1, dtype=b16, device=dev)
        self.HT[HID].fill_(1.0)
        self.dWhh_ext = torch.zeros(GATES, HID + 64, device=dev)
        self.A = torch.zeros(S, B, dtype=i32, device=dev)
        self.R = torch.zeros(S, B, device=dev)
        self.D = torch.zeros(S, B, device=dev)
        self.Q = torch.zeros(R1, 4, device=dev)
        self.Q_t = torch.zeros(R1, 4, device=dev)
        # forward saves (r, z, n, gh_n, h_prev as bf16 in the kernels' lane order): 16 B per lane/tile/quantity
        self.sv = torch.zeros(S * (B // G.LB) * G.RW * G.NSV * 2 * 64 * 4, dtype=i32, device=dev)
        self.dQ = torch.zeros(RS, 4, device=dev)
        self.dGxT = torch.zeros(GATES, RS, dtype=b16, device=dev)
        self.dGhT = torch.zeros(GATES, RS, dtype=b16, device=dev)
        self.key0, self.key1 = (int(x) for x in rng.key_for(self.seed, 7))
        self.updates = 0
        self.launches = 0
        self._g_act = self._g_upd = self._g_iter = None
        self._g_acts, self._g_upds, self._g_iters = {}, {}, {}
        self._build_structs()
        self.pack("on", into=0)
        self.pack("on", into=1)
        self.pack("tg")

    # ---------------------------------------------------------------- structs
    @property
    def _act(self):
        """The actor's launch arguments for the current online set."""
        return self._acts[self._par]

    @property
    def whh8(self) -> torch.Tensor:
        return self._on(self._par)["whh8"]

    @property
    def whhs(self) -> torch.Tensor:
        return self._on(self._par)["whhs"]

    def _on(self, p: int) -> Dict[str, torch.Tensor]:
        return self.pk["on" if p == 0 else "on1"]

    def _build_structs(self) -> None:
        self._acts, self._pack_on = [], []
        for par in (0, 1):
            a = G.ActArgs()
            po = self._on(par)
            a.whh8, a.whhs, a.wih, a.bias4, a.wq = (po[k].data_ptr() for k in ("whh8", "whhs", "wih", "bias4", "wq"))
            a.feat, a.close, a.ret = self.feat.data_ptr(), self.close.data_ptr(), self.ret.data_ptr()
            a.E, a.T, a.S, a.ep_len = self.E, self.T, self.S, self.ep_len
            ag = self.cfg.agent
            a.eps, a.inv_ramp, a.cost = float(ag.epsilon), float(np.float32(1.0 / ag.ramp)), self.cost
            a.inv_ep_len = float(np.float32(1.0 / self.ep_len))
            for n in ("h", "pos", "ep_start", "position", "entry", "ep_ret", "episodes", "last_ret"):
                setattr(a, n, getattr(self, n).data_ptr())
            a.rx, a.ra, a.rr, a.rd, a.rh0 = (self.rx.data_ptr(), self.ra.data_ptr(), self.rr.data_ptr(),
                                             self.rd.data_ptr(), self.rh0.data_ptr())
            a.rctrl, a.cap = self.rctrl.data_ptr(), self.cap
            a.key0, a.key1 = (int(x) for x in rng.key_for(self.seed, 5))
            a.ctrl, a.stats, a.q_out = self.ctrl.data_ptr(), self.stats.data_ptr(), None
            a.done_ctr = self._act_done.data_ptr()   # (used by the pair actor only)
            self._acts.append(a)
        self._packs = {}
        for net, src in (("on0", self.P), ("on1", self.P), ("tg", self.T_P)):
            p = G.PackArgs()
            p.w_hh, p.w_ih, p.b_ih, p.b_hh, p.w_q, p.b_q = (src[n].data_ptr() for n in
                                                             ("w_hh", "w_ih", "b_ih", "b_hh", "w_q", "b_q"))
            pk = self.pk[net] if net == "tg" else self._on(int(net[-1]))
            p.whh8, p.whhs, p.wih, p.bias4, p.wq = (pk[k].data_ptr() for k in ("whh8", "whhs", "wih", "bias4", "wq"))
            if "whhT8" in pk:
                p.whhT8, p.whhTs = pk["whhT8"].data_ptr(), pk["whhTs"].data_ptr()
            self._packs[net] = p
        ga = G.GatherArgs()
        ga.rx, ga.ra, ga.rr, ga.rd, ga.rh0 = (self.rx.data_ptr(), self.ra.data_ptr(), self.rr.data_ptr(),
                                              self.rd.data_ptr(), self.rh0.data_ptr())
        ga.rctrl, ga.cap, ga.S, ga.B = self.rctrl.data_ptr(), self.cap, self.S, self.B
        ga.key0, ga.key1, ga.step = self.key0, self.key1, self.t_ctr.data_ptr()
        ga.X, ga.H0 = self.X.data_ptr(), self.H0.data_ptr()
        ga.A, ga.R, ga.D = self.A.data_ptr(), self.R.data_ptr(), self.D.data_ptr()
        self._gather = ga
        self._fwds = []
        for par in (0, 1):
            f = G.SeqFwdArgs()
            for pk, w in ((self._on(par), f.on), (self.pk["tg"], f.tg)):
                w.whh8, w.whhs, w.wih, w.bias4, w.wq = (pk[k].data_ptr() for k in ("whh8", "whhs", "wih", "bias4",
                                                                                  "wq"))
            f.X, f.H0, f.D = self.X.data_ptr(), self.H0.data_ptr(), self.D.data_ptr()
            f.Q, f.Qt, f.sv = self.Q.data_ptr(), self.Q_t.data_ptr(), self.sv.data_ptr()
            f.HT, f.ldht = self.HT.data_ptr(), int(self.HT.stride(0))
            f.B, f.S = self.B, self.S
            self._fwds.append(f)
        td = G.TDArgs()
        td.Q, td.Qt, td.A, td.R, td.D = (self.Q.data_ptr(), self.Q_t.data_ptr(), self.A.data_ptr(), self.R.data_ptr(),
                                         self.D.data_ptr())
        td.dQ, td.loss, td.B, td.S, td.burn = self.dQ.data_ptr(), self.loss.data_ptr(), self.B, self.S, self.burn
        td.gamma, td.coef = self.gamma, 2.0 / (self.B * (self.S - self.burn) * self.world_size)
        self._td = td
        self._bwds = []
        for par in (0, 1):
            bw = G.SeqBwdArgs()
            bw.sv, bw.dQ, bw.D, bw.wq = (self.sv.data_ptr(), self.dQ.data_ptr(), self.D.data_ptr(),
                                         self.P["w_q"].data_ptr())
            bw.whhT8, bw.whhTs = self._on(par)["whhT8"].data_ptr(), self._on(par)["whhTs"].data_ptr()
            bw.dGxT, bw.dGhT = self.dGxT.data_ptr(), self.dGhT.data_ptr()
            bw.gwq, bw.gbq = self.dP["w_q"].data_ptr(), self.dP["b_q"].data_ptr()
            bw.B, bw.S = self.B, self.S
            self._bwds.append(bw)
        ag = self.cfg.agent
        op = native.OptimParams()
        op.params, op.mask, op.s1, op.s2 = (self.flat.data_ptr(), self.ones.data_ptr(), self.mflat.data_ptr(),
                                            self.vflat.data_ptr())
        op.grad, op.ctrl = self.gflat.data_ptr(), self.opt_ctrl.data_ptr()
        op.G, op.P, op.kind, op.mode = 0, self.flat.numel(), 2, 2
        op.lr, op.beta1, op.beta2, op.eps, op.scale = (self.lr, float(ag.adam_betas[0]), float(ag.adam_betas[1]),
                                                       float(ag.adam_eps), 1.0)
        self._opt = op

    # ---------------------------------------------------------------- actor
    def _auto_grid(self, device: torch.device) -> int:
        """Actor workgroups (one per CU): all CUs, or 7/8 of them when the update runs beside the actor
        (its unroll / BPTT kernels take the rest) -- then trimmed to the fewest workgroups that still
        finish the chunk (or chunk-pair) work in the same number of rounds, freeing CUs for free."""
        cus = torch.cuda.get_device_properties(device).multi_processor_count
        avail = cus if not self.overlap_act else cus - cus // 8
        work = self.E // G.RN
        if self.actor_kernel == "pair":
            work = (work + 1) // 2
        rounds = -(-work // avail)
        return -(-work // rounds)

    def pack(self, net: str = "on", into: Optional[int] = None) -> None:
        """fp32 masters -> MX-fp8 W_hh fragments, bf16 W_ih fragments, biases, W_q (actor/learner layout).
        ``net="on"`` packs into online set ``into`` (default: the current one)."""
        key = "tg" if net == "tg" else f"on{self._par if into is None else int(into)}"
        native.check(self.k.st_gru_pack(self._packs[key], native.stream_handle()), "st_gru_pack")

    def act(self) -> None:
        """All E envs advance S minute bars (one actor launch) and write one replay segment each."""
        if self.actor_kernel == "pair":
            native.check(self.k.st_gru_act_pair(self._acts[self._par], self.grid, native.stream_handle()),
                         "st_gru_act_pair")
        else:
            native.check(self.k.st_gru_act(self._acts[self._par], self.grid, native.stream_handle()), "st_gru_act")

    # ---------------------------------------------------------------- learner
    def update(self, with_act: bool = False, flip: bool = False) -> None:
        """One learner update on B sampled segments: gather -> fused unroll of both nets (MX-fp8) ->
        TD -> fused BPTT (bf16) -> split-K weight-gradient GEMMs -> Adam -> repack the actor weights.
        ``with_act``: the actor launch runs on a side stream right after the gather (see overlap_act).
        ``flip``: re-pack into the other online set without waiting for the actor; the caller then
        switches ``_par`` (the overlapped iteration)."""
        act = self._grads(with_act)
        if self.grad_sync is not None:
            self.grad_sync(self.gflat)
        self._apply(act, flip)

    def _grads(self, with_act: bool = False, join: bool = False):
        """Gather -> unroll -> TD -> BPTT -> weight gradients into ``gflat``.  Returns the actor's side
        stream when it is still running (``join`` makes the main stream wait for it here instead)."""
        sh = native.stream_handle()
        k, kd = self.k, self.kd
        S, B = self.S, self.B
        RS, R1 = S * B, (S + 1) * B
        native.check(k.st_gru_gather(self._gather, sh), "st_gru_gather")
        main = torch.cuda.current_stream(self.dev)
        act = self._act_stream if with_act else None
        if with_act:
            if act is None:
                raise RuntimeError("update(with_act=True) needs overlap_act=True")
            act.wait_stream(main)          # segments sampled: the actor may insert now
            with torch.cuda.stream(act):
                self.act()
        native.check(k.st_gru_seq_fwd(self._fwds[self._par], sh), "st_gru_seq_fwd")
        self.loss.zero_()
        native.check(k.st_gru_td(self._td, sh), "st_gru_td")
        self.gflat.zero_()
        native.check(k.st_gru_seq_bwd(self._bwds[self._par], sh), "st_gru_seq_bwd")
        native.check(kd.st_transpose_bf16(self.X.data_ptr(), XL, self.XT.data_ptr(), R1, RS, XL, sh), "T X")
        # weight gradients; the ones row of HT / ones column RF of X give the bias gradients for free
        gm.gemm_nt(self.dGhT, self.HT[:, :RS], self.dWhh_ext, gm.EPI_F32, splitk="auto")
        gm.gemm_nt(self.dGxT, self.XT[:, :RS], self.dP["w_ih"], gm.EPI_F32, accumulate=True, splitk="auto")
        native.check(k.st_gru_grad_fixup(self.dWhh_ext.data_ptr(), HID + 64, self.dP["w_hh"].data_ptr(),
                                         self.dP["b_hh"].data_ptr(), self.dP["w_ih"].data_ptr(),
                                         self.dP["b_ih"].data_ptr(), sh), "grad fixup")
        if act is not None and join:
            main.wait_stream(act)
            act = None
        return act

    def _apply(self, act=None, flip: bool = False) -> None:
        """Adam on the (synchronised) gradient, then re-pack the actor's MX-fp8 weights."""
        sh = native.stream_handle()
        nl = native.lib()
        native.check(nl.st_advance(self.opt_ctrl.data_ptr(), sh), "advance")
        native.check(nl.st_reduce_optim(self._opt, sh), "adam")
        main = torch.cuda.current_stream(self.dev)
        if flip:
            self.pack("on", into=1 - self._par)   # the running actor reads the current set
            if act is not None:
                main.wait_stream(act)
        else:
            if act is not None:
                main.wait_stream(act)             # the actor reads the packed weights
            self.pack("on")

    def sync_params(self, ctx) -> None:
        """Data-parallel start: every rank takes rank 0's parameters (online and target net)."""
        from ..parallel.dist import broadcast_tensors

        broadcast_tensors(ctx, [self.flat])
        self.tflat.copy_(self.flat)
        self.pack("on", into=0)
        self.pack("on", into=1)
        self.pack("tg")

    def sync_target(self) -> None:
        self.tflat.copy_(self.flat)
        self.pack("tg")

    # ---------------------------------------------------------------- driver
    def _flips(self) -> bool:
        """Whether the overlapped iteration alternates the online sets (not in the split DP capture)."""
        return self.grad_sync is None or self.capture_sync

    def capture(self, iters_per_graph: int = 1) -> None:
        """Warm up, then capture the actor launch, the learner update and (overlap_act) the whole
        iteration into HIP graphs -- one of each per online weight set.  ``iters_per_graph`` k > 1 (even;
        overlapped, alternating sets, no host all-reduce): also k whole iterations per graph, one per
        starting set, which ``iterations(n)`` replays."""
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        flip = self.overlap_act and self._flips()
        with torch.cuda.stream(s):
            if self.overlap_act:
                self.update(with_act=True, flip=flip)   # same op order as the captured iteration
            else:
                self.act()
                self.update()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        if flip:
            self._par ^= 1
        self.launches += 1
        self.updates += 1
        if self.updates % self.target_every == 0:   # the warm-up is a full iteration (as iteration())
            self.sync_target()
        cur = self._par
        self._g_acts, self._g_upds, self._g_iters = {}, {}, {}
        self._g_pre = self._g_pre_act = self._g_post = None
        for par in (0, 1):
            self._par = par
            self._g_acts[par] = g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                self.act()
            if self._flips():
                self._g_upds[par] = g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                    self.update()
                if self.overlap_act:
                    self._g_iters[par] = g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                        self.update(with_act=True, flip=True)
        self._g_iters_k, self._iter_k = {}, 1
        if self.overlap_act and self._flips() and iters_per_graph > 1:
            if iters_per_graph % 2:
                raise ValueError("iters_per_graph must be even (the online sets alternate)")
            for par in (0, 1):
                self._par = par
                self._g_iters_k[par] = g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                    for _ in range(iters_per_graph):
                        self.update(with_act=True, flip=True)
                        self._par ^= 1
            self._iter_k = int(iters_per_graph)
        self._par = cur
        if not self._flips():
            # data parallel: the gradient all-reduce runs between two graphs (gradients | Adam + re-pack),
            # the collective itself stays outside the capture; the actor joins at the end of the first
            # (the online set never alternates here)
            self._g_pre = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_pre, capture_error_mode=_CAPTURE_MODE):
                self._grads()
            if self.overlap_act:
                self._g_pre_act = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._g_pre_act, capture_error_mode=_CAPTURE_MODE):
                    self._grads(with_act=True, join=True)
            self._g_post = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_post, capture_error_mode=_CAPTURE_MODE):
                self._apply()
        self._g_act, self._g_upd, self._g_iter = (self._g_acts.get(0), self._g_upds.get(0), self._g_iters.get(0))
        self._captured = True

    def _replay_dp(self, with_act: bool) -> None:
        (self._g_pre_act if with_act else self._g_pre).replay()
        self.grad_sync(self.gflat)
        self._g_post.replay()

    def act_step(self) -> None:
        g = self._g_acts.get(self._par)
        if g is not None:
            g.replay()
        else:
            self.act()
        self.launches += 1

    def update_step(self) -> None:
        if getattr(self, "_g_pre", None) is not None:
            self._replay_dp(False)
        elif self._g_upds.get(self._par) is not None:
            self._g_upds[self._par].replay()
        else:
            self.update()
        self.updates += 1
        if self.updates % self.target_every == 0:
            self.sync_target()

    def iterations(self, n: int) -> None:
        """n single-update iterations: whole k-iteration graphs (``capture(iters_per_graph=k)``) where no
        target-net copy falls inside one (it runs on the host between graphs), single ones otherwise."""
        k = getattr(self, "_iter_k", 1)
        gs = getattr(self, "_g_iters_k", {})
        while n > 0:
            if gs and n >= k and self.updates // self.target_every == (self.updates + k - 1) // self.target_every:
                gs[self._par].replay()   # k even: the set alternates back
                self.launches += k
                self.updates += k
                if self.updates % self.target_every == 0:
                    self.sync_target()
                n -= k
            else:
                self.iteration()
                n -= 1

    def iteration(self, updates: int = 1) -> None:
        if self.overlap_act and updates >= 1:
            if getattr(self, "_g_pre_act", None) is not None:
                self._replay_dp(True)
            elif self._g_iters.get(self._par) is not None:
                self._g_iters[self._par].replay()
                self._par ^= 1
            else:
                self.update(with_act=True, flip=self._flips())
                if self._flips():
                    self._par ^= 1
            self.launches += 1
            self.updates += 1
            if self.updates % self.target_every == 0:
                self.sync_target()
            updates -= 1
        else:
            self.act_step()
        for _ in range(updates):
            self.update_step()

    # ---------------------------------------------------------------- checkpoint / resume
    _STATE_KEYS = ("flat", "mflat", "vflat", "tflat", "opt_ctrl", "h", "pos", "ep_start", "position", "entry",
                   "ep_ret", "episodes", "last_ret", "rx", "ra", "rr", "rd", "rh0", "rctrl", "ctrl", "stats", "loss")

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Host copies of the parameters, Adam moments, target net, counters, env / recurrent state and
        the replay ring; the minute bars are regenerated from the seed.  Packed (MX-fp8) weights are
        derived and re-packed on load."""
        d = {k: getattr(self, k).detach().cpu().clone() for k in self._STATE_KEYS}
        d["counters"] = torch.tensor([self.updates, self.launches], dtype=torch.int64)
        return d

    def load_state_dict(self, d: Dict[str, torch.Tensor]) -> None:
        for k in self._STATE_KEYS:
            getattr(self, k).copy_(d[k].to(self.dev))
        self.updates, self.launches = (int(x) for x in d["counters"].tolist())
        self.pack("on", into=0)
        self.pack("on", into=1)
        self.pack("tg")

    @property
    def env_steps(self) -> int:
        return self.launches * self.S * self.E

    def stats_dict(self) -> Dict[str, float]:
        st = self.stats.detach().cpu().numpy().astype(np.float64)
        steps = max(1, self.env_steps)
        return {"env_steps": self.env_steps, "updates": self.updates, "reward_per_step": float(st[0] / steps),
                "explore_frac": float(st[1] / steps), "episodes": int(st[2]),
                "episode_return_mean": float(st[3] / st[2]) if st[2] > 0 else float("nan"),
                "replay_segments": int(self.rctrl[1].item()),
                "loss": float(self.loss.item()) / (self.B * (self.S - self.burn))}
