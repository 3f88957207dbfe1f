"""RecurrentDQN — GRU(256) recurrent Q-net on minute-bar sequences (BASELINE.json config 5).

Not in the reference (its learner is a 203->200->3 MLP trained online at batch 1,
`QDecisionPolicyActor.scala:38-77`, over daily closes, `TrainerChildActor.scala:64-103`).
This is the north-star recurrent variant of the same Buy/Sell/Hold agent, built
actor-learner style (R2D2-like stored-state sequence replay):

* **actor** (``act``): one launch of ``csrc/gru.hip::gru_act_kernel`` advances all E envs by
  S minute bars.  W_hh is block-scaled MX-fp8 resident in VGPRs and the gate products run
  on ``v_mfma_scale_f32_16x16x128_f8f6f4`` (the fp8 MFMA path); h stays fp32 on-chip for
  all S steps; every env writes one replay *segment* {x_0..x_S, a, r, done, h_0}.
* **learner** (``update``): samples B segments, unrolls online and target nets over S+1
  steps (bf16 MFMA GEMMs for the gate products, fused elementwise GRU kernels with the
  Q head folded in), double-DQN TD over steps [burn_in, S), backward through time (per-step
  dh GEMM + fused GRU backward), split-K weight-gradient GEMMs, Adam, then re-packs the
  actor's fp8 weights.  Both halves are captured in HIP graphs.

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
from .deep import _Adam, _bind as _bind_deep

HID, GATES, XA, XL = G.HID, G.GATES, G.XA, G.XL


class RecurrentDQN:
    """E minute-bar envs + segment replay + GRU(256) learner on one GPU."""

    def __init__(self, cfg: Config, device: torch.device, envs: int = 65536, seq: int = 16, batch: int = 1024,
                 replay_segments: int = 1 << 17, bars: int = 4096, ep_len: int = 390, burn_in: int = 4,
                 target_every: int = 100, cost: float = 0.01, lr: float = 3e-4, seed: Optional[int] = None,
                 bar_params: Optional[mb.BarParams] = None, actor_grid: int = 256, grad_sync=None):
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
        self.grid = int(actor_grid)
        self.grad_sync = grad_sync
        self.k = G.lib()
        self.kd = _bind_deep()
        dev, f32, b16, i32, u8 = device, torch.float32, torch.bfloat16, torch.int32, torch.uint8
        # ---------------------------------------------------------------- parameters (one flat buffer)
        p0 = gq.init_params(self.seed)
        self._names = ["w_ih", "w_hh", "b_ih", "b_hh", "w_q", "b_q"]
        sizes = [p0[n].numel() for n in self._names]
        self.n_params = sum(sizes)
        self.flat = torch.zeros(self.n_params, device=dev)
        self.gflat = torch.zeros(self.n_params, device=dev)
        self.mflat = torch.zeros(self.n_params, device=dev)
        self.vflat = torch.zeros(self.n_params, device=dev)
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
        # bf16 operand copies (written by the Adam kernel) and the target net
        self.Wih_b = self.P["w_ih"].to(b16).contiguous()
        self.Whh_b = self.P["w_hh"].to(b16).contiguous()
        self.WhhT_b = self.P["w_hh"].t().contiguous().to(b16)
        self._scratch = {n: torch.zeros(self.P[n].shape, dtype=b16, device=dev) for n in ("b_ih", "b_hh", "w_q", "b_q")}
        self.tgt = {"w_ih": self.Wih_b.clone(), "w_hh": self.Whh_b.clone(), "b_ih": self.P["b_ih"].clone(),
                    "b_hh": self.P["b_hh"].clone(), "w_q": self.P["w_q"].clone(), "b_q": self.P["b_q"].clone()}
        self.t_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        # packed actor weights
        nfr = G.RW * 3 * 2 * 2 * 64
        self.whh8 = torch.zeros(nfr * 8, dtype=i32, device=dev)
        self.whhs = torch.zeros(nfr, dtype=i32, device=dev)
        self.wih_pk = torch.zeros(G.RW * 6 * 64 * 8, dtype=torch.int16, device=dev)
        self.bias4 = torch.zeros(4 * HID, device=dev)
        self.wq4 = torch.zeros(4 * HID, device=dev)
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
        self.stats = torch.zeros(4, device=dev)
        self.loss = torch.zeros(1, device=dev)
        # ---------------------------------------------------------------- learner buffers (time-major rows t*B + b)
        B, R1, RS = self.B, (S + 1) * self.B, S * self.B
        self.X = torch.zeros(R1, XL, dtype=b16, device=dev)
        self.XT = torch.zeros(XL, R1, dtype=b16, device=dev)
        self.Hm = torch.zeros(R1, HID, dtype=b16, device=dev)
        self.Hm_t = torch.zeros(R1, HID, dtype=b16, device=dev)
        self.HT = torch.zeros(HID, R1, dtype=b16, device=dev)
        self.Hf = torch.zeros(B, HID, device=dev)
        self.Hf_t = torch.zeros(B, HID, device=dev)
        self.A = torch.zeros(S, B, dtype=i32, device=dev)
        self.R = torch.zeros(S, B, device=dev)
        self.D = torch.zeros(S, B, device=dev)
        self.Gx = torch.zeros(R1, GATES, device=dev)
        self.Gx_t = torch.zeros(R1, GATES, device=dev)
        self.Gh = torch.zeros(B, GATES, device=dev)
        self.Gh_t = torch.zeros(B, GATES, device=dev)
        self.Q = torch.zeros(R1, 4, device=dev)
        self.Q_t = torch.zeros(R1, 4, device=dev)
        self.sv = {k: torch.zeros(RS, HID, device=dev) for k in ("r", "z", "n", "gh", "hp")}
        self.Hq = torch.zeros(RS, HID, dtype=b16, device=dev)
        self.dQ = torch.zeros(RS, 4, device=dev)
        self.DH = torch.zeros(B, HID, device=dev)
        self.dGx = torch.zeros(RS, GATES, dtype=b16, device=dev)
        self.dGh = torch.zeros(RS, GATES, dtype=b16, device=dev)
        self.dGxT = torch.zeros(GATES, RS, dtype=b16, device=dev)
        self.dGhT = torch.zeros(GATES, RS, dtype=b16, device=dev)
        self.key0, self.key1 = (int(x) for x in rng.key_for(self.seed, 7))
        self.updates = 0
        self.launches = 0
        self._g_act = None
        self._g_upd = None
        self._build_structs()
        self.pack()

    # ---------------------------------------------------------------- structs
    def _build_structs(self) -> None:
        a = G.ActArgs()
        a.whh8, a.whhs, a.wih, a.bias4, a.wq = (self.whh8.data_ptr(), self.whhs.data_ptr(), self.wih_pk.data_ptr(),
                                                self.bias4.data_ptr(), self.wq4.data_ptr())
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
        self._act = a
        p = G.PackArgs()
        p.w_hh, p.w_ih, p.b_ih, p.b_hh, p.w_q, p.b_q = (self.P[n].data_ptr() for n in
                                                         ("w_hh", "w_ih", "b_ih", "b_hh", "w_q", "b_q"))
        p.whh8, p.whhs, p.wih, p.bias4, p.wq = (self.whh8.data_ptr(), self.whhs.data_ptr(), self.wih_pk.data_ptr(),
                                                self.bias4.data_ptr(), self.wq4.data_ptr())
        self._pack = p
        ga = G.GatherArgs()
        ga.rx, ga.ra, ga.rr, ga.rd, ga.rh0 = (self.rx.data_ptr(), self.ra.data_ptr(), self.rr.data_ptr(),
                                              self.rd.data_ptr(), self.rh0.data_ptr())
        ga.rctrl, ga.cap, ga.S, ga.B = self.rctrl.data_ptr(), self.cap, self.S, self.B
        ga.key0, ga.key1, ga.step = self.key0, self.key1, self.t_ctr.data_ptr()
        ga.X, ga.Hm, ga.Hm_t, ga.Hf, ga.Hf_t = (self.X.data_ptr(), self.Hm.data_ptr(), self.Hm_t.data_ptr(),
                                                self.Hf.data_ptr(), self.Hf_t.data_ptr())
        ga.A, ga.R, ga.D = self.A.data_ptr(), self.R.data_ptr(), self.D.data_ptr()
        self._gather = ga
        self._fwd_on, self._fwd_tg = [], []
        for t in range(self.S + 1):
            for net, lst in (("on", self._fwd_on), ("tg", self._fwd_tg)):
                f = G.FwdArgs()
                on = net == "on"
                f.Gx = (self.Gx if on else self.Gx_t).data_ptr()
                f.Gh = (self.Gh if on else self.Gh_t).data_ptr()
                f.Hf = (self.Hf if on else self.Hf_t).data_ptr()
                f.Hm = (self.Hm if on else self.Hm_t).data_ptr()
                f.wq = (self.P["w_q"] if on else self.tgt["w_q"]).data_ptr()
                f.bq = (self.P["b_q"] if on else self.tgt["b_q"]).data_ptr()
                f.Q = (self.Q if on else self.Q_t).data_ptr()
                f.D = self.D.data_ptr()
                if on and t < self.S:
                    f.sr, f.sz, f.sn, f.sgh, f.shp = (self.sv[k].data_ptr() for k in ("r", "z", "n", "gh", "hp"))
                    f.Hq = self.Hq.data_ptr()
                f.B, f.S, f.t = self.B, self.S, t
                lst.append(f)
        td = G.TDArgs()
        td.Q, td.Qt, td.A, td.R, td.D = (self.Q.data_ptr(), self.Q_t.data_ptr(), self.A.data_ptr(), self.R.data_ptr(),
                                         self.D.data_ptr())
        td.dQ, td.loss, td.B, td.S, td.burn = self.dQ.data_ptr(), self.loss.data_ptr(), self.B, self.S, self.burn
        td.gamma, td.coef = self.gamma, 2.0 / (self.B * (self.S - self.burn))
        self._td = td
        self._bwd = []
        for t in range(self.S):
            b = G.BwdArgs()
            b.dQ, b.D, b.DH = self.dQ.data_ptr(), self.D.data_ptr(), self.DH.data_ptr()
            b.sr, b.sz, b.sn, b.sgh, b.shp = (self.sv[k].data_ptr() for k in ("r", "z", "n", "gh", "hp"))
            b.wq, b.dGx, b.dGh = self.P["w_q"].data_ptr(), self.dGx.data_ptr(), self.dGh.data_ptr()
            b.B, b.S, b.t = self.B, self.S, t
            self._bwd.append(b)
        ag = self.cfg.agent
        self._adam = []
        for n in self._names:
            ad = _Adam()
            w = self.P[n]
            ad.w, ad.g, ad.m, ad.v, ad.mask = w.data_ptr(), self.dP[n].data_ptr(), self.M1[n].data_ptr(), \
                self.M2[n].data_ptr(), None
            wb = {"w_ih": self.Wih_b, "w_hh": self.Whh_b}.get(n, self._scratch.get(n))
            ad.wb = wb.data_ptr()
            ad.wbT = self.WhhT_b.data_ptr() if n == "w_hh" else None
            ad.t, ad.O, ad.I = self.t_ctr.data_ptr(), int(w.shape[0]), int(w.shape[1])
            ad.lr, ad.beta1, ad.beta2, ad.eps = self.lr, float(ag.adam_betas[0]), float(ag.adam_betas[1]), \
                float(ag.adam_eps)
            self._adam.append(ad)

    # ---------------------------------------------------------------- actor
    def pack(self) -> None:
        """fp32 masters -> the actor's MX-fp8 W_hh fragments, bf16 W_ih fragments, biases, W_q."""
        native.check(self.k.st_gru_pack(self._pack, native.stream_handle()), "st_gru_pack")

    def act(self) -> None:
        """All E envs advance S minute bars (one actor launch) and write one replay segment each."""
        native.check(self.k.st_gru_act(self._act, self.grid, native.stream_handle()), "st_gru_act")

    # ---------------------------------------------------------------- learner
    def _forward(self, on: bool) -> None:
        sh = native.stream_handle()
        Wih = self.Wih_b if on else self.tgt["w_ih"]
        Whh = self.Whh_b if on else self.tgt["w_hh"]
        bih = (self.P["b_ih"] if on else self.tgt["b_ih"]).view(-1)
        bhh = (self.P["b_hh"] if on else self.tgt["b_hh"]).view(-1)
        Gx, Gh, Hm = (self.Gx, self.Gh, self.Hm) if on else (self.Gx_t, self.Gh_t, self.Hm_t)
        fw = self._fwd_on if on else self._fwd_tg
        gm.gemm_nt(self.X, Wih, Gx, gm.EPI_F32, bias=bih)
        B = self.B
        for t in range(self.S + 1):
            gm.gemm_nt(Hm[t * B:(t + 1) * B], Whh, Gh, gm.EPI_F32, bias=bhh)
            native.check(self.k.st_gru_fwd(fw[t], sh), "st_gru_fwd")

    def update(self) -> None:
        """One learner update on B sampled segments (sample -> unroll x2 -> TD -> BPTT -> Adam -> repack)."""
        sh = native.stream_handle()
        k, kd = self.k, self.kd
        S, B = self.S, self.B
        RS, R1 = S * B, (S + 1) * B
        native.check(k.st_gru_gather(self._gather, sh), "st_gru_gather")
        self._forward(True)
        self._forward(False)
        self.loss.zero_()
        native.check(k.st_gru_td(self._td, sh), "st_gru_td")
        self.gflat.zero_()
        for t in reversed(range(S)):
            native.check(k.st_gru_bwd(self._bwd[t], sh), "st_gru_bwd")
            if t > 0:
                gm.gemm_nt(self.dGh[t * B:(t + 1) * B], self.WhhT_b, self.DH, gm.EPI_F32, accumulate=True,
                           splitk="auto")
        native.check(kd.st_transpose_bf16(self.dGh.data_ptr(), GATES, self.dGhT.data_ptr(), RS, RS, GATES, sh), "T dGh")
        native.check(kd.st_transpose_bf16(self.dGx.data_ptr(), GATES, self.dGxT.data_ptr(), RS, RS, GATES, sh), "T dGx")
        native.check(kd.st_transpose_bf16(self.Hm.data_ptr(), HID, self.HT.data_ptr(), R1, RS, HID, sh), "T H")
        native.check(kd.st_transpose_bf16(self.X.data_ptr(), XL, self.XT.data_ptr(), R1, RS, XL, sh), "T X")
        gm.gemm_nt(self.dGhT, self.HT[:, :RS], self.dP["w_hh"], gm.EPI_F32, accumulate=True, splitk="auto")
        gm.gemm_nt(self.dGxT, self.XT[:, :RS], self.dP["w_ih"], gm.EPI_F32, accumulate=True, splitk="auto")
        native.check(kd.st_row_sum_bf16(self.dGxT.data_ptr(), RS, GATES, RS, self.dP["b_ih"].data_ptr(), sh), "db_ih")
        native.check(kd.st_row_sum_bf16(self.dGhT.data_ptr(), RS, GATES, RS, self.dP["b_hh"].data_ptr(), sh), "db_hh")
        native.check(k.st_gru_wq_grad(self.dQ.data_ptr(), self.Hq.data_ptr(), RS, self.dP["w_q"].data_ptr(),
                                      self.dP["b_q"].data_ptr(), sh), "dWq")
        if self.grad_sync is not None:
            self.grad_sync(self.gflat)
        for ad in self._adam:
            native.check(kd.st_adam_tile(ad, sh), "adam")
        native.check(kd.st_counter_inc(self.t_ctr.data_ptr(), sh), "t++")
        self.pack()

    def sync_target(self) -> None:
        self.tgt["w_ih"].copy_(self.Wih_b)
        self.tgt["w_hh"].copy_(self.Whh_b)
        for n in ("b_ih", "b_hh", "w_q", "b_q"):
            self.tgt[n].copy_(self.P[n])

    # ---------------------------------------------------------------- driver
    def capture(self) -> None:
        """Warm up, then capture one actor launch and one learner update into HIP graphs."""
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self.act()
            self.update()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        self.launches += 1
        self.updates += 1
        self._g_act = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_act):
            self.act()
        self._g_upd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_upd):
            self.update()

    def act_step(self) -> None:
        if self._g_act is not None:
            self._g_act.replay()
        else:
            self.act()
        self.launches += 1

    def update_step(self) -> None:
        if self._g_upd is not None:
            self._g_upd.replay()
        else:
            self.update()
        self.updates += 1
        if self.updates % self.target_every == 0:
            self.sync_target()

    def iteration(self, updates: int = 1) -> None:
        self.act_step()
        for _ in range(updates):
            self.update_step()

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
