"""GRU(256) recurrent Q-net (BASELINE config 5): MX-fp8 actor + bf16 learner vs PyTorch references."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(eps=0.9):
    from sharetrade.config import preset_config

    cfg = preset_config("recurrent")
    cfg.agent.epsilon = eps
    return cfg


def test_mx_probe_layout(native_built):
    """v_mfma_scale_f32_16x16x128_f8f6f4: lane l = i + 16q holds row/col i, K 16q+[0,16) and 64+16q+[0,16);
    the scale of (row i, K-block s) comes from lane i + 16s (tools/mx_layout_probe.py)."""
    from sharetrade.ops.gru import mx_probe

    g = torch.Generator().manual_seed(0)
    vals = torch.randint(-8, 9, (2, 64, 32), generator=g).float() * 0.25      # exact in e4m3
    a8 = vals[0].to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    b8 = vals[1].to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    sa = torch.randint(124, 131, (64,), generator=g, dtype=torch.int32)
    sb = torch.randint(124, 131, (64,), generator=g, dtype=torch.int32)
    D = mx_probe(a8, b8, sa.cuda(), sb.cuda()).cpu()
    A = torch.zeros(16, 128)
    Bm = torch.zeros(16, 128)
    for l in range(64):
        i, q = l & 15, l >> 4
        for half, k0 in ((0, 16 * q), (1, 64 + 16 * q)):
            A[i, k0:k0 + 16] = vals[0, l, 16 * half:16 * half + 16] * 2.0 ** (int(sa[i + 16 * (k0 // 32)]) - 127)
            Bm[i, k0:k0 + 16] = vals[1, l, 16 * half:16 * half + 16] * 2.0 ** (int(sb[i + 16 * (k0 // 32)]) - 127)
    ref = A.double() @ Bm.double().t()
    assert torch.allclose(D.double(), ref, rtol=1e-6, atol=1e-6), (D - ref).abs().max()


def test_minute_bars_gpu_matches_numpy(native_built):
    from sharetrade.data import minute_bars as mb

    close, feat = mb.generate_gpu(64, 300, torch.device("cuda", 0), seed=3)
    c_np, f_np = mb.generate_numpy(64, 300, seed=3)
    torch.cuda.synchronize()
    rel = np.abs(close.cpu().numpy() - c_np) / c_np
    assert rel.max() < 1e-4, rel.max()
    f = feat.float().cpu().numpy()
    assert np.allclose(f, f_np, rtol=2e-2, atol=2e-2)


def _small(E=64, S=4, eps=0.9, **kw):
    from sharetrade.trainer.recurrent import RecurrentDQN

    kw.setdefault("bars", 600)
    kw.setdefault("ep_len", 5)
    kw.setdefault("batch", 128)
    kw.setdefault("replay_segments", 1024)
    return RecurrentDQN(_cfg(eps), torch.device("cuda", 0), envs=E, seq=S, burn_in=1, **kw)


def test_pack_is_exact_mx_quantization(native_built):
    from sharetrade.ops.gru import gate_prescale, mx_roundtrip, unpack_whh

    d = _small()
    torch.cuda.synchronize()
    W = d.P["w_hh"].cpu()
    Ws = W * gate_prescale()[:, None]          # the gate pre-scale, applied in fp32 before quantization
    raw = unpack_whh(d.whh8, d.whhs, unscale=False)
    assert torch.equal(raw, mx_roundtrip(Ws))  # 32-element blocks along K, same scale rule as the kernel
    assert torch.allclose(unpack_whh(d.whh8, d.whhs), W, rtol=0.07, atol=1e-6)


def _ref_actor(d, steps, eps_exploit):
    """Host replay of one actor launch: env in float32 (bit-exact), GRU in fp32 with the
    actor's quantization points (MX-fp8 W_hh and h, bf16 W_ih and x)."""
    from sharetrade.env import minute as me
    from sharetrade.ops.gru import gate_prescale, mx_roundtrip, unpack_whh
    from sharetrade.utils import rng

    E, S, T = d.E, d.S, d.T
    Whh = unpack_whh(d.whh8, d.whhs).double()
    gs = gate_prescale()
    # the actor's bf16 W_ih rows carry the gate pre-scale (rounded after scaling): undo it in double
    Wih = (d.P["w_ih"].cpu()[:, :32] * gs[:, None]).to(torch.bfloat16).double() / gs.double()[:, None]
    b_ih, b_hh = d.P["b_ih"].cpu().view(-1).double(), d.P["b_hh"].cpu().view(-1).double()
    Wq, bq = d.P["w_q"].cpu().double(), d.P["b_q"].cpu().view(-1).double()
    close = d.close.cpu().numpy()
    ret = d.ret.cpu().numpy()
    feat = d.feat.float().cpu().numpy()
    k0, k1 = rng.key_for(d.seed, 5)
    pos, es = d.pos.cpu().numpy(), d.ep_start.cpu().numpy()
    states = [me.MinuteEnvState(int(pos[e]), int(es[e])) for e in range(E)]
    h = torch.zeros(E, 256, dtype=torch.float64)
    xs, acts, rews, dones, qs = [], [], [], [], []
    x = torch.tensor(np.stack([me.obs(feat[e, states[e].t], close[e, states[e].t], states[e], d.ep_len)
                               for e in range(E)])).to(torch.bfloat16).double()
    xs.append(x)
    for s in range(S):
        hq = mx_roundtrip(h.float()).double()
        gx = x @ Wih.t() + b_ih
        gh = hq @ Whh.t() + b_hh
        r = torch.sigmoid(gx[:, :256] + gh[:, :256])
        z = torch.sigmoid(gx[:, 256:512] + gh[:, 256:512])
        n = torch.tanh(gx[:, 512:] + r * gh[:, 512:])
        h = (1 - z) * n + z * h
        q = h @ Wq.t() + bq
        qs.append(q)
        a_s, r_s, d_s, xn = [], [], [], []
        for e in range(E):
            gstep = s + int(d.ctrl[0]) * S
            u_exp, u_act, u_rst = me.draws(e, gstep, k0, k1)
            rnd = min(int(u_act * np.float32(3.0)), 2)
            exploit = u_exp < min(np.float32(eps_exploit), np.float32(gstep) * np.float32(1.0 / d.cfg.agent.ramp))
            a = int(torch.argmax(q[e])) if exploit else rnd
            rew, done, _ = me.step(states[e], a, close[e], ret[e], T, d.ep_len, d.cost, u_rst)
            a_s.append(a); r_s.append(rew); d_s.append(done)
            xn.append(me.obs(feat[e, states[e].t], close[e, states[e].t], states[e], d.ep_len))
            if done:
                h[e] = 0
        acts.append(a_s); rews.append(r_s); dones.append(d_s)
        x = torch.tensor(np.stack(xn)).to(torch.bfloat16).double()
        xs.append(x)
    return h, qs, acts, rews, dones, xs, states


@pytest.mark.parametrize("kernel", ["single", "pair"])
def test_actor_matches_reference(native_built, kernel):
    """eps = 0 -> every action is the Philox random draw, so env/replay must match bit for bit
    and the GRU state must match the quantization-aware fp32 reference."""
    d = _small(eps=0.0, actor_kernel=kernel)
    assert d.actor_kernel == kernel
    q_out = torch.zeros(d.E, 4, device="cuda")
    d._act.q_out = q_out.data_ptr()
    h_ref, qs, acts, rews, dones, xs, states = _ref_actor(d, d.S, 0.0)
    d.act()
    torch.cuda.synchronize()
    slots = np.arange(d.E)   # first launch: segment slot = env id
    ra = d.ra.cpu().numpy()[slots]
    rr = d.rr.cpu().numpy()[slots]
    rd = d.rd.cpu().numpy()[slots]
    assert np.array_equal(ra, np.array(acts).T)
    assert np.array_equal(rr, np.array(rews, dtype=np.float32).T)
    assert np.array_equal(rd.astype(bool), np.array(dones).T)
    rx = d.rx.cpu().float()[slots]
    for s in range(d.S + 1):
        assert torch.equal(rx[:, s].double(), xs[s]), s
    assert np.array_equal(d.pos.cpu().numpy(), np.array([st.t for st in states]))
    assert np.array_equal(d.position.cpu().numpy(), np.array([st.pz for st in states]))
    h = d.h.cpu().double()
    err = float((h - h_ref).abs().max())
    assert err < 3e-2, err
    assert float((h - h_ref).abs().mean()) < 2e-3
    qerr = float((q_out[:, :3].cpu().double() - qs[-1]).abs().max())
    assert qerr < 1e-2, qerr
    assert int(d.rctrl[0]) == d.E and int(d.ctrl[0]) == 1


def _ref_unroll(X, h0, p, D, Wdeq, Wbwd=None):
    """Quantization-aware reference of the fused learner: the VALUE of W_hh h is the MX-fp8 product
    (forward-packed W_hh, quantized h); the gradient w.r.t. h flows through the backward-packed
    MX-fp8 W_hh (``Wbwd``), the gradient w.r.t. W_hh through the bf16 master (straight-through)."""
    from sharetrade.ops.gru import mx_roundtrip

    h, qs = h0, []
    for t in range(X.shape[0]):
        gx = X[t][:, :32] @ p["w_ih"][:, :32].t() + p["b_ih"]
        gh_q = mx_roundtrip(h.detach()) @ Wdeq.t() + p["b_hh"]
        if Wbwd is None:
            gh = gh_q
        else:
            gh_h = h @ Wbwd.t()
            gh_w = h.detach() @ p["w_hh"].t() + p["b_hh"]
            gh = gh_q.detach() + (gh_h - gh_h.detach()) + (gh_w - gh_w.detach())
        r = torch.sigmoid(gx[:, :256] + gh[:, :256])
        z = torch.sigmoid(gx[:, 256:512] + gh[:, 256:512])
        n = torch.tanh(gx[:, 512:] + r * gh[:, 512:])
        h = (1 - z) * n + z * h
        qs.append(h @ p["w_q"].t() + p["b_q"])
        if t < D.shape[0]:
            h = h * (1 - D[t])[:, None]
    return torch.stack(qs)


def test_learner_gradients_match_autograd(native_built):
    from sharetrade.ops.gru import unpack_whh, unpack_whhT
    from sharetrade.utils import rng

    d = _small(E=128, S=4, eps=0.5, batch=128)
    for _ in range(3):
        d.act()
    P0 = {n: t.detach().clone().cpu() for n, t in d.P.items()}
    T0 = {n: t.detach().clone().cpu() for n, t in d.T_P.items()}
    W_on = unpack_whh(d.pk["on"]["whh8"], d.pk["on"]["whhs"])
    W_tg = unpack_whh(d.pk["tg"]["whh8"], d.pk["tg"]["whhs"])
    W_bwd = unpack_whhT(d.pk["on"]["whhT8"], d.pk["on"]["whhTs"])
    assert torch.allclose(W_bwd, P0["w_hh"], rtol=0.07, atol=1e-6)
    d.update()
    torch.cuda.synchronize()
    size = int(d.rctrl[1])
    k0, k1 = rng.key_for(d.seed, 7)
    b = np.arange(d.B, dtype=np.uint32)
    c0, c1, _, _ = rng.philox4x32(b, np.zeros_like(b), np.zeros_like(b), np.full_like(b, 0x53455131), k0, k1)
    idx = torch.from_numpy(((c0.astype(np.uint64) << np.uint64(32)) | c1.astype(np.uint64)) % np.uint64(size)).long()
    X = d.rx.cpu()[idx].float().transpose(0, 1)          # [S+1, B, 32]
    A = d.ra.cpu()[idx].long().t()
    R = d.rr.cpu()[idx].t()
    D = d.rd.cpu()[idx].float().t()
    h0 = d.rh0.cpu()[idx].float()
    bf = lambda t: t.to(torch.bfloat16).float()
    p = {"w_ih": bf(P0["w_ih"]).requires_grad_(True), "w_hh": bf(P0["w_hh"]).requires_grad_(True)}
    for n in ("b_ih", "b_hh", "w_q", "b_q"):
        p[n] = P0[n].view(P0[n].shape if n == "w_q" else (-1,)).clone().requires_grad_(True)
    pt = {"w_ih": bf(T0["w_ih"]), "w_hh": bf(T0["w_hh"]), "b_ih": T0["b_ih"].view(-1), "b_hh": T0["b_hh"].view(-1),
          "w_q": T0["w_q"], "b_q": T0["b_q"].view(-1)}
    q = _ref_unroll(X, h0, p, D, W_on, W_bwd)
    with torch.no_grad():
        qt = _ref_unroll(X, h0, pt, D, W_tg)
        a_star = q[1:].argmax(-1, keepdim=True)
        y = R + d.gamma * (1 - D) * qt[1:].gather(-1, a_star)[..., 0]
    qa = q[:d.S].gather(-1, A[..., None])[..., 0]
    loss = ((qa - y)[d.burn:] ** 2).mean()
    loss.backward()
    # forward values: online / target Q of the kernels vs the reference unroll
    assert torch.allclose(d.Q.cpu()[:, :3].view(d.S + 1, d.B, 3), q.detach(), atol=2e-3, rtol=2e-2)
    assert torch.allclose(d.Q_t.cpu()[:, :3].view(d.S + 1, d.B, 3), qt, atol=2e-3, rtol=2e-2)
    got_loss = float(d.loss) / (d.B * (d.S - d.burn))
    assert abs(got_loss - float(loss.detach())) < 3e-2 * float(loss.detach()) + 1e-7, (got_loss, float(loss))
    for n in ("w_ih", "w_hh", "b_ih", "b_hh", "w_q", "b_q"):
        ref = p[n].grad.view(-1)
        got = d.dP[n].cpu().view(-1)
        rel = float((got - ref).norm() / (ref.norm() + 1e-20))
        assert rel < 5e-2, (n, rel)


def test_graph_iterations_train(native_built):
    d = _small(E=256, S=8, eps=0.9, batch=256)
    for _ in range(2):
        d.act()
    d.capture()
    w0 = d.P["w_hh"].clone()
    for _ in range(6):
        d.iteration(1)
    torch.cuda.synchronize()
    s = d.stats_dict()
    assert s["updates"] == 7 and np.isfinite(s["loss"])
    assert s["episodes"] > 0 and np.isfinite(s["episode_return_mean"])
    assert torch.isfinite(d.flat).all() and not torch.equal(w0, d.P["w_hh"])
    assert int(d.t_ctr) == 7


def test_overlapped_actor_matches_same_order_serial(native_built):
    """overlap_act: the actor launch on its own stream beside the update (captured graph) equals the
    same operation order on one stream: identical env / replay state, parameters within fp32
    atomic-order noise."""
    res = []
    for serial in (False, True):
        d = _small(E=256, S=8, eps=0.9, batch=256, overlap_act=True)
        for _ in range(2):
            d.act()
        if serial:
            d._act_stream = torch.cuda.current_stream()   # same op order, one stream, eager
            for _ in range(4):
                d.iteration(1)
        else:
            d.capture()
            for _ in range(3):
                d.iteration(1)
        torch.cuda.synchronize()
        res.append(d)
    a, b = res
    assert a.updates == b.updates == 4 and a.launches == b.launches
    assert int(a.t_ctr) == int(b.t_ctr) == 4
    assert torch.equal(a.rctrl, b.rctrl)
    assert torch.equal(a.stats, b.stats) or torch.allclose(a.stats, b.stats, rtol=1e-6)
    rel = float((a.flat - b.flat).norm() / (b.flat.norm() + 1e-20))
    assert rel < 1e-5, rel


@pytest.mark.parametrize("E,grid", [(96, 1), (256, 3), (1024, 0)])
def test_pair_actor_bit_identical_to_single(native_built, E, grid):
    """gru_act_pair_kernel (two chunks per workgroup, env phase of one beside the MFMA phase of the
    other) == gru_act_kernel bit for bit over several launches with greedy actions: replay, env
    state and h.  E=96 has an odd chunk count (one workgroup's second slot is empty), grid=1 and 3
    loop a workgroup over several pairs."""
    res = []
    for kernel in ("single", "pair"):
        d = _small(E=E, S=8, eps=0.9, actor_kernel=kernel, actor_grid=grid, replay_segments=4 * E)
        q_out = torch.zeros(d.E, 4, device="cuda")
        d._act.q_out = q_out.data_ptr()
        for _ in range(3):
            d.act()
        torch.cuda.synchronize()
        res.append((d, q_out))
    (a, qa), (b, qb) = res
    for n in ("ra", "rr", "rd", "rx", "rh0", "h", "pos", "ep_start", "position", "entry", "ep_ret", "episodes",
              "last_ret", "rctrl", "ctrl"):
        x, y = getattr(a, n), getattr(b, n)
        if x.is_floating_point():                                     # bit patterns (last_ret starts NaN)
            bits = {2: torch.int16, 4: torch.int32}[x.element_size()]
            x, y = x.view(bits), y.view(bits)
        assert torch.equal(x, y), n
    assert torch.equal(qa, qb)
    assert torch.allclose(a.stats, b.stats, rtol=1e-5, atol=1e-5)   # fp32 atomics: per-pair partial sums
    assert int(b.episodes.sum()) > 0


def test_pair_actor_rejects_long_sequences(native_built):
    with pytest.raises(ValueError):
        _small(S=40, actor_kernel="pair", bars=800)
    assert _small(S=40, bars=800).actor_kernel == "single"


def test_k_iteration_graph_matches_single_iterations(native_built):
    """capture(iters_per_graph=4) + iterations(n): 4 whole overlapped iterations (alternating online sets)
    per graph launch, singles where a target copy would fall inside one -- the same sequence as single
    iteration replays: identical replay / env counters, parameters within fp32 atomic-order noise."""
    res = []
    for k in (4, 1):
        d = _small(E=256, S=8, eps=0.9, batch=256, overlap_act=True)
        d.target_every = 6
        for _ in range(2):
            d.act()
        d.capture(iters_per_graph=k)
        d.iterations(9)
        torch.cuda.synchronize()
        res.append(d)
    a, b = res
    assert a.updates == b.updates == 10 and a.launches == b.launches
    assert int(a.t_ctr) == int(b.t_ctr) == 10
    assert a._par == b._par
    assert torch.equal(a.rctrl, b.rctrl)
    rel = float((a.flat - b.flat).norm() / (b.flat.norm() + 1e-20))
    assert rel < 1e-5, rel
    relt = float((a.tflat - b.tflat).norm() / (b.tflat.norm() + 1e-20))
    assert relt < 1e-5, relt
