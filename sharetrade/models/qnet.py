"""Q-network: flat parameter layout, initialisation and a plain-PyTorch oracle.

Reference graph (`QDecisionPolicyActor.scala:38-50`)::

    x:[?,203] -> relu(x W1 + b1) [200] -> relu(h1 W2 + b2) [3]      (output ReLU = quirk Q3)
    loss = (y - q)^2 ; AdaGrad(0.01).minimize(loss)                 (biases are tf.constant, Q4)

Here the network is a general MLP (``ModelConfig.hidden`` = list of widths).
Parameters live in ONE flat fp32 buffer laid out exactly as the HIP kernels
consume them (so the optimizer, the RCCL gradient all-reduce and the
checkpoint writer all see a single contiguous tensor):

* every weight is stored transposed, ``W^T[out_p][in_p]`` row-major, so a
  16x16x32 MFMA A-fragment (8 consecutive k of one row) is one 16-byte load;
* ``in_p`` of layer 0 is ``round_up(input_dim + 1, 32)``: column ``input_dim``
  (203) is a constant-1 feature, so layer-0's bias lives in that column of
  ``W0^T`` and the fused kernel needs no separate bias path for it;
* hidden widths are padded to multiples of 32 (MFMA K granularity), the action
  dimension to 16; every pad entry is zero and stays zero (its gradient is 0);
* later layers carry an explicit bias vector ``b_l[out_p]``.

The oracle functions below (forward / backward / optimizers) are the fp32
references that every HIP kernel test compares against.  ``emulate_bf16``
rounds at exactly the points where the fused bf16 kernel rounds.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..config import ModelConfig

OUT_PAD = 16
SEG_ALIGN = 64  # elements (256 B for fp32, 128 B for bf16)


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class Segment:
    name: str
    offset: int
    shape: Tuple[int, ...]

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


class QNetLayout:
    """Flat-buffer layout of an MLP Q-network (see module docstring)."""

    def __init__(self, input_dim: int, hidden: Sequence[int], n_actions: int = 3):
        self.input_dim = int(input_dim)
        self.hidden = [int(h) for h in hidden]
        self.n_actions = int(n_actions)
        self.bias_col = self.input_dim  # constant-1 feature index in layer 0
        dims = [self.input_dim] + self.hidden + [self.n_actions]
        pdims = [round_up(self.input_dim + 1, 32)] + [round_up(h, 32) for h in self.hidden] + [OUT_PAD]
        self.dims = dims
        self.pdims = pdims
        self.n_layers = len(dims) - 1
        self.segments: Dict[str, Segment] = {}
        off = 0
        for l in range(self.n_layers):
            shp = (pdims[l + 1], pdims[l])
            self.segments[f"W{l}"] = Segment(f"W{l}", off, shp)
            off = round_up(off + shp[0] * shp[1], SEG_ALIGN)
            if l > 0:
                self.segments[f"b{l}"] = Segment(f"b{l}", off, (pdims[l + 1],))
                off = round_up(off + pdims[l + 1], SEG_ALIGN)
        self.numel = off

    @classmethod
    def from_config(cls, m: ModelConfig) -> "QNetLayout":
        return cls(m.input_dim, m.hidden, m.n_actions)

    @property
    def in_p(self) -> int:
        return self.pdims[0]

    def n_real_params(self) -> int:
        n = 0
        for l in range(self.n_layers):
            n += self.dims[l] * self.dims[l + 1] + self.dims[l + 1]
        return n

    # ----------------------------------------------------------- views
    def w(self, flat: torch.Tensor, l: int) -> torch.Tensor:
        s = self.segments[f"W{l}"]
        return flat[s.offset:s.offset + s.numel].view(*s.shape)

    def b(self, flat: torch.Tensor, l: int) -> torch.Tensor:
        """Bias of layer ``l`` (a view; layer 0's bias is a column of W0^T)."""
        if l == 0:
            return self.w(flat, 0)[:, self.bias_col]
        s = self.segments[f"b{l}"]
        return flat[s.offset:s.offset + s.numel]

    def describe(self) -> Dict[str, object]:
        return {
            "dims": self.dims,
            "padded_dims": self.pdims,
            "numel": self.numel,
            "segments": {k: (v.offset, v.shape) for k, v in self.segments.items()},
        }

    # ----------------------------------------------------------- masks
    def trainable_mask(self, train_bias: bool) -> torch.Tensor:
        m = torch.zeros(self.numel, dtype=torch.float32)
        for l in range(self.n_layers):
            wl = self.w(m, l)
            wl[: self.dims[l + 1], : self.dims[l]] = 1.0
            if train_bias:
                self.b(m, l)[: self.dims[l + 1]] = 1.0
        return m


def philox_normal(rows: int, cols: int, std: float, seed: int, stream: int) -> torch.Tensor:
    """Host mirror of ``csrc/series.hip: init_normal_kernel``: element (r, c) = std * Box-Muller normal
    of Philox4x32-10 counter (r * cols + c, 0, stream, 0x1417), fp32 arithmetic (values agree with the
    device to a few ulps: libm vs device transcendentals)."""
    import numpy as np

    from ..utils import rng

    k0, k1 = rng.key_for(seed, 0)
    n = rows * cols
    i = np.arange(n, dtype=np.uint64)
    r0, r1, _, _ = rng.philox4x32((i & np.uint64(0xFFFFFFFF)).astype(np.uint32), np.zeros(n, np.uint32),
                                  np.full(n, stream, np.uint32), np.full(n, 0x1417, np.uint32),
                                  np.full(n, k0, np.uint32), np.full(n, k1, np.uint32))
    u1 = ((r0 >> np.uint32(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)
    u2 = rng.u24(r1)
    z = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.283185307179586) * u2)
    return torch.from_numpy((np.float32(std) * z.astype(np.float32)).reshape(rows, cols))


def init_params(layout: QNetLayout, m: ModelConfig, seed: int = 0, device=None,
                host_mirror: bool = False) -> torch.Tensor:
    """fp32 flat params; ``W ~ N(0, init_std)`` (tf.RandomNormalInitializer,
    QDecisionPolicyActor.scala:41,45) or He-normal; biases = ``bias_init``.

    ``m.init_rng``: ``"philox"`` (default) draws W from the counter-based Philox + Box-Muller
    generator: by the ``init_normal`` HIP kernel (csrc/series.hip) whenever a GPU and the native library
    are present -- also for a host-side ``device`` (drawn on the GPU, copied over), so a host learner
    (PolicyServer, serve_eval) and a device engine get bit-identical weights for one seed -- and by its
    NumPy mirror on a machine without a GPU (the same values up to libm ulps: logf / cosf vs NumPy).
    ``"torch"`` uses torch's CPU generator and reproduces the seeded runs of rounds 1-2.  The result
    lives on ``device`` (CPU by default).  ``host_mirror``: always draw with the NumPy mirror (tests pin
    the mirror against the kernel with it, since a GPU-less host relies on the mirror)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    flat = torch.zeros(layout.numel, dtype=torch.float32, device=dev)
    kdev = _kernel_device(dev) if (m.init_rng == "philox" and not host_mirror) else None
    use_kernel = kdev is not None
    if use_kernel:
        from ..ops import native
        from ..utils import rng

        k0, k1 = rng.key_for(int(seed), 0)
        out = flat
        flat = torch.zeros(layout.numel, dtype=torch.float32, device=kdev)
    g = torch.Generator().manual_seed(int(seed)) if m.init_rng == "torch" else None
    for l in range(layout.n_layers):
        fan_in, fan_out = layout.dims[l], layout.dims[l + 1]
        std = m.init_std if m.init == "normal" else math.sqrt(2.0 / fan_in)
        wl = layout.w(flat, l)
        if use_kernel:
            native.init_normal(wl, fan_out, fan_in, float(std), int(k0), int(k1), l)
        elif m.init_rng == "philox":
            wl[:fan_out, :fan_in] = philox_normal(fan_out, fan_in, std, seed, l).to(dev)
        elif m.init_rng == "torch":
            wl[:fan_out, :fan_in] = (torch.randn(fan_out, fan_in, generator=g) * std).to(dev)
        else:
            raise KeyError(f"model.init_rng: {m.init_rng!r}")
        layout.b(flat, l)[:fan_out] = m.bias_init
    if use_kernel and out.device != flat.device:
        out.copy_(flat)
        return out
    return flat


def _kernel_device(dev: torch.device):
    """Where the init_normal kernel draws for ``dev``: ``dev`` itself if it is a GPU, the current GPU
    when ``dev`` is the host and a GPU plus the native library exist, else None (NumPy mirror)."""
    if dev.type == "cuda":
        return dev
    try:
        # torch.cuda first: on a machine without a GPU, loading the HIP library (native.available()) starts
        # runtime threads that slowed the CPU actor runtime ~3x
        if torch.cuda.is_available():
            from ..ops import native

            if native.available():
                return torch.device("cuda", torch.cuda.current_device())
    except Exception:  # noqa: BLE001 -- no usable GPU: host mirror
        pass
    return None


# ---------------------------------------------------------------- oracle
def _bf(x: torch.Tensor, on: bool) -> torch.Tensor:
    return x.to(torch.bfloat16).float() if on else x


def pad_input(layout: QNetLayout, x: torch.Tensor) -> torch.Tensor:
    """[B, input_dim] -> [B, in_p] with the constant-1 bias column."""
    B = x.shape[0]
    xp = torch.zeros(B, layout.in_p, dtype=torch.float32, device=x.device)
    xp[:, : layout.input_dim] = x
    xp[:, layout.bias_col] = 1.0
    return xp


def forward(flat: torch.Tensor, layout: QNetLayout, x: torch.Tensor, output_relu: bool,
            emulate_bf16: bool = False) -> Tuple[torch.Tensor, List[torch.Tensor], torch.Tensor]:
    """Returns ``(q_padded [B, 16], acts, xpad)``; ``acts[l]`` is the (post-ReLU)
    input of layer ``l+1`` at the precision the kernel keeps it."""
    xp = _bf(pad_input(layout, x), emulate_bf16)
    a = xp
    acts: List[torch.Tensor] = []
    for l in range(layout.n_layers):
        w = _bf(layout.w(flat, l), emulate_bf16)
        z = a @ w.t()
        if l > 0:
            z = z + layout.b(flat, l)
        last = l == layout.n_layers - 1
        if not last:
            a = _bf(torch.relu(z), emulate_bf16)
            acts.append(a)
        else:
            q = torch.relu(z) if output_relu else z
    return q, acts, xp


def backward(flat: torch.Tensor, layout: QNetLayout, xp: torch.Tensor, acts: List[torch.Tensor],
             q: torch.Tensor, dq: torch.Tensor, output_relu: bool,
             emulate_bf16: bool = False) -> torch.Tensor:
    """Gradient (flat, fp32) of ``sum(dq * q)`` w.r.t. the parameters.

    ``dq`` is [B, 16] (already containing the loss scale).  With the output
    ReLU the gradient is masked by ``q > 0`` (ReluGrad)."""
    grad = torch.zeros_like(flat)
    dz = dq * (q > 0).float() if output_relu else dq
    dz = _bf(dz, emulate_bf16)
    ins = [xp] + acts
    for l in reversed(range(layout.n_layers)):
        a_in = ins[l]
        layout.w(grad, l).copy_(dz.t() @ a_in)
        if l > 0:
            layout.b(grad, l).copy_(dz.sum(0))
            w = _bf(layout.w(flat, l), emulate_bf16)
            dh = dz @ w
            dz = _bf(dh * (a_in > 0).float(), emulate_bf16)
    return grad


# ------------------------------------------------------------- optimizers
class OptimState:
    """Optimizer state for the flat parameter buffer (same layout)."""

    def __init__(self, kind: str, numel: int, init_acc: float = 0.1, device=None):
        self.kind = kind
        self.t = 0
        dev = device if device is not None else "cpu"
        if kind == "adagrad":
            self.s1 = torch.full((numel,), float(init_acc), dtype=torch.float32, device=dev)
            self.s2 = torch.zeros(0, dtype=torch.float32, device=dev)
        elif kind == "adam":
            self.s1 = torch.zeros(numel, dtype=torch.float32, device=dev)
            self.s2 = torch.zeros(numel, dtype=torch.float32, device=dev)
        elif kind == "sgd":
            self.s1 = torch.zeros(0, dtype=torch.float32, device=dev)
            self.s2 = torch.zeros(0, dtype=torch.float32, device=dev)
        else:
            raise KeyError(f"unknown optimizer {kind}")

    def to(self, device) -> "OptimState":
        self.s1 = self.s1.to(device)
        self.s2 = self.s2.to(device)
        return self


def optimizer_step_ref(params: torch.Tensor, grad: torch.Tensor, st: OptimState, mask: torch.Tensor,
                       lr: float, betas=(0.9, 0.999), eps: float = 1e-8) -> None:
    """In-place reference update.

    AdaGrad follows TF's ApplyAdagrad (``acc += g^2; w -= lr * g / sqrt(acc)``),
    the op `tf.train.AdaGrad(0.01).minimize` emits (QDecisionPolicyActor.scala:50)."""
    g = grad * mask
    st.t += 1
    if st.kind == "adagrad":
        st.s1 += g * g
        params -= lr * g / torch.sqrt(st.s1)
    elif st.kind == "adam":
        b1, b2 = betas
        st.s1.mul_(b1).add_((1 - b1) * g)
        st.s2.mul_(b2).add_((1 - b2) * g * g)
        c1 = 1 - b1 ** st.t
        c2 = 1 - b2 ** st.t
        params -= lr * (st.s1 / c1) / (torch.sqrt(st.s2 / c2) + eps) * mask
    else:
        params -= lr * g
