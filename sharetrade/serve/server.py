"""Policy serving: many concurrent ``SelectionAction`` clients -> one batched GPU launch.

The reference serialises every decision through one actor mailbox and one TF session run
(``QDecisionPolicyActor.scala:52-62``; 10 workers x 5,846 steps of blocking ``ask``s,
``TrainerChildActor.scala:93``).  :class:`PolicyServer` keeps the trained flagship Q-net resident
on the GPU and answers request batches with one ``csrc/qserve.hip`` launch;
:class:`DynamicBatcher` collects single requests from any number of client threads into those
batches (up to ``max_batch`` rows, or whatever arrived within ``max_delay_us`` of the first one),
through pinned host staging buffers: one host->device copy, one launch, one device->host copy per
batch.

Weights can be swapped while serving (:meth:`PolicyServer.load_params`, e.g. from a running
``VectorEngine`` or a checkpoint); a batch always sees one consistent weight set.
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..config import Config, preset_config
from ..env import trading as tr
from ..models import qnet as qn
from ..utils import rng
from . import kernel as K

ArrayLike = Union[torch.Tensor, np.ndarray, Sequence[float]]


class PolicyServer:
    """Batched greedy / epsilon-greedy action selection for the flagship 2x128 Q-net.

    ``backend``: ``"native"`` (the HIP kernel; needs a GPU and raises if the library is missing),
    ``"torch"`` (the fp32 oracle with bf16 rounding emulated: CPU tests) or ``"auto"``.
    """

    def __init__(self, cfg: Optional[Config] = None, params: Optional[torch.Tensor] = None,
                 device: Optional[torch.device] = None, backend: str = "auto", seed: Optional[int] = None):
        self.cfg = cfg or preset_config("flagship")
        m, a = self.cfg.model, self.cfg.agent
        self.layout = qn.QNetLayout.from_config(m)
        self.H = m.history
        # request rows are staged at a 16-byte-aligned stride: the kernel's dwordx4 gather path
        self.ld = (self.H + 2 + 3) // 4 * 4
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
                torch.device("cpu")
        self.device = device
        if backend == "auto":
            backend = "native" if device.type == "cuda" else "torch"
        if backend not in ("native", "torch"):
            raise ValueError(f"backend: {backend!r}")
        if backend == "native" and device.type != "cuda":
            raise ValueError("the native serving backend needs a GPU device")
        self.backend = backend
        self.seed = int(a.seed if seed is None else seed)
        self.key = tuple(int(x) for x in rng.key_for(self.seed, 0))
        self.params = torch.zeros(self.layout.numel, dtype=torch.float32, device=device)
        self.params_bf = torch.zeros(self.layout.numel, dtype=torch.bfloat16, device=device)
        self._lock = threading.Lock()      # one weight set per batch
        self.seq = 0                       # draws of batch n use counter (row, n, 2)
        self.batches = 0
        self.requests = 0
        self._kern = None
        if backend == "native":
            self._kern = K.ServeKernel(self.layout, self.params, self.params_bf, history=self.H,
                                       feat_mode=tr.FEATURES[self.cfg.env.features], output_relu=m.output_relu,
                                       budget0=self.cfg.env.budget, epsilon=a.epsilon, ramp=a.ramp, key=self.key)
        self.load_params(params if params is not None else qn.init_params(self.layout, m, seed=a.seed))

    # ---------------------------------------------------------------- weights
    def load_params(self, flat: torch.Tensor) -> None:
        """Replace the served weights (fp32 flat params in the engine layout; copied)."""
        flat = flat.detach().float().reshape(-1)
        if flat.numel() != self.layout.numel:
            raise ValueError(f"expected {self.layout.numel} flat params, got {flat.numel()}")
        with self._lock:
            if self.device.type == "cuda":
                # launches already queued (any stream: the batcher has its own) still read the old set
                torch.cuda.synchronize(self.device)
            self.params.copy_(flat.to(self.device))
            self.params_bf.copy_(self.params.to(torch.bfloat16))
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()

    @classmethod
    def from_engine(cls, engine, backend: str = "auto", averaged: bool = True) -> "PolicyServer":
        """Serve a ``VectorEngine``'s weights (same config, same device): its Polyak average when it keeps
        one (``engine.ema_decay > 0``) and ``averaged``, else the live parameters."""
        w = engine.serving_params if averaged else engine.params
        return cls(engine.cfg, params=w, device=engine.device, backend=backend)

    # ---------------------------------------------------------------- inference
    def _rows(self, states: ArrayLike) -> torch.Tensor:
        x = torch.as_tensor(states, dtype=torch.float32)
        if x.dim() == 1:
            x = x.view(1, -1)
        if x.dim() != 2 or x.shape[1] != self.H + 2:
            raise ValueError(f"request rows must be [B, {self.H + 2}] (prices, budget, shares), got {tuple(x.shape)}")
        return x

    def infer(self, states: ArrayLike, steps: Optional[ArrayLike] = None,
              return_q: bool = False) -> Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        """Actions (int32 [B], on the server's device) for request rows [B, H+2]; ``steps`` (the
        ``SelectionAction`` step of each row) turns on the epsilon-greedy draw, None = greedy."""
        x = self._rows(states)
        if self.backend == "native":
            xd = torch.empty(x.shape[0], self.ld, dtype=torch.float32, device=self.device)
            xd[:, : self.H + 2].copy_(x, non_blocking=True)
            x = xd
        else:
            x = x.to(self.device)
        st = None if steps is None else torch.as_tensor(steps, dtype=torch.float32).reshape(-1).to(self.device)
        if st is not None and st.numel() != x.shape[0]:
            raise ValueError("one step per request row")
        with self._lock:
            seq = self.seq
            self.seq += 1
            self.batches += 1
            self.requests += int(x.shape[0])
            if self.backend == "native":
                acts = torch.empty(x.shape[0], dtype=torch.int32, device=self.device)
                q = torch.empty(x.shape[0], 3, dtype=torch.float32, device=self.device) if return_q else None
                self._kern.launch(x, acts, q, st, seq=seq)
            else:
                acts, q = self._torch_select(x, st, seq)
        return (acts, q) if return_q else acts

    def _torch_select(self, x: torch.Tensor, st: Optional[torch.Tensor], seq: int):
        c, m, a = self.cfg, self.cfg.model, self.cfg.agent
        return K.reference_select(self.params, self.layout, x, history=self.H, feat_mode=c.env.features,
                                  output_relu=m.output_relu, budget0=c.env.budget, epsilon=a.epsilon,
                                  ramp=a.ramp, key_seed=self.seed, seq=seq, steps=st)

    def launch_into(self, x: torch.Tensor, acts: torch.Tensor, steps: Optional[torch.Tensor], seq: int,
                    q: Optional[torch.Tensor] = None) -> None:
        """Native launch on preallocated device buffers (the batcher's path; no allocation)."""
        with self._lock:
            self.batches += 1
            self.requests += int(x.shape[0])
            self._kern.launch(x, acts, q, steps, seq=seq)


class DynamicBatcher:
    """Collects single ``(state, step)`` requests from client threads into server batches.

    ``submit`` returns a ``Future`` resolving to the action index (0 Buy, 1 Sell, 2 Hold).  A batch
    closes at ``max_batch`` requests or ``max_delay_us`` after its first request.  The native path
    stages rows in pinned host memory and reuses device buffers sized for ``max_batch``.
    """

    def __init__(self, server: PolicyServer, max_batch: int = 4096, max_delay_us: float = 200.0,
                 greedy: bool = False):
        self.server = server
        self.max_batch = int(max_batch)
        self.max_delay = float(max_delay_us) * 1e-6
        self.greedy = greedy
        self._cv = threading.Condition()
        self._q: List[Tuple[np.ndarray, float, Future]] = []
        self._stop = False
        self.batch_sizes: List[int] = []
        W = server.ld   # aligned row stride (the first H + 2 values of a row are the request)
        self._native = server.backend == "native"
        if self._native:
            dev = server.device
            self._h_x = torch.zeros(self.max_batch, W, dtype=torch.float32, pin_memory=True)
            self._h_s = torch.empty(self.max_batch, dtype=torch.float32, pin_memory=True)
            self._h_a = torch.empty(self.max_batch, dtype=torch.int32, pin_memory=True)
            self._d_x = torch.empty(self.max_batch, W, dtype=torch.float32, device=dev)
            self._d_s = torch.empty(self.max_batch, dtype=torch.float32, device=dev)
            self._d_a = torch.empty(self.max_batch, dtype=torch.int32, device=dev)
            self._stream = torch.cuda.Stream(dev)
        self._thread = threading.Thread(target=self._loop, name="sharetrade-serve-batcher", daemon=True)
        self._thread.start()

    def submit(self, state: ArrayLike, step: float = 0.0) -> Future:
        row = np.asarray(state.cpu() if isinstance(state, torch.Tensor) else state, dtype=np.float32).reshape(-1)
        if row.size != self.server.H + 2:
            raise ValueError(f"a request row holds {self.server.H + 2} values, got {row.size}")
        fut: Future = Future()
        with self._cv:
            if self._stop:
                raise RuntimeError("batcher is closed")
            self._q.append((row, float(step), fut))
            self._cv.notify()
        return fut

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join()

    def __enter__(self) -> "DynamicBatcher":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def _take(self) -> List[Tuple[np.ndarray, float, Future]]:
        with self._cv:
            while not self._q and not self._stop:
                self._cv.wait()
            if not self._q:
                return []
            deadline = time.perf_counter() + self.max_delay
            while len(self._q) < self.max_batch and not self._stop:
                left = deadline - time.perf_counter()
                if left <= 0:
                    break
                self._cv.wait(left)
            batch, self._q = self._q[: self.max_batch], self._q[self.max_batch:]
            return batch

    def _loop(self) -> None:
        while True:
            batch = self._take()
            if not batch:
                return
            try:
                acts = self._run(batch)
            except BaseException as e:  # noqa: BLE001 -- every waiting client gets the error
                for _, _, f in batch:
                    f.set_exception(e)
                continue
            self.batch_sizes.append(len(batch))
            for (_, _, f), a in zip(batch, acts):
                f.set_result(int(a))

    def _run(self, batch) -> np.ndarray:
        n = len(batch)
        X = np.stack([b[0] for b in batch])
        S = np.asarray([b[1] for b in batch], dtype=np.float32)
        if not self._native:
            return self.server.infer(X, None if self.greedy else S).cpu().numpy()
        srv = self.server
        with srv._lock:
            seq = srv.seq
            srv.seq += 1
        self._h_x[:n, : X.shape[1]].numpy()[:] = X
        self._h_s[:n].numpy()[:] = S
        with torch.cuda.stream(self._stream):
            self._d_x[:n].copy_(self._h_x[:n], non_blocking=True)
            self._d_s[:n].copy_(self._h_s[:n], non_blocking=True)
            srv.launch_into(self._d_x[:n], self._d_a, None if self.greedy else self._d_s, seq)
            self._h_a[:n].copy_(self._d_a[:n], non_blocking=True)
        self._stream.synchronize()
        return self._h_a[:n].numpy().copy()

    def stats(self) -> Dict[str, float]:
        bs = self.batch_sizes
        return {"batches": len(bs), "requests": int(sum(bs)), "mean_batch": float(np.mean(bs)) if bs else 0.0,
                "max_batch": int(max(bs)) if bs else 0}
