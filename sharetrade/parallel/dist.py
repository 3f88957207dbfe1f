"""Data parallelism over ``torch.distributed`` — RCCL over xGMI on MI355X, gloo on CPU.

The reference's only parallelism is the Akka router broadcasting ``Train`` to
10 rollout actors that share ONE learner mailbox (`TrainerRouterActor.scala:36,
60-66,86-88`): asynchronous, Hogwild-like online learning.  Its
multi-GPU analogue here is synchronous data parallelism, one process per GPU:

==========================  ==========================================  =============================
reference message pattern   here                                        collective
==========================  ==========================================  =============================
``router.route(Train(d))``  every rank starts from rank 0's weights     ``broadcast`` (params + opt)
``UpdateQ`` into one mailbox  local fused step -> ONE flat fp32 bucket   ``all_reduce(SUM)`` per step
``GetPortfolio`` ×N + mean  per-rank (n, Σx, Σx²)                       ``all_reduce(SUM)``
``Trained`` to the parent   done flags                                  ``all_reduce(MIN)``
==========================  ==========================================  =============================

Sizing for xGMI (point-to-point, 7 links x ~153 GB/s per GPU): the 2x128 net's
gradient is 47 k fp32 = 189 KB, so a step's all-reduce is latency-bound (one
fused call, no bucketing); the 4x1024 net's 13.4 MB bucket is split into
``bucket_mb`` chunks so RCCL can pipeline them across rings.
"""
from __future__ import annotations

import datetime
import math
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    group: Optional[object] = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_rank() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: Optional[str] = None, device: Optional[str] = None, timeout_s: float = 600.0) -> DistContext:
    """Initialise from the torchrun environment (RANK / WORLD_SIZE / MASTER_*).

    ``backend=None`` picks ``nccl`` (= RCCL on ROCm) when a GPU is present,
    else ``gloo``.  One process per GPU: the process binds ``cuda:LOCAL_RANK``."""
    rank, world, local = env_rank()
    use_gpu = (device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
    if use_gpu:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world <= 1:
        return DistContext(rank, world, local, "none", dev, None)
    be = backend or ("nccl" if use_gpu else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
    if be == "nccl":
        kw["device_id"] = dev
    if not dist.is_initialized():
        dist.init_process_group(**kw)
    return DistContext(rank, world, local, be, dev, dist.group.WORLD)


def shutdown(ctx: Optional[DistContext] = None) -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


class GradSync:
    """Flat-bucket gradient all-reduce.

    The parameter layout is one contiguous buffer (sharetrade/models/qnet.py), so
    the whole gradient is ONE tensor; it is reduced in ``bucket_mb`` slices
    (a single call below the threshold).  ``average=False`` because the engine
    pre-scales the loss by 1/(global batch); ``compress="bf16"`` halves the bytes
    on the wire for the large configs (fp32 accumulate on both ends)."""

    def __init__(self, ctx: DistContext, numel: int, bucket_mb: float = 4.0, compress: Optional[str] = None):
        self.ctx = ctx
        self.numel = numel
        self.compress = compress
        elem = 2 if compress == "bf16" else 4
        per = max(1, int(bucket_mb * 1024 * 1024 // elem))
        self.slices = [(o, min(numel, o + per)) for o in range(0, numel, per)]
        self._wire: Optional[torch.Tensor] = None
        self.calls = 0
        self.timing = False
        self._events = []        # (start, end) CUDA events of timed calls, or (t0, t1) host seconds
        self._timed_ms = 0.0
        self._timed_n = 0

    def enable_timing(self, on: bool = True) -> None:
        """Record the wall time of every all-reduce on the stream (metrics ``allreduce_ms``)."""
        self.timing = on

    def pop_timing_ms(self) -> Optional[float]:
        """Mean all-reduce time (ms) over the calls since the last pop; synchronizes recorded events."""
        for a, b in self._events:
            if isinstance(a, float):
                self._timed_ms += (b - a) * 1e3
            else:
                b.synchronize()
                self._timed_ms += a.elapsed_time(b)
            self._timed_n += 1
        self._events = []
        if self._timed_n == 0:
            return None
        m = self._timed_ms / self._timed_n
        self._timed_ms, self._timed_n = 0.0, 0
        return m

    def all_reduce(self, grad: torch.Tensor, async_op: bool = False):
        if not self.ctx.is_distributed:
            return None
        if self.timing and not async_op:
            if grad.is_cuda:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                self._all_reduce(grad, False)
                b.record()
            else:
                a = time.perf_counter()
                self._all_reduce(grad, False)
                b = time.perf_counter()
            self._events.append((a, b))
            return None
        return self._all_reduce(grad, async_op)

    def start(self, grad: torch.Tensor):
        """Enqueue the all-reduce of ``grad`` without waiting (fp32 wire); returns ``wait()``, which
        makes the CURRENT stream wait for the result (host never blocks on RCCL)."""
        if not self.ctx.is_distributed:
            return lambda: None
        if self.compress:
            self.all_reduce(grad)
            return lambda: None
        hs = self._all_reduce(grad, async_op=True)
        hs = hs if isinstance(hs, list) else [hs]

        def wait():
            for h in hs:
                h.wait()
        return wait

    def _all_reduce(self, grad: torch.Tensor, async_op: bool = False):
        g = self.ctx.group
        self.calls += 1
        if self.compress == "bf16":
            if self._wire is None or self._wire.device != grad.device:
                self._wire = torch.empty(self.numel, dtype=torch.bfloat16, device=grad.device)
            self._wire.copy_(grad)
            hs = [dist.all_reduce(self._wire[a:b], group=g, async_op=True) for a, b in self.slices]
            for h in hs:
                h.wait()
            grad.copy_(self._wire)
            return None
        if len(self.slices) == 1:
            return dist.all_reduce(grad, group=g, async_op=async_op)
        hs = [dist.all_reduce(grad[a:b], group=g, async_op=True) for a, b in self.slices]
        if async_op:
            return hs
        for h in hs:
            h.wait()
        return None


def broadcast_tensors(ctx: DistContext, tensors: Sequence[torch.Tensor], src: int = 0) -> None:
    if not ctx.is_distributed:
        return
    for t in tensors:
        if t is not None and t.numel():
            dist.broadcast(t, src, group=ctx.group)


def global_mean_std(ctx: DistContext, values: torch.Tensor) -> Dict[str, float]:
    """Mean / population std over every rank's values (the router's GetAvg/GetStd,
    `TrainerRouterActor.scala:89-94,148-151`) via one all_reduce of (n, Σx, Σx²);
    NaN entries (episodes not finished) are excluded like untrained workers."""
    v = values.detach().double().flatten()
    ok = ~torch.isnan(v)
    v = v[ok]
    s = torch.stack([torch.tensor(float(v.numel()), dtype=torch.float64, device=v.device), v.sum(),
                     (v * v).sum()])
    if ctx.is_distributed:
        s = s.to(ctx.device)
        dist.all_reduce(s, group=ctx.group)
    n, sx, sxx = (float(x) for x in s.cpu())
    if n == 0:
        return {"n": 0, "mean": math.nan, "std": math.nan}
    m = sx / n
    return {"n": int(n), "mean": m, "std": math.sqrt(max(0.0, sxx / n - m * m))}


def all_gather_values(ctx: DistContext, values: torch.Tensor) -> torch.Tensor:
    """Concatenate every rank's 1-D tensor (equal lengths) in rank order."""
    if not ctx.is_distributed:
        return values
    v = values.contiguous().to(ctx.device)
    out = [torch.empty_like(v) for _ in range(ctx.world_size)]
    dist.all_gather(out, v, group=ctx.group)
    return torch.cat(out)


def all_done(ctx: DistContext, done: bool) -> bool:
    """Completion barrier (each worker's ``Trained`` to the router): MIN over ranks."""
    if not ctx.is_distributed:
        return bool(done)
    t = torch.tensor([1 if done else 0], dtype=torch.int32, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.group)
    return bool(int(t.item()))


def max_over_ranks(ctx: DistContext, x: float) -> float:
    if not ctx.is_distributed:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctx.group)
    return float(t.item())
