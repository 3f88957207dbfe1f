"""Model checkpoints: the deterministic C++ archive writer (`csrc/runtime/ckpt.cpp`)
plus a verifying NumPy/torch reader.

Reference: ``saveSnapshot((session, iteration))`` every 500 ``UpdateQ``s with an
empty body (`QDecisionPolicyActor.scala:74,91-93`, quirk Q13) — no model state
is ever saved or resumed.  Here the learner state (parameters, optimizer
accumulators, update counter, RNG counters, env state) is written as a named
tensor archive whose bytes depend only on the state ("bit-compatible"): saving
the same state twice yields byte-identical files, and a resumed run continues
bit-exactly (tested in ``tests/test_persistence.py``).
"""
from __future__ import annotations

import ctypes as C
import json
import mmap
import os
import struct
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from . import native

MAGIC = b"STCKPT01"
END = b"STCKEND1"

_DT = [
    (torch.float32, np.float32), (torch.float64, np.float64), (torch.float16, np.float16),
    (torch.bfloat16, None), (torch.int32, np.int32), (torch.int64, np.int64), (torch.uint8, np.uint8),
    (torch.int8, np.int8), (torch.bool, np.bool_), (torch.int16, np.int16),
]
_TORCH_TO_CODE = {t: i for i, (t, _) in enumerate(_DT)}


class CheckpointError(RuntimeError):
    pass


def _canon_meta(meta: Optional[Dict[str, Any]]) -> bytes:
    return json.dumps(meta or {}, sort_keys=True, separators=(",", ":")).encode()


def save(path: str, tensors: Dict[str, torch.Tensor], meta: Optional[Dict[str, Any]] = None,
         fsync: bool = True) -> int:
    """Write ``tensors`` (insertion order is the archive order) atomically.
    Returns the file size in bytes."""
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    names, dtypes, ndims, shapes, ptrs, sizes, keep = [], [], [], [], [], [], []
    for k, t in tensors.items():
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(t)
        t = t.detach().to("cpu").contiguous()
        if t.dtype not in _TORCH_TO_CODE:
            raise CheckpointError(f"unsupported dtype {t.dtype} for {k}")
        keep.append(t)
        names.append(k.encode())
        dtypes.append(_TORCH_TO_CODE[t.dtype])
        ndims.append(t.dim())
        shapes.extend(int(s) for s in t.shape)
        ptrs.append(t.data_ptr() if t.numel() else 0)
        sizes.append(t.numel() * t.element_size())
    n = len(names)
    m = _canon_meta(meta)
    r = native.lib().st_ckpt_write(
        path.encode(), n, (C.c_char_p * max(1, n))(*names), (C.c_int * max(1, n))(*dtypes),
        (C.c_int * max(1, n))(*ndims), (C.c_int64 * max(1, len(shapes)))(*shapes),
        (C.c_void_p * max(1, n))(*ptrs), (C.c_uint64 * max(1, n))(*sizes), m, len(m), int(fsync))
    del keep
    if r < 0:
        raise CheckpointError(f"checkpoint write failed: {path}")
    return int(r)


def load(path: str, device: Optional[str] = None, verify: bool = True) -> Tuple[Dict[str, torch.Tensor], Dict]:
    """Read an archive; verifies the header CRC and every tensor's CRC."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 8 + 20 or data[:8] != MAGIC or data[-8:] != END:
        raise CheckpointError(f"not a sharetrade checkpoint: {path}")
    table_end, head_crc = struct.unpack_from("<QI", data, len(data) - 20)
    if verify and native.crc_mask(native.crc32c(data[:table_end])) != head_crc:
        raise CheckpointError("checkpoint header CRC mismatch")
    version, n, meta_len = struct.unpack_from("<IIQ", data, 8)
    if version != 1:
        raise CheckpointError(f"unsupported checkpoint version {version}")
    i = 24
    meta = json.loads(data[i:i + meta_len].decode() or "{}")
    i = (i + meta_len + 63) & ~63
    out: Dict[str, torch.Tensor] = {}
    for _ in range(n):
        (nl,) = struct.unpack_from("<H", data, i)
        i += 2
        name = data[i:i + nl].decode()
        i += nl
        dt, nd = data[i], data[i + 1]
        i += 2
        shape = struct.unpack_from("<" + "q" * nd, data, i)
        i += 8 * nd
        off, nbytes, crc = struct.unpack_from("<QQI", data, i)
        i += 20
        blob = data[off:off + nbytes]
        if verify and native.crc_mask(native.crc32c(blob)) != crc:
            raise CheckpointError(f"tensor {name}: CRC mismatch")
        tdt = _DT[dt][0]
        if tdt == torch.bfloat16:
            t = torch.frombuffer(bytearray(blob), dtype=torch.int16).view(torch.bfloat16) if nbytes else \
                torch.empty(0, dtype=torch.bfloat16)
        else:
            t = torch.from_numpy(np.frombuffer(blob, dtype=_DT[dt][1]).copy()) if nbytes else \
                torch.empty(0, dtype=tdt)
        t = t.reshape(shape)
        out[name] = t.to(device) if device else t
    return out, meta


def file_crc(path: str) -> int:
    with open(path, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        try:
            return native.crc32c(bytes(mm))
        finally:
            mm.close()


class CheckpointManager:
    """Periodic checkpoints ``<dir>/ckpt-<step:012d>.stck`` with retention."""

    def __init__(self, directory: str, keep: int = 3, interval: int = 500):
        self.dir = directory
        self.keep = keep
        self.interval = interval

    def path_for(self, step: int) -> str:
        return os.path.join(self.dir, f"ckpt-{step:012d}.stck")

    def should_save(self, step: int) -> bool:
        # QDecisionPolicyActor.scala:74 — `iteration % 500 == 0 && iteration != 0`
        return self.interval > 0 and step != 0 and step % self.interval == 0

    def save(self, step: int, tensors: Dict[str, torch.Tensor], meta: Optional[Dict[str, Any]] = None) -> str:
        p = self.path_for(step)
        save(p, tensors, dict(meta or {}, step=step))
        self._gc()
        return p

    def list(self):
        if not os.path.isdir(self.dir):
            return []
        return sorted(f for f in os.listdir(self.dir) if f.startswith("ckpt-") and f.endswith(".stck"))

    def latest(self) -> Optional[str]:
        for f in reversed(self.list()):
            p = os.path.join(self.dir, f)
            try:
                load(p, verify=True)
                return p
            except CheckpointError:
                continue
        return None

    def _gc(self) -> None:
        files = self.list()
        for f in files[:-self.keep] if self.keep > 0 else []:
            try:
                os.remove(os.path.join(self.dir, f))
            except OSError:
                pass
