
from . import torch_ops  # noqa: F401  -- registers torch.ops.sharetrade.* (sharetrade/ops/torch_ops.py)
