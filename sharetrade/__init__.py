"""sharetrade — MI355X-native actor-distributed deep-RL trading engine.

Capabilities of cosmir17/Scala-akka-tensorflow-sharetrade-helper, rebuilt
MI355X-first: a Python actor control plane (message API, FSMs, supervision,
routing, persistence) over a HIP/CDNA4 data plane (fused Q-learning step
kernels, RCCL data parallelism).  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"

from .config import ACTIONS, Config, preset_config  # noqa: F401
