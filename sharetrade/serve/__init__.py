"""Policy serving: batched ``SelectionAction`` inference on the GPU (``csrc/qserve.hip``).

* :class:`PolicyServer` — resident weights, one launch per request batch, hot weight swaps;
* :class:`DynamicBatcher` — single requests from many client threads -> server batches;
* :class:`PolicyServingActor` — the reference's actor message API over the server.
"""
from .actor import LoadPolicy, PolicyLoaded, PolicyServingActor
from .kernel import ServeKernel, reference_select, supported
from .server import DynamicBatcher, PolicyServer

__all__ = ["PolicyServer", "DynamicBatcher", "PolicyServingActor", "LoadPolicy", "PolicyLoaded", "ServeKernel",
           "reference_select", "supported"]
