"""distributeddataparallel_amd (xddp) — an MI355X-native data-parallel training engine.

Capabilities of the reference ``Balaji-Kesavan/DistributedDataparallel`` (a PyTorch DDP
script) rebuilt for AMD Instinct MI355X (gfx950): a native C++ Reducer on
autograd hooks, RCCL-over-xGMI and CPU TCP communicators, a native TCP store, and
hand-written HIP kernels for the per-step hot path.
"""
from ._native import load as _load_native

__version__ = "0.1.0"

from . import distributed  # noqa: E402
from .parallel.distributed import DistributedDataParallel, DDP  # noqa: E402,F401
from .parallel.join import Join, Joinable, JoinHook  # noqa: E402,F401


def native():
    """The loaded native extension module."""
    return _load_native()
