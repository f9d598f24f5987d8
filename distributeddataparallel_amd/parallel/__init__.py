from .distributed import DDP, BuiltinCommHookType, DistributedDataParallel  # noqa: F401
from .join import Join, Joinable, JoinHook  # noqa: F401
