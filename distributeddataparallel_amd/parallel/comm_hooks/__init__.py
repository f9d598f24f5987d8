"""DDP communication hooks and their registry (reference: ``ddp_comm_hooks/__init__.py:58-140``)."""
from enum import Enum
from functools import partial

from . import debugging_hooks, default_hooks


def _ddp_comm_hook_wrapper(comm_hook, model, state):
    model.register_comm_hook(state, comm_hook)


def _powerSGD_comm_hook_wrapper(comm_hook, model, state, matrix_approximation_rank, start_powerSGD_iter=1_000):
    from .powerSGD_hook import PowerSGDState

    st = PowerSGDState(process_group=state, matrix_approximation_rank=matrix_approximation_rank,
                       start_powerSGD_iter=start_powerSGD_iter)
    model.register_comm_hook(st, comm_hook)


def _lazy(modname, attr):
    def f(*a, **k):
        import importlib

        return getattr(importlib.import_module(f"{__name__}.{modname}"), attr)(*a, **k)

    f.__name__ = attr
    f.__qualname__ = attr
    return f


class DDPCommHookType(Enum):
    ALLREDUCE = partial(_ddp_comm_hook_wrapper, comm_hook=default_hooks.allreduce_hook)
    FP16_COMPRESS = partial(_ddp_comm_hook_wrapper, comm_hook=default_hooks.fp16_compress_hook)
    BF16_COMPRESS = partial(_ddp_comm_hook_wrapper, comm_hook=default_hooks.bf16_compress_hook)
    QUANTIZE_PER_TENSOR = partial(_ddp_comm_hook_wrapper,
                                  comm_hook=_lazy("quantization_hooks", "quantization_pertensor_hook"))
    QUANTIZE_PER_CHANNEL = partial(_ddp_comm_hook_wrapper,
                                   comm_hook=_lazy("quantization_hooks", "quantization_perchannel_hook"))
    POWER_SGD = partial(_powerSGD_comm_hook_wrapper, comm_hook=_lazy("powerSGD_hook", "powerSGD_hook"),
                        matrix_approximation_rank=1)
    POWER_SGD_RANK2 = partial(_powerSGD_comm_hook_wrapper, comm_hook=_lazy("powerSGD_hook", "powerSGD_hook"),
                              matrix_approximation_rank=2)
    BATCHED_POWER_SGD = partial(_powerSGD_comm_hook_wrapper,
                                comm_hook=_lazy("powerSGD_hook", "batched_powerSGD_hook"),
                                matrix_approximation_rank=1)
    NOOP = partial(_ddp_comm_hook_wrapper, comm_hook=debugging_hooks.noop_hook)


def register_ddp_comm_hook(comm_hook_type: DDPCommHookType, model, state=None):
    comm_hook_type.value(model=model, state=state)
