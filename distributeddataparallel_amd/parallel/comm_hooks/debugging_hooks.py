"""Debugging hooks (reference: ``ddp_comm_hooks/debugging_hooks.py:10``)."""
import torch


def noop_hook(_, bucket) -> torch.futures.Future:
    """Skip communication entirely; useful to measure the compute-only step time."""
    fut = torch.futures.Future()
    fut.set_result(bucket.buffer())
    return fut
