"""``torch.distributed``-style collective API over xddp's native communicators."""
from .c10d import *  # noqa: F401,F403
from .c10d import (  # noqa: F401
    Backend, GroupMember, ProcessGroup, ReduceOp, Work, all_gather, all_gather_into_tensor, all_gather_object,
    all_reduce, all_to_all_single, barrier, broadcast, broadcast_object_list, coalescing, destroy_process_group,
    get_backend, get_default_group, get_local_rank, get_process_group_ranks, get_rank, get_world_size,
    init_process_group, irecv, is_available, is_initialized, isend, monitored_barrier, new_group, recv,
    reduce_scatter_tensor, send,
)
