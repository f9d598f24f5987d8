"""Multi-process test harness (MultiProcessTestCase analogue): run a module-level
function in W spawned ranks on the CPU backend and surface the first failure."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _entry(rank, fn, world, backend, args):
    sys.path.insert(0, os.environ.get("XDDP_PKG_ROOT", REPO))
    from distributeddataparallel_amd import distributed as xdist

    root = os.environ.get("XDDP_PKG_ROOT")
    if root:  # a sanitizer run: every rank must run the instrumented extension, not the repo's
        from distributeddataparallel_amd._native import load

        assert load().__file__.startswith(root), load().__file__

    xdist.init_process_group(backend, rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        xdist.destroy_process_group()


def run_ranks(fn, world=2, backend="cpu", args=(), env=None):
    from distributeddataparallel_amd.utils.spawn import free_ports, spawn

    p_store, p_torch = free_ports(2)  # distinct: the xddp and torch stores each bind one
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(p_store), "OMP_NUM_THREADS": "1",
           "XDDP_TEST_TORCH_PORT": str(p_torch), **(env or {})}
    spawn(_entry, args=(fn, world, backend, args), nprocs=world, env=env)
