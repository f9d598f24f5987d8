"""Launchers (torchrun / xddp.run / spawn), failure handling, fault injection, sampler."""
import os
import subprocess
import sys
import time

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "workers", "ddp_worker.py")


def _env(**kw):
    e = dict(os.environ)
    e.update({"OMP_NUM_THREADS": "1", "PYTHONPATH": REPO})
    e.update({k: str(v) for k, v in kw.items()})
    return e


def test_torchrun_agent_store_bootstrap():
    """The driver launches N>1 via torch.distributed.run; xddp must bootstrap through the agent store."""
    from distributeddataparallel_amd.utils.spawn import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), WORKER]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "RANK 0/2 OK" in r.stdout and "RANK 1/2 OK" in r.stdout


def test_xddp_run_launcher():
    cmd = [sys.executable, "-m", "distributeddataparallel_amd.run", "--nproc-per-node", "3", WORKER]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=180, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    for i in range(3):
        assert f"RANK {i}/3 OK" in r.stdout


def test_fault_injection_kills_group():
    cmd = [sys.executable, "-m", "distributeddataparallel_amd.run", "--nproc-per-node", "2", "--grace-period", "2",
           WORKER]
    t0 = time.time()
    r = subprocess.run(cmd, env=_env(XDDP_FAULT_INJECT="rank=1,step=2,mode=exit,code=13", WORKER_STEPS=50),
                       capture_output=True, text=True, timeout=180, cwd=REPO)
    assert r.returncode == 13, (r.returncode, r.stderr[-2000:])
    assert "failed with exit code 13" in r.stderr
    assert time.time() - t0 < 90


def test_restart_after_fault():
    cmd = [sys.executable, "-m", "distributeddataparallel_amd.run", "--nproc-per-node", "2", "--max-restarts", "1",
           "--grace-period", "2", WORKER]
    r = subprocess.run(cmd, env=_env(XDDP_FAULT_INJECT="rank=0,step=3,mode=exit,code=7"), capture_output=True,
                       text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "RANK 0/2 OK restart=1" in r.stdout and "restarting the group" in r.stderr


def _bad_worker(rank):
    if rank == 1:
        raise ValueError("boom from rank 1")
    time.sleep(30)


def test_spawn_propagates_child_exception():
    from distributeddataparallel_amd.utils.spawn import ProcessRaisedException, spawn

    t0 = time.time()
    with pytest.raises(ProcessRaisedException) as ei:
        spawn(_bad_worker, nprocs=2)
    assert "boom from rank 1" in str(ei.value) and ei.value.error_index == 1
    assert time.time() - t0 < 25


@pytest.mark.parametrize("n,world,drop_last,shuffle", [(50000, 8, False, True), (103, 4, False, True),
                                                       (103, 4, True, True), (10, 3, False, False)])
def test_sampler_matches_reference(n, world, drop_last, shuffle):
    from torch.utils.data.distributed import DistributedSampler as RefSampler

    from distributeddataparallel_amd.data import DistributedSampler

    ds = list(range(n))
    for rank in range(world):
        a = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, seed=3, drop_last=drop_last)
        b = RefSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, seed=3, drop_last=drop_last)
        for ep in (0, 1):
            a.set_epoch(ep)
            b.set_epoch(ep)
            assert list(a) == list(b)
        assert len(a) == len(b)


def test_reference_workload_example_runs_and_resumes(tmp_path):
    """examples/train_ddp_cifar.py (the ref:dpp.py workflow) on the CPU backend, with checkpoint+resume."""
    ck = tmp_path / "ck.pt"
    ex = os.path.join(REPO, "examples", "train_ddp_cifar.py")
    base = [sys.executable, ex, "--spawn", "2", "--backend", "cpu", "--synthetic-len", "256", "--max-steps", "3",
            "--batch-size", "8"]
    r = subprocess.run(base + ["--epochs", "1", "--checkpoint", str(ck)], env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 0, Batch 0, Loss:" in r.stdout and ck.exists()
    r = subprocess.run(base + ["--epochs", "2", "--resume", str(ck)], env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 1, Batch 0" in r.stdout and "Epoch 0," not in r.stdout
