"""Cross-rank replica check (utils/replicas.py): checksums agree for identical
replicas and name the rank whose bucket was corrupted after its all-reduce
(XDDP_FAULT_CORRUPT, injected inside the Reducer's finalize); bench.py reports it and exits 3."""
import json
import os
import subprocess
import sys

import pytest
import torch

from _dist_utils import run_ranks

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_checksum_is_order_and_bit_sensitive():
    from distributeddataparallel_amd.utils.replicas import checksum

    a = [torch.arange(10, dtype=torch.float32), torch.ones(3, dtype=torch.int64)]
    c0 = checksum(a)
    assert torch.equal(c0, checksum([t.clone() for t in a]))
    assert not torch.equal(c0, checksum(a[::-1]))  # order matters (position-seeded hash)
    b = [a[0].clone(), a[1].clone()]
    b[0][3] = torch.nextafter(b[0][3], torch.tensor(100.0))  # one ulp
    assert not torch.equal(c0[1:], checksum(b)[1:])
    p = [a[0].flip(0), a[1]]  # same values, permuted: the sum agrees, the hash does not
    assert checksum(p)[0] == c0[0] and not torch.equal(checksum(p)[1:], c0[1:])


def _w_ddp_check(rank, world, corrupt):
    import torch.nn.functional as F

    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd.models import MLP

    torch.manual_seed(0)
    m = MLP(784, 32, 10)
    ddp = xddp.DDP(m)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(5 + rank)
    for it in range(4):
        x, y = torch.randn(8, 1, 28, 28, generator=g), torch.randint(0, 10, (8,), generator=g)
        opt.zero_grad()
        try:
            F.cross_entropy(ddp(x), y).backward()
        except RuntimeError as e:  # XDDP_CHECK_REPLICAS=2 checks before forwards 2 and 4
            assert corrupt and "replicas diverged" in str(e) and "[1]" in str(e), e
            assert it == 3, it  # corrupted in iteration 2 (-> params after step 2), found before forward 4
            return
        opt.step()
    rep = ddp.check_replicas()
    if corrupt:
        raise AssertionError(f"the per-forward check missed the corruption: {rep}")
    assert rep["replicas_identical"] and rep["mismatch_ranks"] == [] and rep["max_abs_diff"] == 0.0, rep


def test_ddp_periodic_replica_check_clean():
    run_ranks(_w_ddp_check, world=2, args=(False,), env={"XDDP_CHECK_REPLICAS": "2"})


def test_ddp_periodic_replica_check_names_corrupted_rank():
    run_ranks(_w_ddp_check, world=2, args=(True,), env={"XDDP_CHECK_REPLICAS": "2",
                                                       "XDDP_FAULT_CORRUPT": "rank=1,iter=2"})


@pytest.mark.parametrize("corrupt", [False, True])
def test_bench_reports_replica_divergence(corrupt):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("XDDP_FAULT_CORRUPT", None)
    if corrupt:
        env["XDDP_FAULT_CORRUPT"] = "rank=1,iter=3"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--backend", "cpu", "--model", "mlp", "--steps", "3", "--warmup", "1", "--diag-steps", "0"],
                       capture_output=True, text=True, env=env, timeout=600, cwd="/tmp")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(lines[0])
    if corrupt:
        assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
        assert out["replicas_identical"] is False and out["replica_mismatch_ranks"] == [1], out
        assert out["replica_max_abs_diff"] > 0
    else:
        assert r.returncode == 0, r.stderr[-3000:]
        assert out["replicas_identical"] is True and out["replica_max_abs_diff"] == 0.0, out
