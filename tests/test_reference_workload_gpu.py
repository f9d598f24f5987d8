"""The reference workload as the reference runs it (``ref:dpp.py:14-15, 35, 38-41``):
``examples/train_ddp_cifar.py`` — ResNet-18 with a 10-class head, fp32, batch 32, plain
``SGD(lr=0.01)``, CIFAR-shaped synthetic data — on RCCL with one rank for 50 steps, once on xddp
(own DDP + Reducer + RCCL communicator, own fp32 BatchNorm kernels, MIOpen convs) and once on the
reference stack (torch DDP + torch BatchNorm over torch.distributed nccl = RCCL). Every step's
rank-0 loss must agree within 1e-4 relative."""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _losses(impl, port):
    from distributeddataparallel_amd.utils.spawn import free_port

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), XDDP_NO_AUTOBUILD="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "examples", "train_ddp_cifar.py"), "--impl", impl,
                        "--backend", "rccl", "--max-steps", "50", "--log-every", "1", "--epochs", "1",
                        "--synthetic-len", "4096", "--batch-size", "32"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=REPO)
    assert r.returncode == 0, (impl, r.stdout[-2000:], r.stderr[-4000:])
    return [float(m) for m in re.findall(r"Loss: ([-0-9.eE+naif]+)", r.stdout)]


def test_reference_workload_fp32_loss_parity_vs_torch_ddp():
    a, b = _losses("xddp", 0), _losses("torch", 1)
    assert len(a) == len(b) == 50, (len(a), len(b))
    worst = max(abs(x - y) / max(abs(y), 1e-12) for x, y in zip(a, b))
    assert worst <= 1e-4, (worst, list(zip(a, b))[:10], list(zip(a, b))[-5:])
