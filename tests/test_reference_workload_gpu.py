"""The reference workload as the reference runs it (``ref:dpp.py:14-15, 35, 38-41``):
ResNet-18 with a 10-class head, fp32, batch 32, plain ``SGD(lr=0.01)``, CIFAR-shaped data.

* One step's gradients of the xddp fp32 path (FusedBatchNorm2d kernels, channels_last, MIOpen
  convs) against an fp64 CPU model of the same weights and batch: <= 1e-4 relative per parameter.
* 50 DDP training steps (xddp DDP + Reducer + RCCL communicator, one rank) on the reference data
  pipeline, teacher-forced against fp64: every step's loss within 1e-5 and every gradient within
  1e-4 relative. Free-running trajectories cannot be compared over 50 steps: this workload is
  chaotic (on the CPU, torch fp32 vs fp64 differ by 2.3e-4 in the step-1 loss and by 2-6 % by
  step 3-4; a 1e-7 relative weight perturbation does the same), so
* ``examples/train_ddp_cifar.py`` free-running on RCCL vs the reference stack (torch DDP + torch
  BatchNorm) on the CPU / gloo in fp32 is asserted on its opening steps only (within 1e-5).

The oracle is torch on the CPU, not torch on the GPU: on this MI355X image torch's own fp32 NCHW
path (MIOpen's algorithm choice) carries ~7.6e-3 relative gradient error against fp64 on this model
(``scripts/ref_grad_parity.py``), so its loss trajectory drifts from any fp32-accurate run within a
few steps; that trajectory is printed for the record, not asserted."""
import os
import re
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_model_fp32_gradients_vs_fp64():
    from distributeddataparallel_amd.models import SimpleCNN
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    torch.manual_seed(0)
    ref = SimpleCNN().double()
    x = torch.randn(32, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (32,))
    F.cross_entropy(ref(x), y).backward()
    m = SimpleCNN(norm_layer=FusedBatchNorm2d).cuda().to(memory_format=torch.channels_last)
    m.load_state_dict(ref.state_dict())
    F.cross_entropy(m(x.float().cuda().contiguous(memory_format=torch.channels_last)), y.cuda()).backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        err = (p.grad.double().cpu() - q.grad).abs().max().item() / (q.grad.abs().max().item() + 1e-30)
        assert err <= 1e-4, (n, err)


def _losses(impl, backend):
    from distributeddataparallel_amd.utils.spawn import free_port

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), XDDP_NO_AUTOBUILD="1", OMP_NUM_THREADS="16")
    r = subprocess.run([sys.executable, os.path.join(REPO, "examples", "train_ddp_cifar.py"), "--impl", impl,
                        "--backend", backend, "--max-steps", "50", "--log-every", "1", "--epochs", "1",
                        "--synthetic-len", "4096", "--batch-size", "32"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=REPO)
    assert r.returncode == 0, (impl, backend, r.stdout[-2000:], r.stderr[-4000:])
    return [float(m) for m in re.findall(r"Loss: ([-0-9.eE+naif]+)", r.stdout)]


def test_reference_workload_fp32_teacher_forced_50_steps():
    """50 DDP training steps of the reference workload on xddp (RCCL, one rank), each step's loss and
    every gradient checked against fp64 on the same parameters and batch (tests/_ref_teacher_forced.py)."""
    from distributeddataparallel_amd.utils.spawn import free_port

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), XDDP_NO_AUTOBUILD="1", OMP_NUM_THREADS="16")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "_ref_teacher_forced.py"), "50"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=REPO)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    rows = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("step ")]
    assert len(rows) == 50, r.stdout[-2000:]
    worst_l = max(float(t[2]) for t in rows)
    worst_g = max(float(t[3]) for t in rows)
    print(f"teacher-forced 50 steps: worst loss rel {worst_l:.2e}, worst grad rel {worst_g:.2e}")
    assert worst_l <= 1e-5 and worst_g <= 1e-4, (worst_l, worst_g, rows[:5])


def test_reference_workload_fp32_trajectory_vs_torch_ddp():
    """The example script itself, free-running: xddp (GPU, RCCL) against the reference stack (torch
    DDP + torch BN, CPU / gloo, fp32). The first steps agree to ~1e-7 (the r6 box: steps 0-3 within
    4e-7); past that the workload's chaos (see tests/_ref_teacher_forced.py) separates any two fp32
    runs, torch's own GPU run included, so only the opening steps are asserted."""
    a = _losses("xddp", "rccl")
    b = _losses("torch", "cpu")
    c = _losses("torch", "rccl")
    assert len(a) == len(b) == len(c) == 50, (len(a), len(b), len(c))
    rel = [abs(x - y) / max(abs(y), 1e-12) for x, y in zip(a, b)]
    drift = [abs(x - y) / max(abs(y), 1e-12) for x, y in zip(c, b)]
    print(f"opening 3 steps: xddp GPU vs torch CPU {max(rel[:3]):.2e}; torch GPU vs torch CPU {max(drift[:3]):.2e}")
    print("step  xddp-gpu  torch-cpu  torch-gpu")
    for i in range(0, 50, 5):
        print(f"{i:4d}  {a[i]:.6f}  {b[i]:.6f}  {c[i]:.6f}")
    assert max(rel[:3]) <= 1e-5, (rel[:5], list(zip(a, b))[:5])
