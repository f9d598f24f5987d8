"""The reference workload as the reference runs it (``ref:dpp.py:14-15, 35, 38-41``):
ResNet-18 with a 10-class head, fp32, batch 32, plain ``SGD(lr=0.01)``, CIFAR-shaped data.

* One step's gradients of the xddp fp32 path (FusedBatchNorm2d kernels, channels_last, MIOpen
  convs) against an fp64 CPU model of the same weights and batch: <= 1e-4 relative per parameter.
* 50 DDP training steps (xddp DDP + Reducer + RCCL communicator, one rank) on the reference data
  pipeline, teacher-forced against fp64: every step's loss within 1e-5 and the gradients within
  1e-4 relative in at least 30 of 50 steps (the others hit fp32-vs-fp64 ReLU / max-pool near-tie
  flips, which reroute whole gradient paths; see the test's docstring).
  Free-running trajectories cannot be compared over 50 steps: this workload is chaotic (on the
  CPU, torch fp32 vs fp64 differ by 2.3e-4 in the step-1 loss and by 2-6 % by step 3-4; a 1e-7
  relative weight perturbation does the same), so
* ``examples/train_ddp_cifar.py`` free-running on RCCL vs the reference stack (torch DDP + torch
  BatchNorm) on the CPU / gloo in fp32 is asserted on step 0 only (within 1e-6).

torch's own fp32 NCHW path on this image carries ~7.6e-3 relative gradient error against fp64 on
this model (``scripts/ref_grad_parity.py``); its GPU trajectory is printed for the record only."""
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
    gradients checked against fp64 on the same parameters and batch (tests/_ref_teacher_forced.py):
    the loss of every step within 1e-5, and every gradient — xddp's own kernels' (every BatchNorm
    weight / bias, through the fused BN backward; the fc layer) and the library convs' — within 1e-4
    in at least 30 of the 50 steps (median step within 1e-4); the worst step is printed. The other
    steps carry 1e-3 - 3e-1 relative errors in a few layers whichever conv implementation runs
    (MIOpen, MIOpen without its implicit-GEMM solvers, or PyTorch's native convolutions:
    XDDP_TEST_NO_MIOPEN=1) and with r5's BN kernels alike, and which steps they hit changes from run to run: a ReLU or max-pool decision
    that fp32 and fp64 resolve differently (a near-tie) reroutes a whole gradient path, and the
    library's run-to-run rounding moves which near-ties flip (r6 diagnosis, commit log)."""
    from distributeddataparallel_amd.utils.spawn import free_port

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), XDDP_NO_AUTOBUILD="1", OMP_NUM_THREADS="16")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "_ref_teacher_forced.py"), "50"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=REPO)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    rows = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("step ")]
    assert len(rows) == 50, r.stdout[-2000:]
    loss = [float(t[2]) for t in rows]
    grad = [float(t[3]) for t in rows]
    own = [float(t[5]) for t in rows]
    ok_steps = sum(gv <= 1e-4 for gv in grad)
    print(f"teacher-forced 50 steps: worst loss rel {max(loss):.2e}, worst own-kernel grad rel {max(own):.2e}, "
          f"all-grad rel <= 1e-4 in {ok_steps}/50 steps (worst {max(grad):.2e} on {rows[grad.index(max(grad))][4]})")
    own_ok = sum(ov <= 1e-4 for ov in own)
    assert max(loss) <= 1e-5, rows
    # a kernel bug is systematic (every step); the near-tie flips hit 10-30 % of the steps on the
    # boxes measured (35-48 of 50 clean)
    assert sorted(own)[len(own) // 2] <= 1e-4, rows
    assert own_ok >= 30 and ok_steps >= 30, rows


def test_reference_workload_fp32_trajectory_vs_torch_ddp():
    """The example script itself, free-running: xddp (GPU, RCCL) against the reference stack (torch
    DDP + torch BN, CPU / gloo, fp32). Step 0 agrees to ~1e-7; the step-1 loss is bimodal (2.46965 or
    2.47021 across runs of either stack, and a 1e-7 relative weight perturbation switches it on the
    CPU: a discontinuity of the loss surface), so later steps are printed, not asserted."""
    a = _losses("xddp", "rccl")
    b = _losses("torch", "cpu")
    c = _losses("torch", "rccl")
    assert len(a) == len(b) == len(c) == 50, (len(a), len(b), len(c))
    rel = [abs(x - y) / max(abs(y), 1e-12) for x, y in zip(a, b)]
    drift = [abs(x - y) / max(abs(y), 1e-12) for x, y in zip(c, b)]
    print(f"step 0: xddp GPU vs torch CPU {rel[0]:.2e}; torch GPU vs torch CPU {drift[0]:.2e}")
    print("step  xddp-gpu  torch-cpu  torch-gpu")
    for i in list(range(0, 5)) + list(range(5, 50, 5)):
        print(f"{i:4d}  {a[i]:.6f}  {b[i]:.6f}  {c[i]:.6f}")
    assert rel[0] <= 1e-6, (rel[:3], list(zip(a, b))[:3])
