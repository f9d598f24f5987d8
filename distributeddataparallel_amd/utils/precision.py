"""fp32-accurate library convolutions for fp32 training (the reference workload, ``ref:dpp.py``).

xddp runs the reference's fp32 ResNet-18 on its own fp32 BatchNorm kernels and the library (MIOpen)
convolutions. On MI355X (ROCm 7.x MIOpen) the implicit-GEMM conv solvers that MIOpen picks for some
fp32 channels_last weight gradients are not fp32-accurate: 50 teacher-forced DDP steps of the
reference model against an fp64 oracle (``tests/_ref_teacher_forced.py``) showed relative weight-
gradient errors of 8-14 % on the stride-2 3x3 convs (``layer3.0.conv1``, ``layer2.1.conv1``) in
some steps, ~6e-6 everywhere else. With the implicit-GEMM solvers disabled
(``MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0``) every step of every parameter stayed within 3e-6; with
``cudnn.deterministic`` only one stem step still failed (2.6e-2). torch's own fp32 NCHW stack on the
same image carries ~7.6e-3 (``scripts/ref_grad_parity.py``).

:func:`accurate_fp32_convs` sets that switch for the process unless the user chose otherwise. It must
run before the first convolution (MIOpen caches the setting); bf16 runs do not call it (their convs
are xddp's own kernels). It is opt-in (``bench.py --accurate-convs 1``,
``examples/train_ddp_cifar.py --accurate-convs``): MIOpen's fallback for channels_last fp32 convs is
slow — the reference workload ran 1,546 img/s with it vs 9,636-10,723 without on one MI355X (torch's
NCHW stack: 5,913-7,170 vs 7,115-7,237; profiles/r6_bench_reference_fp32.txt). A remaining stem-conv
(7x7 / 2, 3 channels) weight gradient stayed 2.7e-2 off fp64 in one of 50 steps even with it.
"""
from __future__ import annotations

import os

__all__ = ["accurate_fp32_convs"]


def accurate_fp32_convs() -> bool:
    """Disable MIOpen's implicit-GEMM conv solvers for this process (fp32-accurate convs). Returns
    whether the switch is now in effect (False when the user set it to something else)."""
    os.environ.setdefault("MIOPEN_DEBUG_CONV_IMPLICIT_GEMM", "0")
    return os.environ["MIOPEN_DEBUG_CONV_IMPLICIT_GEMM"] == "0"
