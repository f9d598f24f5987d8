"""The BatchNorm-backward finalize folded into the reduce kernel's last arrivals
(``batch_norm.hip`` BwdFin + ``dev::tail_arrive``; opt-in ``XDDP_BN_TAIL=1``, measured slower:
profiles/r6_bn_finalize_fold.txt) against the separate finalize launch (the default): bitwise
equal on the ResNet-50 stage shapes and the backward's mask / residual / coefficient forms, bitwise deterministic over 200 launches under uneven load (a GEMM
stream competing for the CUs, so arrival order varies), and no reducer ever hits its spin bound.
The separate path itself is checked against fp32 references in tests/test_norm_gpu.py."""
import os

import pytest
import torch

from distributeddataparallel_amd._native import load

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, C, H, W): the four ResNet-50 stage shapes at bs256 (BN inputs of the bottleneck convs), a
# block output (C = 4 x width), the layer-4 output, and small shapes where the row blocks are
# fewer than the channel vectors (reducers finalize several vectors each) or C / 8 is odd
SHAPES = [(256, 64, 56, 56), (256, 128, 28, 28), (256, 256, 14, 14), (256, 512, 7, 7), (256, 256, 56, 56),
          (256, 2048, 7, 7), (2, 32, 3, 5), (3, 40, 5, 7)]


def _inputs(shape, dt, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    cl = torch.channels_last
    x = torch.randn(shape, device=DEV, generator=g).to(dt).contiguous(memory_format=cl)
    r = torch.randn(shape, device=DEV, generator=g).to(dt).contiguous(memory_format=cl)
    C = shape[1]
    w = (torch.rand(C, device=DEV, generator=g) + 0.5).to(dt)
    b = (torch.randn(C, device=DEV, generator=g) * 0.1).to(dt)
    g1 = torch.randn(shape, device=DEV, generator=g).to(dt).contiguous(memory_format=cl)
    g2 = torch.randn(shape, device=DEV, generator=g).to(dt).contiguous(memory_format=cl)
    return x, r, w, b, g1, g2


def _forms(C_, x, r, w, b, g1, g2):
    """(name, thunk) for the backward forms the ResNet step uses."""
    yr, mean_r, inv_r, ss_r, bits = C_.bn_forward(x, w, b, None, None, None, True, 0.1, False, 1e-5, r, True, True)
    y, mean, inv, ss, _ = C_.bn_forward(x, w, b, None, None, None, True, 0.1, False, 1e-5, None, True, False)
    return [
        # 3x3 BN + ReLU: mask recomputed from scale/shift, elementwise pass
        ("relu_ss", lambda: C_.bn_backward(g1, x, None, w, mean, inv, ss, True, False, True, None, None)),
        # the same folded into the consumer GEMM (coef [5, C] with scale/shift)
        ("relu_ss_coef", lambda: C_.bn_backward(g1, x, None, w, mean, inv, ss, True, False, True, None, None, True)),
        # block output: bit mask, two incoming gradients, d(residual) from the reduce pass, coef only
        ("res_dual_coef", lambda: C_.bn_backward(g1, x, None, w, mean_r, inv_r, ss_r, True, True, True, g2, bits,
                                                 True)),
        # residual, mask from y, single gradient, elementwise pass
        ("res_y", lambda: C_.bn_backward(g1, x, yr, w, mean_r, inv_r, ss_r, True, True, True, None, None)),
        # no ReLU (downsample BN), coefficients only, no weight gradient
        ("plain_coef", lambda: C_.bn_backward(g1, x, None, w, mean, inv, ss, False, False, False, None, None, True)),
    ]


def _run(thunk, tail):
    old = os.environ.get("XDDP_BN_TAIL")
    os.environ["XDDP_BN_TAIL"] = "1" if tail else "0"
    try:
        out = thunk()
    finally:
        if old is None:
            os.environ.pop("XDDP_BN_TAIL")
        else:
            os.environ["XDDP_BN_TAIL"] = old
    return [None if t is None else t.clone() for t in out]


def _assert_bitwise(a, b, what):
    for i, (u, v) in enumerate(zip(a, b)):
        assert (u is None) == (v is None), f"{what}: output {i} presence differs"
        if u is not None:
            assert torch.equal(u, v), f"{what}: output {i} differs (max abs {(u.float() - v.float()).abs().max()})"


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_bn_backward_tail_bitwise_equals_separate_finalize(shape, dt):
    if dt == torch.float32 and shape[0] == 256 and shape[2] == 56:
        pytest.skip("fp32 at the largest shapes: covered by the bf16 run (same kernels, half the memory)")
    C_ = load()
    torch.manual_seed(0)
    for name, thunk in _forms(C_, *_inputs(shape, dt)):
        ref = _run(thunk, tail=False)
        got = _run(thunk, tail=True)
        torch.cuda.synchronize()
        _assert_bitwise(got, ref, f"{shape} {dt} {name}")
    assert not C_.bn_tail_timeouts(torch.cuda.current_device())


def test_bn_backward_tail_deterministic_under_uneven_load():
    """200 folded launches while another stream runs GEMMs (blocks arrive in varying order, some
    delayed behind the GEMM's): every result bitwise equal to the first; no spin timeouts."""
    C_ = load()
    shape = (256, 256, 14, 14)
    x, r, w, b, g1, g2 = _inputs(shape, torch.bfloat16, seed=3)
    forms = dict(_forms(C_, x, r, w, b, g1, g2))
    thunks = [forms["res_dual_coef"], forms["relu_ss"]]
    first = [_run(t, tail=True) for t in thunks]
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16)
    for it in range(200):
        if it % 20 == 0:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(4):
                    a = (a @ a).clamp_(-1, 1)
        for t, f in zip(thunks, first):
            _assert_bitwise(_run(t, tail=True), f, f"launch {it}")
    torch.cuda.synchronize()
    assert not C_.bn_tail_timeouts(torch.cuda.current_device())
