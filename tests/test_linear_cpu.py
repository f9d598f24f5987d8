"""ops/linear.py on the CPU: the library-GEMM custom Functions (linear / multi_linear) and their
autocast behaviour. Under autocast with fp32 weights the custom Functions (no custom_fwd /
custom_bwd) would produce bf16 outputs with fp32 saved operands and fail in backward, so every
path defers to F.linear there; forward and backward must match F.linear under the same autocast."""
import weakref

import torch
import torch.nn.functional as F

from distributeddataparallel_amd.ops import linear as L


def _ref(x, ws):
    return [F.linear(x, w) for w in ws]


def test_linear_and_multi_linear_match_eager_fp32():
    torch.manual_seed(0)
    x = torch.randn(6, 32, requires_grad=True)
    ws = [torch.randn(16, 32, requires_grad=True) for _ in range(3)]
    r = torch.randn(6, 16, requires_grad=True)
    outs = list(L.multi_linear(x, *ws)) + [L.linear(x, ws[0], r)]
    sum(o.square().sum() for o in outs).backward()
    got = [x.grad.clone()] + [w.grad.clone() for w in ws] + [r.grad.clone()]
    for t in [x, r, *ws]:
        t.grad = None
    outs = _ref(x, ws) + [r + F.linear(x, ws[0])]
    sum(o.square().sum() for o in outs).backward()
    want = [x.grad] + [w.grad for w in ws] + [r.grad]
    for g, w in zip(got, want):
        torch.testing.assert_close(g, w, rtol=1e-5, atol=1e-5)


def test_backward_under_autocast_with_fp32_weights():
    torch.manual_seed(1)
    x = torch.randn(8, 64, requires_grad=True)
    ws = [torch.randn(32, 64, requires_grad=True) for _ in range(2)]
    with torch.autocast("cpu", dtype=torch.bfloat16):
        a, b = L.multi_linear(x, *ws)
        c = L.linear(x, ws[1])
        d = L.linear(x, ws[0], residual=torch.randn(8, 32))
        loss = (a.float().sum() + b.float().square().sum() + c.float().mean() + d.float().sum())
    loss.backward()  # raised a dtype mismatch before the autocast guard
    got = [x.grad.clone(), ws[0].grad.clone(), ws[1].grad.clone()]
    assert all(g.dtype == torch.float32 for g in got)
    for t in [x, *ws]:
        t.grad = None
    torch.manual_seed(1)
    x.data.copy_(torch.randn(8, 64))
    for w in ws:
        w.data.copy_(torch.randn(32, 64))
    with torch.autocast("cpu", dtype=torch.bfloat16):
        a, b = F.linear(x, ws[0]), F.linear(x, ws[1])
        c = F.linear(x, ws[1])
        d = torch.randn(8, 32) + F.linear(x, ws[0])
        loss = (a.float().sum() + b.float().square().sum() + c.float().mean() + d.float().sum())
    loss.backward()
    for g, w in zip(got, [x.grad, ws[0].grad, ws[1].grad]):
        torch.testing.assert_close(g, w, rtol=0, atol=0)


def test_grad_targets_are_weak():
    """A registered gradient target is held weakly: dropping the owner's views frees them, and a
    dead registration falls back to a plain dW."""
    w = torch.randn(4, 8, requires_grad=True)
    views = [torch.zeros(4, 8)]
    L.set_grad_targets([w], views)
    ref = weakref.ref(views[0])
    del views
    assert ref() is None  # the registry did not keep the bucket view alive
    x = torch.randn(3, 8)
    L.linear(x, w).sum().backward()
    torch.testing.assert_close(w.grad, torch.ones(3, 4).t() @ x)
