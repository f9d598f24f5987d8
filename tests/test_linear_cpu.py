"""ops/linear.py on the CPU (fp32): ``multi_linear`` (one input, several weights, the input
gradient accumulated in GEMMs) and ``linear`` with a residual (one beta = 1 GEMM) match the plain
autograd composition of the same math."""
import torch
import torch.nn.functional as F

from distributeddataparallel_amd.ops.linear import linear, multi_linear


def test_multi_linear_matches_separate_linears():
    torch.manual_seed(0)
    x = torch.randn(2, 5, 16, dtype=torch.float64, requires_grad=True)
    ws = [torch.randn(n, 16, dtype=torch.float64, requires_grad=True) for n in (16, 8, 8)]
    outs = multi_linear(x, *ws)
    gs = [torch.randn_like(o) for o in outs]
    torch.autograd.backward(outs, gs)
    got = [x.grad.clone()] + [w.grad.clone() for w in ws]
    x.grad = None
    for w in ws:
        w.grad = None
    ref = [F.linear(x, w) for w in ws]
    for o, r in zip(outs, ref):
        torch.testing.assert_close(o, r)
    torch.autograd.backward(ref, gs)
    for a, b in zip(got, [x.grad] + [w.grad for w in ws]):
        torch.testing.assert_close(a, b)


def test_multi_linear_unused_output_and_frozen_weight():
    torch.manual_seed(1)
    x = torch.randn(3, 16, dtype=torch.float64, requires_grad=True)
    w1 = torch.randn(8, 16, dtype=torch.float64, requires_grad=True)
    w2 = torch.randn(4, 16, dtype=torch.float64)  # no grad wanted
    a, b = multi_linear(x, w1, w2)
    a.sum().backward()  # b unused: its gradient is None
    torch.testing.assert_close(x.grad, w1.sum(0).expand(3, 16))
    torch.testing.assert_close(w1.grad, x.detach().sum(0).expand(8, 16))


def test_linear_residual_is_one_gemm_with_the_same_gradients():
    torch.manual_seed(2)
    x = torch.randn(2, 5, 16, dtype=torch.float64, requires_grad=True)
    w = torch.randn(12, 16, dtype=torch.float64, requires_grad=True)
    r = torch.randn(2, 5, 12, dtype=torch.float64, requires_grad=True)
    y = linear(x, w, r)
    g = torch.randn_like(y)
    y.backward(g)
    got = (x.grad.clone(), w.grad.clone(), r.grad.clone())
    x.grad = w.grad = r.grad = None
    yr = r + F.linear(x, w)
    torch.testing.assert_close(y, yr)
    yr.backward(g)
    for a, b in zip(got, (x.grad, w.grad, r.grad)):
        torch.testing.assert_close(a, b)
