"""Fused softmax cross-entropy (csrc/kernels/cross_entropy.hip via ops/cross_entropy.py) vs fp32
PyTorch F.cross_entropy on the upcast logits: loss and logits gradient, with ignored rows, at a
small vocabulary and at Llama-3's 128,256 classes."""
import pytest
import torch
import torch.nn.functional as F

from distributeddataparallel_amd.ops.cross_entropy import cross_entropy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,vocab,scale", [(64, 1000, 3.0), (37, 128256, 2.0), (8, 4096, 30.0)])
def test_cross_entropy_matches_fp32_torch(rows, vocab, scale):
    torch.manual_seed(0)
    x = (torch.randn(rows, vocab, device="cuda") * scale).to(torch.bfloat16)
    t = torch.randint(0, vocab, (rows,), device="cuda")
    t[::5] = -100  # ignored rows
    a = x.clone().requires_grad_(True)
    loss = cross_entropy(a, t)
    loss.backward()
    b = x.clone().requires_grad_(True)
    ref = F.cross_entropy(b.float(), t)
    ref.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    assert a.grad.dtype == torch.bfloat16
    torch.testing.assert_close(a.grad.float(), b.grad.float(), rtol=2e-2, atol=1e-2 * b.grad.abs().max().item())
    assert torch.equal(a.grad[::5], torch.zeros_like(a.grad[::5]))  # ignored rows: no gradient


def test_cross_entropy_scaled_upstream_gradient():
    torch.manual_seed(1)
    x = torch.randn(16, 512, device="cuda").to(torch.bfloat16)
    t = torch.randint(0, 512, (16,), device="cuda")
    a = x.clone().requires_grad_(True)
    (3.0 * cross_entropy(a, t)).backward()
    b = x.clone().requires_grad_(True)
    (3.0 * F.cross_entropy(b.float(), t)).backward()
    torch.testing.assert_close(a.grad.float(), b.grad.float(), rtol=2e-2, atol=1e-2 * b.grad.abs().max().item())


def test_cross_entropy_out_of_range_target_raises():
    """A target outside [0, V) that is not ignore_index: NaN loss at once, IndexError at the next
    check (torch raises too); ignore_index rows stay legal."""
    from distributeddataparallel_amd.ops.cross_entropy import check_targets

    check_targets(block=True)  # clean slate
    x = torch.randn(8, 512, device="cuda").to(torch.bfloat16)
    t = torch.randint(0, 512, (8,), device="cuda")
    t[3] = 512
    t[5] = -100
    loss = cross_entropy(x.clone().requires_grad_(True), t)
    assert torch.isnan(loss).item()
    with pytest.raises(IndexError, match="out of bounds"):
        check_targets(block=True)
    check_targets(block=True)  # the flag was consumed
    t[3] = -7
    cross_entropy(x, t)
    torch.cuda.synchronize()
    with pytest.raises(IndexError):
        cross_entropy(x, torch.zeros(8, dtype=torch.long, device="cuda"))  # raised lazily by the next call


def test_cross_entropy_captures_in_hip_graph():
    """The fused cross-entropy inside a HIP-graph capture (bench.py --graphs on an LM config): no
    event query / record or host copy during capture, and replays reproduce the eager loss and
    gradient for new data copied into the static inputs."""
    torch.manual_seed(2)
    rows, vocab = 32, 2048
    x = (torch.randn(rows, vocab, device="cuda") * 2).to(torch.bfloat16).requires_grad_(True)
    t = torch.randint(0, vocab, (rows,), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm up outside the capture
        for _ in range(2):
            x.grad = None
            cross_entropy(x, t).backward()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    x.grad = None
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        loss = cross_entropy(x, t)
        loss.backward()
    for seed in (3, 4):
        torch.manual_seed(seed)
        with torch.no_grad():
            x.copy_((torch.randn(rows, vocab, device="cuda") * 2).to(torch.bfloat16))
        t.copy_(torch.randint(0, vocab, (rows,), device="cuda"))
        g.replay()
        torch.cuda.synchronize()
        b = x.detach().clone().requires_grad_(True)
        ref = F.cross_entropy(b.float(), t)
        ref.backward()
        torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(x.grad.float(), b.grad.float(), rtol=2e-2, atol=1e-2 * b.grad.abs().max().item())
