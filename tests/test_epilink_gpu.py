"""EpiLink extra-consumer safety: a third consumer of a bottleneck output (a forward
hook feeding an auxiliary loss) must not be skipped by the linked backward (conv1's GEMM epilogue
masks and reduces the producer's BN-backward partials for the two consumers it knows about).
With the check, the linked model's gradients match the unlinked model's (XDDP_CONV_EPI=0) to
bf16 noise, while the auxiliary term itself moves them far more than that noise."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _grads(epi: str, aux: float):
    from distributeddataparallel_amd.models import resnet50
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    os.environ["XDDP_CONV_EPI"] = epi
    try:
        torch.manual_seed(0)
        m = resnet50(norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        with torch.no_grad():  # well-conditioned residual branches (see test_headline_gpu.py)
            for name, mod in m.named_modules():
                if name.endswith("bn3"):
                    mod.weight.fill_(0.2)
        feats = []

        def hook(_mod, _inp, out):
            feats.append(out[0] if isinstance(out, tuple) else out)

        h = m.layer2[1].register_forward_hook(hook)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(8, 3, 96, 96, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (8,), device="cuda", generator=g)
        loss = F.cross_entropy(m(x).float(), y) + aux * feats[0].float().mean()
        loss.backward()
        h.remove()
        return {n: p.grad.float().clone() for n, p in m.named_parameters() if n.startswith(("conv1", "layer1", "layer2"))}
    finally:
        os.environ.pop("XDDP_CONV_EPI", None)


def _rel(a, b):
    num = sum((a[n] - b[n]).norm() ** 2 for n in a) ** 0.5
    den = sum(b[n].norm() ** 2 for n in b) ** 0.5
    return (num / den).item()


def test_extra_consumer_of_linked_block_output():
    linked, unlinked = _grads("1", 60.0), _grads("0", 60.0)
    no_aux = _grads("1", 0.0)
    path_noise, aux_effect = _rel(linked, unlinked), _rel(no_aux, unlinked)
    print(f"\nlinked vs unlinked rel {path_noise:.4f}; aux-term effect {aux_effect:.4f}")
    assert aux_effect > 0.1, aux_effect  # the auxiliary gradient is a large part of these grads
    assert path_noise < 0.25 * aux_effect, (path_noise, aux_effect)
