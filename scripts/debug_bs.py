"""Forward parity of the fused ResNet-50 vs torch bf16 at several batch sizes: per-stage output
relative error and the loss (same weights, same input)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    from distributeddataparallel_amd.models import resnet50
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    torch.manual_seed(0)
    fused = resnet50(norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    ref = resnet50().cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    ref.load_state_dict(fused.state_dict())
    names = ["maxpool", "layer1", "layer2", "layer3", "layer4"]
    for bs in [int(v) for v in os.environ.get("BS", "16,64,128,192,256").split(",")]:
        g = torch.Generator(device="cuda").manual_seed(1234)
        x = torch.randn(bs, 3, 224, 224, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (bs,), device="cuda", generator=g)
        acts = {}

        def mk(tag, name):
            def h(_m, _i, out):
                acts[(tag, name)] = (out[0] if isinstance(out, tuple) else out).float()
            return h

        hs = []
        for tag, m in (("f", fused), ("r", ref)):
            for n in names:
                hs.append(getattr(m, n).register_forward_hook(mk(tag, n)))
        # stem fused path has no maxpool module call: hook layer1 input instead
        with torch.no_grad():
            lf = F.cross_entropy(fused(x).float(), y).item()
            lr = F.cross_entropy(ref(x).float(), y).item()
        for h in hs:
            h.remove()
        errs = []
        for n in names:
            if ("f", n) in acts and ("r", n) in acts:
                a, b = acts[("f", n)], acts[("r", n)]
                errs.append(f"{n} {((a - b).norm() / (b.norm() + 1e-12)).item():.4f}")
        print(f"bs {bs}: loss fused {lf:.4f} torch-bf16 {lr:.4f} | " + " ".join(errs), flush=True)
        fused.zero_grad()


if __name__ == "__main__":
    main()
