"""Loss curves of the bench configuration (ResNet-50, one fixed synthetic batch of 256 random
images / random labels, SGD lr 0.1 momentum 0.9 wd 1e-4, no warmup) for three stacks from the
same initial weights: xddp (fused kernels + DDP Reducer + FusedSGD with fp32 master weights),
torch bf16 (nn.BatchNorm2d, MIOpen, torch SGD on bf16 params) and torch fp32. Explains the
bench's final_loss: lr 0.1 without warmup on a random-init ResNet-50 is unstable at first in
every stack; the loss spikes above ln(1000) before the batch is memorized."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

STEPS = int(os.environ.get("STEPS", "40"))


def main():
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as dist
    from distributeddataparallel_amd.models import resnet50
    from distributeddataparallel_amd.ops import FusedBatchNorm2d
    from distributeddataparallel_amd.optim import FusedSGD
    from distributeddataparallel_amd.utils.spawn import free_port

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
    g = torch.Generator(device="cuda").manual_seed(1234)
    x = torch.randn(256, 3, 224, 224, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (256,), device="cuda", generator=g)
    torch.manual_seed(0)
    fused = resnet50(norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    sd = {k: v.detach().clone() for k, v in fused.state_dict().items()}  # (the live tensors get trained)
    curves = {}

    ddp = xddp.DDP(fused, device_ids=[0], gradient_as_bucket_view=True)
    opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, master_weights=True)
    la = []
    for _ in range(STEPS):
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(ddp(x).float(), y)
        loss.backward()
        opt.step()
        la.append(loss.item())
    curves["xddp bf16"] = la
    del ddp, opt, fused
    torch.cuda.empty_cache()

    for name, dtype in (("torch bf16", torch.bfloat16), ("torch fp32", torch.float32)):
        m = resnet50().cuda().to(dtype).to(memory_format=torch.channels_last)
        m.load_state_dict({k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()})
        o = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        xx = x.to(dtype)
        lb = []
        for _ in range(STEPS):
            o.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(xx).float(), y)
            loss.backward()
            o.step()
            lb.append(loss.item())
        curves[name] = lb
        del m, o
        torch.cuda.empty_cache()
    dist.destroy_process_group()
    print(f"# ResNet-50 bs256 fixed batch, SGD lr 0.1 momentum 0.9 wd 1e-4, {STEPS} steps, same init")
    print("step " + " ".join(f"{k:>11s}" for k in curves))
    for i in range(STEPS):
        print(f"{i:4d} " + " ".join(f"{curves[k][i]:11.3f}" for k in curves))


if __name__ == "__main__":
    main()
