"""The reference workload (``ref:dpp.py``) on xddp: ResNet-18 with a 10-class head, CIFAR-10,
DistributedSampler, batch 32/rank, SGD(lr=0.01), CrossEntropy, rank-0 loss log every 100
batches — one process per GPU over RCCL (or per CPU rank over the native CPU backend).

Differences from the reference, by design: no pretrained-weight or
dataset download (random init; CIFAR-10 *binary* files are used if present under --data,
otherwise a synthetic CIFAR-shaped dataset), MASTER_ADDR/PORT defaulted, device bound per
rank, optional checkpointing.

    python -m distributeddataparallel_amd.run --nproc-per-node 8 examples/train_ddp_cifar.py
    python examples/train_ddp_cifar.py --spawn 2 --backend cpu --epochs 1 --max-steps 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

import distributeddataparallel_amd as xddp  # noqa: E402
from distributeddataparallel_amd import distributed as dist  # noqa: E402
from distributeddataparallel_amd.data import CIFAR10Binary, DistributedSampler, SyntheticImages  # noqa: E402
from distributeddataparallel_amd.models import SimpleCNN  # noqa: E402
from distributeddataparallel_amd.utils.checkpoint import load_checkpoint, save_checkpoint  # noqa: E402
from distributeddataparallel_amd.utils.precision import accurate_fp32_convs  # noqa: E402


def train(rank, args):
    backend = args.backend or ("rccl" if torch.cuda.is_available() else "cpu")
    if backend != "cpu" and args.accurate_convs:
        accurate_fp32_convs()  # fp32-accurate MIOpen convolutions (utils/precision.py), before the first conv
    if args.impl == "torch":  # the reference's own stack, for parity runs (torch DDP + torch BN, NCHW)
        return train_torch(rank, args, backend)
    dist.init_process_group(backend)
    world = dist.get_world_size()
    torch.manual_seed(0)
    dataset = CIFAR10Binary(args.data) if CIFAR10Binary.available(args.data) else SyntheticImages(
        length=args.synthetic_len, shape=(3, 32, 32))
    sampler = DistributedSampler(dataset, num_replicas=world, rank=dist.get_rank(), shuffle=True)
    loader = DataLoader(dataset, batch_size=args.batch_size, sampler=sampler, num_workers=args.workers,
                        pin_memory=backend == "rccl")
    device = torch.device("cuda", torch.cuda.current_device()) if backend == "rccl" else torch.device("cpu")
    use_fused = backend == "rccl"
    if use_fused:
        from distributeddataparallel_amd.ops import FusedBatchNorm2d

        model = SimpleCNN(norm_layer=FusedBatchNorm2d).to(device).to(memory_format=torch.channels_last)
    else:
        model = SimpleCNN().to(device)
    model = xddp.DDP(model, device_ids=[device.index] if use_fused else None)
    criterion = nn.CrossEntropyLoss()
    optimizer = torch.optim.SGD(model.parameters(), lr=args.lr)
    start_epoch = 0
    if args.resume and os.path.exists(args.resume):
        st = load_checkpoint(args.resume, model, optimizer, map_location=device)
        start_epoch = (st.get("step") or 0) + 1
    step = 0
    for epoch in range(start_epoch, args.epochs):
        model.train()
        sampler.set_epoch(epoch)
        for batch_idx, (data, target) in enumerate(loader):
            data = data.to(device, non_blocking=True)
            if use_fused:
                data = data.contiguous(memory_format=torch.channels_last)
            target = target.to(device, non_blocking=True)
            optimizer.zero_grad()
            loss = criterion(model(data), target)
            loss.backward()
            optimizer.step()
            if batch_idx % args.log_every == 0 and dist.get_rank() == 0:
                print(f"Epoch {epoch}, Batch {batch_idx}, Loss: {loss.item()}", flush=True)
            step += 1
            if args.max_steps and step >= args.max_steps:
                break
        if args.checkpoint:
            save_checkpoint(args.checkpoint, model, optimizer, step=epoch)
    dist.destroy_process_group()


def train_torch(rank, args, backend):
    """The same loop on torch.nn.parallel.DistributedDataParallel over torch.distributed (nccl =
    RCCL on ROCm, or gloo), with torch's BatchNorm2d in NCHW: the reference script's stack."""
    import torch.distributed as tdist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29512")
    gpu = backend != "cpu"
    tdist.init_process_group("nccl" if gpu else "gloo", rank=int(os.environ.get("RANK", rank)),
                             world_size=int(os.environ.get("WORLD_SIZE", 1)))
    world = tdist.get_world_size()
    torch.manual_seed(0)
    dataset = CIFAR10Binary(args.data) if CIFAR10Binary.available(args.data) else SyntheticImages(
        length=args.synthetic_len, shape=(3, 32, 32))
    sampler = DistributedSampler(dataset, num_replicas=world, rank=tdist.get_rank(), shuffle=True)
    loader = DataLoader(dataset, batch_size=args.batch_size, sampler=sampler, num_workers=args.workers)
    device = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    model = torch.nn.parallel.DistributedDataParallel(SimpleCNN().to(device),
                                                      device_ids=[device.index] if gpu else None)
    criterion = nn.CrossEntropyLoss()
    optimizer = torch.optim.SGD(model.parameters(), lr=args.lr)
    step = 0
    for epoch in range(args.epochs):
        sampler.set_epoch(epoch)
        for batch_idx, (data, target) in enumerate(loader):
            data, target = data.to(device), target.to(device)
            optimizer.zero_grad()
            loss = criterion(model(data), target)
            loss.backward()
            optimizer.step()
            if batch_idx % args.log_every == 0 and tdist.get_rank() == 0:
                print(f"Epoch {epoch}, Batch {batch_idx}, Loss: {loss.item()}", flush=True)
            step += 1
            if args.max_steps and step >= args.max_steps:
                break
    tdist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--data", default="data")
    ap.add_argument("--synthetic-len", type=int, default=50000)
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--backend", default=None)
    ap.add_argument("--spawn", type=int, default=0, help="spawn N local ranks (mp.spawn-style) instead of a launcher")
    ap.add_argument("--max-steps", type=int, default=0)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--resume", default=None)
    ap.add_argument("--log-every", type=int, default=100, help="rank-0 loss print interval (reference: 100)")
    ap.add_argument("--accurate-convs", action="store_true",
                    help="MIOpen's implicit-GEMM fp32 conv solvers off: fp32-accurate weight gradients, slower "
                         "channels_last convs (utils/precision.py)")
    ap.add_argument("--impl", choices=["xddp", "torch"], default="xddp",
                    help="torch = torch DDP + torch BatchNorm (the reference stack), for parity runs")
    args = ap.parse_args()
    if args.spawn:
        from distributeddataparallel_amd.utils.spawn import spawn

        spawn(train, args=(args,), nprocs=args.spawn)
    else:
        train(int(os.environ.get("RANK", 0)), args)


if __name__ == "__main__":
    main()
