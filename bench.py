#!/usr/bin/env python
"""Headline benchmark: ResNet-50 bf16 data-parallel training throughput (images/s, whole job).

BASELINE.json metric: "images/sec (whole node) ResNet-50 DDP at 1/2/4/8 MI355X; scaling
efficiency", config "ResNet-50 bf16 DDP on 8×MI355X, synthetic ImageNet-shaped input".

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``. W untimed steps, then
exactly K timed steps bracketed by barrier + synchronize on both sides; the MAX elapsed over
ranks is reported; rank 0 prints ONE JSON line. Weak scaling: the per-GPU batch is fixed as N
grows. Launch modes for N>1 (one rank per GPU over RCCL):

* under ``torch.distributed.run`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in the env);
* directly (``python bench.py --gpus N``): the parent starts N fresh child processes with
  RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT set — before touching the GPU — forwards
  rank 0's JSON line and exits non-zero if any child fails (the reference's own launch model:
  ``world_size = device_count()`` + ``mp.spawn``, ``ref:dpp.py:60-62``).

Each step is a full training step: synthetic batch already on the device, forward,
cross-entropy, backward with bucketed RCCL all-reduce overlapped with backward (xddp Reducer),
fused SGD (momentum 0.9, wd 1e-4, fp32 master weights) — nothing skipped. Besides the headline
number the JSON reports what the communicator saw (``nranks``), the rebuilt bucket layout, the
Reducer's sampled backward comm / overlap times (measured AFTER the timed region, in extra
diagnostic steps, so the timed loop is untouched), the achieved all-reduce bus bandwidth per
bucket size (N>1), model-FLOPs utilisation, and, given ``--baseline-json`` of the N=1 run, the
scaling efficiency.

CPU rehearsal of the same paths: ``python bench.py --gpus 2 --device cpu --backend cpu --model mlp``.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity)
FP32_DENSE_PEAK_TFLOPS = 157.3  # MI355X dense fp32 MFMA peak
LR_WARMUP_STEPS = 30  # linear lr warmup (optimizer steps)
LOSS_GUARD = 1.1  # warn when the final loss ends above 1.1x the first step's
REPLICA_DIVERGED = 3  # exit code of a run whose ranks' parameters differ after the timed steps


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch-size", type=int, default=None, help="per-rank (micro-)batch")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--backend", default=None, help="xddp backend: rccl (GPU default), peer (IPC peer memory, "
                    "ranks may share a GPU) or cpu")
    ap.add_argument("--impl", choices=["xddp", "torch"], default="xddp",
                    help="xddp = this framework; torch = torch.nn.parallel.DDP reference stack (comparison only)")
    ap.add_argument("--norm", choices=["xddp", "torch"], default="xddp", help="BatchNorm implementation")
    ap.add_argument("--bucket-cap-mb", type=float, default=None,
                    help="explicit cap = reference bucketing; default = xGMI bucket policy")
    ap.add_argument("--bucket-policy", default=None, help="xgmi | reference")
    ap.add_argument("--comm-dtype", default="none", help="gradient comm dtype (none = param dtype)")
    ap.add_argument("--grad-as-bucket-view", type=int, default=1)
    ap.add_argument("--channels-last", type=int, default=1)
    ap.add_argument("--no-sync-accum", type=int, default=1,
                    help="micro-batches per optimizer step: k-1 under no_sync(), the last one syncs "
                         "(each micro-batch has --batch-size samples)")
    ap.add_argument("--seq-len", type=int, default=4096, help="LM configs: tokens per sequence")
    ap.add_argument("--checkpoint", type=int, default=0, help="activation checkpointing (transformers)")
    ap.add_argument("--graphs", type=int, default=0, help="replay the whole DDP step as one captured HIP graph")
    ap.add_argument("--diag-steps", type=int, default=3,
                    help="untimed steps after the timed region with comm timers on every step")
    ap.add_argument("--busbw-iters", type=int, default=5, help="all-reduce bandwidth probe iterations (N>1)")
    ap.add_argument("--probe-peer", type=int, default=None,
                    help="N>1: also probe the two-shot peer-memory all-reduce at the bucket sizes with a separate "
                         "peer instance (default: on at N>1 unless the comm calibration already timed that route)")
    ap.add_argument("--comm-calibrate", choices=["auto", "0", "1"], default="auto",
                    help="init-time comm calibration (XDDP_COMM_CALIBRATE; distributed/calibrate.py): peer-path "
                         "self-check, RCCL vs peer timings at the bucket sizes, fitted alpha / bus bandwidth for the "
                         "bucket policy, per-size route table. auto = on at N>1 on the rccl / peer backends")
    ap.add_argument("--baseline-json", default=None, help="N=1 result line -> scaling_efficiency")
    ap.add_argument("--launch-timeout", type=float, default=1500.0, help="self-launch: kill children after this")
    ap.add_argument("--tunableop", choices=["auto", "off", "use", "tune"], default="auto",
                    help="hipBLASLt/rocBLAS GEMM solution selection via torch TunableOp: use = the tuned "
                         "results shipped in tuning/tunableop (auto: for transformer models), tune = search "
                         "and write gpurun_out/tunableop_<model>.csv")
    ap.add_argument("--overlap-optim", choices=["auto", "0", "1"], default="auto",
                    help="run the optimizer inside backward on a side stream (DDP.register_overlapped_optimizer; "
                         "auto = on for AdamW (transformer) configs at N>1, off otherwise)")
    ap.add_argument("--overlap-schedule", choices=["tail", "backward"], default="tail",
                    help="tail: updates deferred under the chunked tail all-reduce; backward: each bucket's "
                         "update right after its own all-reduce")
    ap.add_argument("--force-rccl-launch", type=int, default=0,
                    help="issue real RCCL kernels even at N=1 (XDDP_RCCL_FORCE_LAUNCH): the comm-stream "
                         "schedule becomes visible in a one-GPU kernel trace")
    ap.add_argument("--dtype", choices=["auto", "bf16", "fp32"], default="auto",
                    help="parameter / activation dtype (auto: bf16 on the GPU, fp32 on the CPU)")
    ap.add_argument("--optimizer", choices=["auto", "sgd", "adamw"], default="auto",
                    help="auto: SGD for the conv / MLP configs, AdamW for the transformers")
    ap.add_argument("--lr", type=float, default=None, help="default 0.1 (SGD) / 1e-4 (AdamW)")
    ap.add_argument("--momentum", type=float, default=0.9, help="SGD momentum")
    ap.add_argument("--weight-decay", type=float, default=None, help="default 1e-4 (SGD) / 0.1 (AdamW)")
    ap.add_argument("--lr-warmup", type=int, default=None,
                    help=f"linear lr warmup steps (default {30}; 0 = constant lr)")
    ap.add_argument("--recipe", choices=["default", "reference"], default="default",
                    help="reference = the reference script's own recipe (ref:dpp.py:38-41): fp32, plain "
                         "SGD(lr=0.01) without momentum / weight decay / master copy / warmup")
    ap.add_argument("--accurate-convs", type=int, default=0,
                    help="fp32: MIOpen's implicit-GEMM conv solvers off (fp32-accurate weight gradients, but the "
                         "channels_last fallback runs ~6x slower; utils/precision.py)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)
    if a.recipe == "reference":
        a.dtype, a.optimizer, a.lr, a.momentum, a.weight_decay, a.lr_warmup = "fp32", "sgd", 0.01, 0.0, 0.0, 0
    if a.batch_size is None:
        # LM configs: one 4096-token sequence per rank (Llama-3-8B pure DDP sizing on 288 GB)
        a.batch_size = 1 if a.model.startswith("llama") else {"mlp": 64, "simplecnn": 32}.get(a.model, 256)
    if a.backend is None:
        a.backend = "rccl" if a.device == "cuda" else "cpu"
    return a


# ------------------------------------------------------------------------------ self-launch
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child_preexec():
    try:  # children die with the parent (PR_SET_PDEATHSIG = SIGTERM)
        import ctypes

        ctypes.CDLL("libc.so.6").prctl(1, signal.SIGTERM)
    except OSError:
        pass


def self_launch(args, argv) -> int:
    """Start one fresh child per rank; never touches the GPU in this (parent) process."""
    n = args.gpus
    port = _free_port()
    procs = []
    json_lines = []

    def pump(stream):
        for raw in iter(stream.readline, b""):
            line = raw.decode(errors="replace")
            if line.startswith('{"metric"'):
                json_lines.append(line.strip())
            else:
                sys.stderr.write(line)
                sys.stderr.flush()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), XDDP_BENCH_CHILD="1")
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                             stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                             preexec_fn=_child_preexec)
        procs.append(p)
    t = threading.Thread(target=pump, args=(procs[0].stdout,), daemon=True)
    t.start()
    deadline = time.time() + args.launch_timeout
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        # 3 = the rank finished but the replicas diverged: every rank exits that way after the same
        # collectives, so keep waiting for the others (rank 0 prints the JSON line) instead of killing
        bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0, REPLICA_DIVERGED)]
        if bad:
            failed = bad[0]
            break
        if all(c is not None for c in codes):
            diverged = [(i, c) for i, c in enumerate(codes) if c == REPLICA_DIVERGED]
            failed = diverged[0] if diverged else None
            break
        if time.time() > deadline:
            failed = (-1, "timeout")
            break
        time.sleep(0.2)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        end = time.time() + 10
        for p in procs:
            try:
                p.wait(max(0.1, end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if failed[1] == REPLICA_DIVERGED:
            print("[bench] the ranks' replicas diverged (exit 3; see replica_mismatch_ranks)", file=sys.stderr, flush=True)
        else:
            print(f"[bench] rank {failed[0]} failed ({failed[1]}); all ranks stopped", file=sys.stderr, flush=True)
    t.join(timeout=10)
    if json_lines:  # (also after a failure: a diverged-replica run still reports its line)
        print(json_lines[-1], flush=True)
    if failed is not None:
        return 1 if failed[1] == "timeout" else (failed[1] if isinstance(failed[1], int) and failed[1] > 0 else 1)
    return 0 if json_lines else 1


# ------------------------------------------------------------------------------ MIOpen tuning db
def _install_miopen_tuning():
    """MIOpen conv tuning (MI355X-specific): the repo ships a find-db + perf-db + kernel cache
    made by an exhaustive search on MI355X (tuning/miopen); each process copies it to a private
    temp dir (MIOpen writes to it) so first steps do not pay the search."""
    src = os.path.join(REPO, "tuning", "miopen")
    if os.environ.get("XDDP_MIOPEN_DB", "") == "none" or not os.path.isdir(src):
        return
    import shutil
    import tempfile

    dst = tempfile.mkdtemp(prefix=f"xddp_miopen_{os.environ.get('LOCAL_RANK', '0')}_")
    for sub, var in (("db", "MIOPEN_USER_DB_PATH"), ("cache", "MIOPEN_CUSTOM_CACHE_DIR")):
        if os.path.isdir(os.path.join(src, sub)) and var not in os.environ:
            shutil.copytree(os.path.join(src, sub), os.path.join(dst, sub))
            os.environ[var] = os.path.join(dst, sub)


def _install_tunableop(args):
    """GEMM tuning (MI355X-specific): torch's TunableOp benchmarks every rocBLAS/hipBLASLt
    solution for each GEMM shape once; the winners for the transformer configs are shipped in
    tuning/tunableop (made on MI355X with ``--tunableop tune``) and loaded read-only."""
    mode = args.tunableop
    if mode == "auto":
        mode = "use" if (args.model.startswith("vit") or is_lm(args)) else "off"
    if mode == "off" or args.device != "cuda":
        return None
    import shutil
    import tempfile

    name = f"tunableop_{args.model}.csv"
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    if mode == "tune":
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
        os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(REPO, "gpurun_out", name)
        return "tune"
    src = os.path.join(REPO, "tuning", "tunableop", name)
    if not os.path.isfile(src):
        os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "0"
        return None
    dst = os.path.join(tempfile.mkdtemp(prefix=f"xddp_tunableop_{os.environ.get('LOCAL_RANK', '0')}_"), name)
    shutil.copy(src, dst)
    # (torch may insert the device ordinal before the extension when it opens the file)
    shutil.copy(src, dst[:-4] + os.environ.get("LOCAL_RANK", "0") + ".csv")
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "0"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = dst
    return "use"


# ------------------------------------------------------------------------------ model / data
def is_lm(args):
    return args.model.startswith("llama")


def is_conv(args):
    return args.model.startswith("resnet") or args.model == "simplecnn"


def build_model(args, device, dtype):
    import torch

    from distributeddataparallel_amd import models

    if is_conv(args):
        norm_layer = None
        if args.norm == "xddp" and device.type == "cuda":
            from distributeddataparallel_amd.ops.batch_norm import FusedBatchNorm2d

            norm_layer = FusedBatchNorm2d
        if args.model == "simplecnn":  # the reference's model: ResNet-18 with a 10-class head
            m = models.SimpleCNN(norm_layer=norm_layer)
        else:
            m = getattr(models, args.model)(norm_layer=norm_layer)
    elif args.model.startswith("vit"):
        m = getattr(models, args.model)(checkpoint_activations=bool(args.checkpoint))
    elif args.model == "llama3_8b":
        with torch.device(device):
            m = models.llama3_8b(max_seq_len=args.seq_len, checkpoint_activations=bool(args.checkpoint))
    elif args.model == "llama_tiny":
        m = models.llama_tiny(max_seq_len=args.seq_len)
    elif args.model == "mlp":  # BASELINE.json config 1 (MNIST-shaped)
        m = models.MLP()
    else:
        raise SystemExit(f"unknown model {args.model}")
    m = m.to(device=device, dtype=dtype)
    if args.channels_last and is_conv(args) and device.type == "cuda":
        m = m.to(memory_format=torch.channels_last)
    return m


def sample_shape(args):
    if is_lm(args):
        return (args.seq_len,)
    if args.model == "mlp":
        return (1, 28, 28)
    return (3, args.image_size, args.image_size)


def num_classes(args, model):
    if is_lm(args):
        return model.cfg.vocab_size
    return 10 if args.model in ("simplecnn", "mlp") else 1000


def train_flops_per_sample(args):
    """Model FLOPs of one forward+backward per sample (torch FlopCounterMode on the meta device;
    plain torch ops, so the count is independent of which kernels run)."""
    import torch
    from torch.utils.flop_counter import FlopCounterMode

    from distributeddataparallel_amd import models

    try:
        nb = 1
        with torch.device("meta"):
            if is_conv(args):
                m = models.SimpleCNN() if args.model == "simplecnn" else getattr(models, args.model)()
                nb = 2  # (training-mode BatchNorm needs > 1 value per channel at a 1x1 feature map)
                x = torch.empty(nb, *sample_shape(args))
            elif args.model.startswith("vit"):
                m = getattr(models, args.model)()
                x = torch.empty(1, *sample_shape(args))
            elif args.model == "llama3_8b":
                m = models.llama3_8b(max_seq_len=args.seq_len)
                x = torch.zeros(1, args.seq_len, dtype=torch.long)
            elif args.model == "llama_tiny":
                m = models.llama_tiny(max_seq_len=args.seq_len)
                x = torch.zeros(1, args.seq_len, dtype=torch.long)
            else:
                m = models.MLP()
                x = torch.empty(1, *sample_shape(args))
        with FlopCounterMode(display=False) as fc:
            m(x).float().sum().backward()
        return float(fc.get_total_flops()) / nb
    except Exception as e:  # noqa: BLE001 — MFU is a diagnostic, never fail the bench over it
        print(f"[bench] flop count failed: {e}", file=sys.stderr)
        return None


# ------------------------------------------------------------------------------ main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    os.environ.setdefault("LOCAL_RANK", str(local_rank))
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(_free_port())
    if args.force_rccl_launch:
        os.environ["XDDP_RCCL_FORCE_LAUNCH"] = "1"
    if args.device == "cuda":
        _install_miopen_tuning()
    tunableop = _install_tunableop(args)
    sys.path.insert(0, REPO)
    if args.device == "cuda" and args.dtype == "fp32" and is_conv(args) and args.accurate_convs:
        # fp32 runs take MIOpen's convolutions: optionally fp32-accurate ones (utils/precision.py), both impls
        from distributeddataparallel_amd.utils.precision import accurate_fp32_convs

        accurate_fp32_convs()

    import torch
    import torch.nn.functional as F

    gpu = args.device == "cuda"
    dev_index = local_rank
    if gpu and args.backend in ("peer", "cpu"):  # these backends let several ranks share a GPU
        dev_index = local_rank % max(1, torch.cuda.device_count())
    if gpu:
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
        torch.backends.cudnn.benchmark = bool(int(os.environ.get("XDDP_CUDNN_BENCHMARK", "0")))
    else:
        device = torch.device("cpu")
    if args.dtype == "auto":
        args.dtype = "bf16" if gpu else "fp32"
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    if args.optimizer == "auto":
        args.optimizer = "sgd" if (is_conv(args) or args.model == "mlp") else "adamw"
    sgd = args.optimizer == "sgd"
    lr = args.lr if args.lr is not None else (0.1 if sgd else 1e-4)
    wd = args.weight_decay if args.weight_decay is not None else (1e-4 if sgd else 0.1)
    master = gpu and dtype != torch.float32  # fp32 master weights only for low-precision params
    warmup_steps = LR_WARMUP_STEPS if args.lr_warmup is None else args.lr_warmup

    def sync():
        if gpu:
            torch.cuda.synchronize()

    rccl_env = {}
    calib = args.comm_calibrate == "1" or (args.comm_calibrate == "auto" and world > 1 and gpu
                                           and args.backend in ("rccl", "peer") and args.impl == "xddp")
    if calib:
        # outside the timed region: runs once in the DDP constructor. The peer lanes are created on
        # probation and only used if every rank's self-check passes and they measure faster.
        os.environ.setdefault("XDDP_COMM_CALIBRATE", "1")
        if args.backend == "rccl":
            os.environ.setdefault("XDDP_PEER_ALLREDUCE", "auto")
    if args.probe_peer is None:
        args.probe_peer = int(world > 1 and not calib)
    if args.impl == "xddp":
        import distributeddataparallel_amd as xddp
        from distributeddataparallel_amd import distributed as dist
        from distributeddataparallel_amd.optim import FusedAdamW, FusedSGD
        from distributeddataparallel_amd.parallel.bucket_policy import rccl_env_defaults

        rccl_env = rccl_env_defaults(world, args.backend)
        dist.init_process_group(args.backend, device_id=dev_index if gpu else None)
    else:
        import torch.distributed as dist

        dist.init_process_group("nccl" if gpu else "gloo", device_id=device if gpu else None)

    torch.manual_seed(0)
    model = build_model(args, device, dtype)
    conv = is_conv(args)
    if args.impl == "xddp":
        comm_dtype = None if args.comm_dtype == "none" else getattr(torch, args.comm_dtype)
        ddp = xddp.DDP(model, device_ids=[dev_index] if gpu else None, bucket_cap_mb=args.bucket_cap_mb,
                       bucket_policy=args.bucket_policy, gradient_as_bucket_view=bool(args.grad_as_bucket_view),
                       comm_dtype=comm_dtype)
        if sgd:
            opt = FusedSGD(ddp.parameters(), lr=lr, momentum=args.momentum, weight_decay=wd, master_weights=master)
        else:
            opt = FusedAdamW(ddp.parameters(), lr=lr, weight_decay=wd, master_weights=True)
    else:
        ddp = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[local_rank] if gpu else None, bucket_cap_mb=args.bucket_cap_mb or 25,
            gradient_as_bucket_view=bool(args.grad_as_bucket_view))
        if sgd:
            opt = torch.optim.SGD(ddp.parameters(), lr=lr, momentum=args.momentum, weight_decay=wd)
        else:
            opt = torch.optim.AdamW(ddp.parameters(), lr=lr, weight_decay=wd)

    B = args.batch_size
    micro = max(1, args.no_sync_accum)
    # auto: at N=1 there is nothing to hide. At N>1 the last bucket's all-reduce is exposed
    # (Llama's 1.05 GB embedding gradient is ready last and forms the tail alone); the "tail"
    # schedule defers every other bucket's AdamW update until the tail's (chunked) collectives are
    # launched, so the updates run while the links carry the tail. (Updating during backward instead
    # measured no gain on one MI355X — Llama-3-8B 16,726 vs 16,779 tok/s, ViT-L/16 1,984 vs 1,970
    # img/s: hipBLASLt's backward GEMMs occupy every CU.)
    overlap_ok = args.impl == "xddp" and hasattr(opt, "step_params") and micro == 1 and not args.graphs
    overlap = args.overlap_optim == "1" or (args.overlap_optim == "auto" and world > 1 and overlap_ok)
    if overlap and not overlap_ok:
        raise SystemExit("--overlap-optim 1 needs the xddp DDP, an AdamW config, one micro-batch and no --graphs")
    if overlap:
        ddp.register_overlapped_optimizer(opt, schedule=args.overlap_schedule)
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    ncls = num_classes(args, model)
    if is_lm(args):
        xs = [torch.randint(0, ncls, (B, args.seq_len), device=device, generator=g) for _ in range(micro)]
        ys = [torch.randint(0, ncls, (B, args.seq_len), device=device, generator=g) for _ in range(micro)]
    else:
        mf = torch.channels_last if (args.channels_last and conv and gpu) else torch.contiguous_format
        xs = [torch.randn(B, *sample_shape(args), device=device, generator=g).to(dtype).contiguous(memory_format=mf)
              for _ in range(micro)]
        ys = [torch.randint(0, ncls, (B,), device=device, generator=g) for _ in range(micro)]

    from distributeddataparallel_amd.ops.cross_entropy import cross_entropy as fused_xent

    def loss_fn(out, tgt):
        if is_lm(args):
            # fp32 softmax cross-entropy over the bf16 logits without an fp32 copy of them
            # (ops/cross_entropy.py; --impl torch keeps F.cross_entropy on the upcast logits)
            flat, t = out.reshape(-1, out.shape[-1]), tgt.reshape(-1)
            if args.impl == "xddp" and os.environ.get("XDDP_FUSED_XENT", "1") != "0":
                return fused_xent(flat, t)
            return F.cross_entropy(flat.float(), t)
        return F.cross_entropy(out.float(), tgt)

    graphed = None
    if args.graphs:
        if micro > 1:
            raise SystemExit("--graphs does not combine with --no-sync-accum")
        from distributeddataparallel_amd.utils.graphs import GraphedTrainStep

        graphed = GraphedTrainStep(ddp, opt, loss_fn, xs[0], ys[0], warmup_steps=3)

    # Linear learning-rate warmup over the first LR_WARMUP_STEPS optimizer steps (Goyal et al.'s
    # large-batch recipe): lr 0.1 + momentum 0.9 from step 0 on a random-init ResNet-50 fitting a
    # fixed batch leaves the descent at step ~11 in torch fp32 as well
    # (profiles/r2_loss_curves_bench_config.txt). Host-side floats only: no kernel, no sync.
    base_lrs = [grp["lr"] for grp in opt.param_groups]
    n_opt_steps = [0]

    def set_lr():
        f = min(1.0, (n_opt_steps[0] + 1) / warmup_steps) if warmup_steps > 0 else 1.0
        for grp, lr in zip(opt.param_groups, base_lrs):
            grp["lr"] = lr * f
        n_opt_steps[0] += 1

    def step():
        if graphed is None:
            set_lr()
        if graphed is not None:
            return graphed(xs[0], ys[0])
        opt.zero_grad(set_to_none=True)
        for i in range(micro - 1):
            with ddp.no_sync():
                loss_fn(ddp(xs[i]), ys[i]).backward()
        loss = loss_fn(ddp(xs[-1]), ys[-1])
        loss.backward()
        if not overlap:  # (overlapped: every bucket was stepped during backward)
            opt.step()
        return loss

    first_loss = None
    traj = []  # every step's loss tensor (references only: no copy, no sync in the timed loop)
    for i in range(args.warmup):
        tw = time.perf_counter()
        loss = step()
        traj.append(loss.detach() if graphed is None else loss.detach().clone())
        if first_loss is None:
            first_loss = float(loss.float().item())
        if rank == 0:
            sync()
            print(f"[bench] warmup step {i + 1}/{args.warmup}: {time.perf_counter() - tw:.2f}s", file=sys.stderr,
                  flush=True)
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
        traj.append(loss.detach() if graphed is None else loss.detach().clone())
    host_elapsed = time.perf_counter() - t0  # the host's enqueue time: ~elapsed when the host bounds the step
    sync()
    dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    et = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(et, op=dist.ReduceOp.MAX)
    elapsed = float(et.item())
    final_loss = float(loss.float().item())
    lt = torch.stack([t.float().reshape(()) for t in traj]).cpu()
    loss_min, loss_max = float(lt.min()), float(lt.max())
    del traj

    # ---------------- replica check (outside the timed region): every rank's parameters and
    # buffers must be bit-identical after the timed steps (utils/replicas.py); a diverged run exits
    # non-zero and names the ranks
    replicas = None
    if args.impl == "xddp":
        if ddp.will_sync_module_buffers():
            ddp._sync_buffers()  # BN running stats took local updates in the last forward
        replicas = ddp.check_replicas(max_diff=world > 1)
        if not replicas["replicas_identical"]:
            print(f"[bench] rank {rank}: REPLICAS DIVERGED: ranks {replicas['mismatch_ranks']} disagree with the "
                  f"majority (max |param - rank0 param| = {replicas['max_abs_diff']})", file=sys.stderr, flush=True)

    # ---------------- diagnostics (outside the timed region)
    diag = {}
    if args.impl == "xddp" and replicas["replicas_identical"]:
        diag = diagnostics(args, ddp, step, sync, dist, device, world, overlap)

    ms = elapsed / args.steps * 1e3
    per_step_samples = B * micro * world
    units = per_step_samples * args.steps * (args.seq_len if is_lm(args) else 1)
    value = units / elapsed
    if rank == 0:
        flops = train_flops_per_sample(args)
        if args.model == "resnet50":
            metric = "images/sec (whole node) ResNet-50 DDP at 1/2/4/8 MI355X; scaling efficiency"
        elif is_lm(args):
            metric = f"tokens/sec (whole node) {args.model} pure DDP"
        else:
            metric = f"images/sec (whole node) {args.model} DDP"
        eff = None
        if args.baseline_json:
            try:
                with open(args.baseline_json) as f:
                    base = json.loads(f.read().strip().splitlines()[-1])
                eff = round(value / (world * float(base["value"])), 4)
            except (OSError, ValueError, KeyError) as e:
                print(f"[bench] cannot read baseline {args.baseline_json}: {e}", file=sys.stderr)
        out = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "tokens/s" if is_lm(args) else "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "host_ms_per_step": round(host_elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": ("synthetic (random token ids; random-init weights)" if is_lm(args) else
                     f"synthetic (random {'x'.join(map(str, sample_shape(args)))} inputs, random labels; "
                     "random-init weights)"),
            "config": {
                "model": args.model,
                "global_batch": per_step_samples,
                "per_gpu_batch": B * micro,
                "micro_batch": B,
                "seq_len": args.seq_len if is_lm(args) else None,
                "image_size": args.image_size if (conv or args.model.startswith("vit")) else None,
                "parallelism": f"dp{world}",
                "impl": args.impl,
                "backend": args.backend if args.impl == "xddp" else ("nccl" if gpu else "gloo"),
                "norm": args.norm,
                "optimizer": (f"SGD(lr={lr:g}, momentum={args.momentum:g}, wd={wd:g})" if sgd
                              else f"AdamW(lr={lr:g}, wd={wd:g})") + (" fp32 master weights" if master else ""),
                "recipe": args.recipe,
                "miopen_implicit_gemm": os.environ.get("MIOPEN_DEBUG_CONV_IMPLICIT_GEMM", "default"),
                "optimizer_schedule": args.overlap_schedule if overlap else "after backward",
                "channels_last": bool(args.channels_last),
                "comm_dtype": args.comm_dtype,
                "gradient_as_bucket_view": bool(args.grad_as_bucket_view),
                "micro_batches": micro,
                "hip_graphs": bool(args.graphs),
                "rccl_env_defaults": rccl_env,
                "gemm_tuning": tunableop or "off",
            },
            "initial_loss": round(first_loss, 4) if first_loss is not None else None,
            "final_loss": round(final_loss, 4),
            "loss_min": round(loss_min, 4),
            "loss_max": round(loss_max, 4),
            "lr_warmup_steps": warmup_steps if graphed is None else 0,
            "scaling_efficiency": eff,
            "replicas_identical": None if replicas is None else replicas["replicas_identical"],
            "replica_mismatch_ranks": None if replicas is None else replicas["mismatch_ranks"],
            "replica_max_abs_diff": None if replicas is None else replicas["max_abs_diff"],
        }
        bad = [v for v in (final_loss, loss_max) if v != v or v in (float("inf"), float("-inf"))]
        if first_loss is not None and (bad or final_loss > LOSS_GUARD * first_loss):
            # divergence guard: the number is still a throughput, but say the training went wrong
            # (the run fits one fixed batch, so its loss should not end above where it started)
            out["warning"] = (f"loss diverged: final {final_loss:.4g} > {LOSS_GUARD}x the first step's "
                              f"{first_loss:.4g} (min {loss_min:.4g}, max {loss_max:.4g})")
        if flops:
            tf = flops * per_step_samples / (ms * 1e-3) / 1e12
            out["model_tflops_per_gpu"] = round(tf / world, 1)
            peak = BF16_DENSE_PEAK_TFLOPS if dtype == torch.bfloat16 else FP32_DENSE_PEAK_TFLOPS
            out["mfu"] = round(tf / world / peak, 4) if gpu else None
            out["mfu_peak_tflops"] = peak if gpu else None
        out.update(diag)
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    dist.destroy_process_group()  # (TunableOp writes its results file at process exit)
    if replicas is not None and not replicas["replicas_identical"]:
        return REPLICA_DIVERGED  # every rank: the run's parameters diverged (see the JSON line / stderr)
    return 0


def diagnostics(args, ddp, step, sync, dist, device, world, overlap=False):
    """Comm observability: communicator rank count, rebuilt buckets, sampled
    backward comm / overlap (Reducer hipEvent timers on every diagnostic step), and the
    achieved all-reduce bus bandwidth of each bucket size when N>1."""
    import torch

    red = ddp.reducer
    pg = ddp.process_group
    out = {"nranks": int(pg.comm.size()), "comm_backend": pg.backend}
    sizes = list(red.bucket_sizes_bytes())
    out["buckets"] = {"count": len(sizes), "bytes": sizes, **ddp.bucket_plan.as_dict()}
    from distributeddataparallel_amd.parallel.bucket_policy import tail_report

    ost = getattr(ddp, "_overlap_state", None)
    out["buckets"]["tail"] = tail_report(sizes, ddp.bucket_plan, world, args.overlap_schedule if overlap else None,
                                         ost["last_chunks"] if ost else 0)
    # what the communicator itself reports (RCCL at N>1: version, ranks, channels and rings parsed
    # from its init log) and every rank's device
    info = pg.comm_info()
    if world > 1:
        dev = torch.tensor([device.index if device.type == "cuda" else -1], dtype=torch.long, device=device)
        allv = torch.zeros(world, dtype=torch.long, device=device)
        pg.allgather_into_tensor(allv, dev).wait()
        info["rank_devices"] = [int(v) for v in allv.tolist()]
    out["comm_info"] = info
    out["comm_calibration"] = getattr(ddp, "comm_calibration", None)
    if args.graphs or args.diag_steps <= 0:
        return out
    red.reset_runtime_stats()
    ddp._set_ddp_runtime_logging_sample_rate(1)
    for _ in range(args.diag_steps + 1):  # the last step harvests the previous one's timers
        step()
        sync()  # timers are harvested at the next forward only once their events completed
    d = ddp._get_ddp_logging_data()
    launched = int(d.get("num_collectives_launched") or 0)
    ms = lambda k: None if d.get(k) is None else round(d[k] / 1e6, 3)  # noqa: E731
    # Comm = the collectives' own durations (hipEvents on the comm stream); exposed = backward end
    # (last bucket launched) -> finalize end. Nothing is reported as comm when no collective crossed
    # a link (N=1: every collective is a local identity).
    comm = ms("avg_backward_comm_time") if launched else None
    ov = ms("avg_backward_compute_comm_overlap_time") if launched else None
    out["comm"] = {
        "collectives_launched": launched,
        "avg_backward_compute_ms": ms("avg_backward_compute_time"),
        "avg_backward_comm_ms": comm,
        "avg_overlap_ms": ov,
        "exposed_comm_ms": ms("avg_backward_exposed_comm_time") if launched else None,
        "overlap_pct": round(100.0 * ov / comm, 1) if (launched and comm) else None,
        "per_bucket_comm_ms": [round(t / 1e6, 4) for t in d.get("bucket_comm_times", [])] if launched else None,
        "timed_iterations": int(d.get("num_timed_iterations") or 0),
        "grouped_launches": int(d.get("num_grouped_launches") or 0),
    }
    ddp._set_ddp_runtime_logging_sample_rate(100)
    if world > 1 and args.busbw_iters > 0:
        dt = next(p for p in ddp.module.parameters()).dtype
        if ddp._comm_dtype is not None:
            dt = ddp._comm_dtype
        esz = torch.empty(0, dtype=dt).element_size()

        def probe(run, nbytes):
            buf = torch.ones(max(1, nbytes // esz), dtype=dt, device=device)
            for _ in range(2):
                run(buf)
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.busbw_iters):
                run(buf)
            sync()
            t = (time.perf_counter() - t0) / args.busbw_iters
            tt = torch.tensor([t], dtype=torch.float64, device=device)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
            return {"bytes": nbytes, "ms": round(t * 1e3, 4),
                    "busbw_GBps": round(2.0 * (world - 1) / world * nbytes / t / 1e9, 1)}

        out["allreduce_busbw"] = [probe(lambda b: pg.allreduce(b, dist.ReduceOp.AVG).wait(), n)
                                  for n in sorted(set(sizes))]
        if args.probe_peer and pg.backend == "rccl" and device.type == "cuda" and world <= 8:
            # the same sizes through the two-shot peer-memory all-reduce (all 7 xGMI links)
            from distributeddataparallel_amd._native import load

            C = load()
            peer = C.PeerAllReduce(C.PrefixStore("bench_peer", pg.store), pg.rank(), world, device.index,
                                   1 << 20, 64 << 20, 60.0)
            try:
                out["peer_two_shot_busbw"] = [probe(lambda b: peer.allreduce_two_shot(b, 1), n)
                                              for n in sorted(set(sizes))]
                if peer.status() != 0:
                    out["peer_two_shot_busbw"] = "timed out"
            finally:
                sync()
                peer.close()
    return out


if __name__ == "__main__":
    sys.exit(main())
