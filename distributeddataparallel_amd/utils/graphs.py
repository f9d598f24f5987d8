"""HIP-graph capture of a whole DDP training step (forward, backward with bucketed RCCL
all-reduces, optimizer step) — "HIP streams and graphs instead of a tracing compiler".

Small-batch data-parallel steps (the reference's own workload: ResNet-18 on 32x32 CIFAR,
batch 32 per GPU, ``ref:dpp.py``) issue hundreds of short kernels per step and are bound by
launch latency; replaying one captured graph removes that host cost.

Requirements (checked where possible):
  * static shapes; ``find_unused_parameters=False`` (its bitmap needs a host read);
  * buckets already rebuilt — done by the eager warmup steps run here before capture;
  * an optimizer whose step is pure device work (``FusedSGD``, torch SGD/momentum);
  * the Reducer's collectives go to the RCCL comm stream, which joins the capture through an
    event wait and rejoins the compute stream before the end of the step;
  * MIOpen in immediate mode (``cudnn.benchmark`` off during warmup + capture; the solutions are
    compiled by the eager warmup steps and replayed from the graph). With Find/benchmark mode a
    captured ResNet stem conv (3 input channels) got MIOpen's ASM V4R1 implicit-GEMM solver on
    some MI355X boxes and returned NaN weight gradients from the second replay on — reproduced with
    a plain torch model, torch SGD and ``torch.cuda.graph`` (no xddp code); disabling those
    solvers or benchmark mode fixes it (scripts/dbg/graph_dbg.py, scripts/dbg/gpu_graph_env.sh).
    ``XDDP_GRAPH_CUDNN_BENCHMARK=1`` opts back into Find mode.
"""
from __future__ import annotations

import os
from typing import Callable

import torch


class GraphedTrainStep:
    def __init__(self, model, optimizer, loss_fn: Callable, example_input: torch.Tensor,
                 example_target: torch.Tensor, warmup_steps: int = 3, set_to_none: bool = True):
        if getattr(model, "find_unused_parameters", False):
            raise ValueError("HIP-graph capture needs find_unused_parameters=False")
        self.model, self.optimizer, self.loss_fn = model, optimizer, loss_fn
        self.static_input = example_input.clone()
        self.static_target = example_target.clone()
        prev_bench = torch.backends.cudnn.benchmark
        torch.backends.cudnn.benchmark = os.environ.get("XDDP_GRAPH_CUDNN_BENCHMARK", "0") == "1"
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        if hasattr(model, "_rebind_grad_accumulators"):
            # AccumulateGrad nodes created at DDP construction run on the construction stream;
            # re-create them on the capture stream so backward stays inside the capture
            model._rebind_grad_accumulators(side)
        with torch.cuda.stream(side):
            for _ in range(max(2, warmup_steps)):  # >=2: bucket rebuild happens in iteration 1
                optimizer.zero_grad(set_to_none=set_to_none)
                loss_fn(model(self.static_input), self.static_target).backward()
                optimizer.step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        optimizer.zero_grad(set_to_none=set_to_none)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: the communicator's watchdog thread keeps polling live (non-captured) work
        try:
            with torch.cuda.graph(self.graph, stream=side, capture_error_mode="thread_local"):
                self.static_loss = loss_fn(model(self.static_input), self.static_target)
                self.static_loss.backward()
                optimizer.step()
        finally:
            torch.backends.cudnn.benchmark = prev_bench

    def __call__(self, inputs: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if inputs.data_ptr() != self.static_input.data_ptr():
            self.static_input.copy_(inputs, non_blocking=True)
        if target.data_ptr() != self.static_target.data_ptr():
            self.static_target.copy_(target, non_blocking=True)
        self.graph.replay()
        return self.static_loss
