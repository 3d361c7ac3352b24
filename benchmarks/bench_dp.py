#!/usr/bin/env python3
"""Data-parallel training-step benchmark (BASELINE.json configs 4 and 5):

  resnet50   - ResNet-50-shaped gradient set (25.6 M params, 161 tensors)
  llama3_8b  - Llama-3-8B gradient set (8.03 B params, 16.06 GB bf16), bucket-fused

Each step: a synthetic backward that produces every gradient with a real GEMM
(grad[out, in] = dY^T X over `--tokens` rows, in reverse parameter order - the order
autograd produces them), the bucketed reducer allreducing full buckets on its own stream
while later gradients are still being computed, then an SGD update. Reported per step:
total time, compute-only time (same step without communication), communication-only time
(allreduce of all buckets back to back) and the exposed communication = total - compute.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/bench_dp.py --model llama3_8b
    python benchmarks/bench_dp.py --model resnet50            # 1 GPU (allreduce is a no-op)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.models.grad_sets import gradient_shapes, numel  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import BucketedGradReducer, TorchDistComm, XgmiCommunicator  # noqa: E402
from akka_allreduce_1_amd.parallel.comm import init_distributed  # noqa: E402


def gemm_shape(shape: tuple[int, ...]) -> tuple[int, int]:
    if len(shape) == 1:
        return shape[0], 1
    out = shape[0]
    return out, numel(shape) // out


class SyntheticBackward:
    def __init__(self, params, tokens: int, dtype, dev):
        self.params = params
        self.tokens = tokens
        mo = max(gemm_shape(tuple(p.shape))[0] for p in params)
        mi = max(gemm_shape(tuple(p.shape))[1] for p in params)
        self.dy = fill_uniform(torch.empty(tokens, mo, dtype=dtype, device=dev), seed=1)
        self.x = fill_uniform(torch.empty(tokens, mi, dtype=dtype, device=dev), seed=2)

    def flops(self) -> float:
        return sum(2.0 * self.tokens * numel(tuple(p.shape)) for p in self.params if p.dim() > 1)

    def run(self, reducer: BucketedGradReducer | None, hook=None) -> None:
        hook = hook if hook is not None else (reducer._on_grad_ready if reducer is not None else None)
        for p in reversed(self.params):  # autograd order
            o, i = gemm_shape(tuple(p.shape))
            g = p.grad.view(o, i)
            if i > 1:
                torch.matmul(self.dy[:, :o].t(), self.x[:, :i], out=g)
            else:
                g.copy_(self.dy[0, :o].view(o, 1))
            if hook is not None:
                hook(p)  # what the post-accumulate-grad hook does


def timed(fn, steps: int, dev) -> float:
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    dist.barrier()
    dt = (time.perf_counter() - t0) / steps
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item() * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["resnet50", "llama3_8b"], default="resnet50")
    ap.add_argument("--tokens", type=int, default=1024, help="rows of the synthetic backward GEMMs")
    ap.add_argument("--bucket-mib", type=int, default=64)
    ap.add_argument("--engine", choices=["xgmi", "rccl"], default="xgmi")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layers", type=int, default=32, help="llama3_8b: transformer layers (32 = full model)")
    ap.add_argument("--sync", choices=["native", "torch"], default="native", help="reducer stream ordering")
    ap.add_argument("--event-scope", type=int, default=1, help="native events: 0 system, 1 device, 2 no fence")
    ap.add_argument("--comm-grid", type=int, default=0, help="xgmi workgroups per launch (0 = engine default)")
    args = ap.parse_args()
    rank, world, local = init_distributed("nccl")
    dev = torch.device("cuda", local)
    dtype = torch.bfloat16
    shapes = gradient_shapes(args.model) if args.model != "llama3_8b" else \
        __import__("akka_allreduce_1_amd.models.grad_sets", fromlist=["x"]).llama3_8b_shapes(args.layers)
    params = [torch.nn.Parameter(torch.zeros(s, dtype=dtype, device=dev)) for _, s in shapes]
    comm = XgmiCommunicator(grid=args.comm_grid) if args.engine == "xgmi" else TorchDistComm()
    reducer = BucketedGradReducer(params, comm, bucket_bytes=args.bucket_mib << 20, op="avg", sync=args.sync,
                                  event_scope=args.event_scope)
    reducer.remove_hooks()  # the synthetic backward calls the hook itself
    bwd = SyntheticBackward(params, args.tokens, dtype, dev)
    lr = 1e-3
    grads = [p.grad for p in params]

    def step_overlap():
        bwd.run(reducer)
        reducer.wait()
        torch._foreach_add_(params, grads, alpha=-lr)

    def step_compute():
        bwd.run(None)
        torch._foreach_add_(params, grads, alpha=-lr)

    def step_comm():
        for b in reducer.buckets:
            comm.allreduce_(b.buffer, op="avg")

    def step_serial():  # no overlap: all gradients, then all buckets
        bwd.run(None)
        step_comm()
        torch._foreach_add_(params, grads, alpha=-lr)

    with torch.no_grad():
        for f in (step_overlap, step_compute, step_comm, step_serial):
            for _ in range(args.warmup):
                f()
        t_overlap = timed(step_overlap, args.steps, dev)
        t_compute = timed(step_compute, args.steps, dev)
        t_comm = timed(step_comm, args.steps, dev)
        t_serial = timed(step_serial, args.steps, dev)
    nbytes = sum(b.nbytes for b in reducer.buckets)
    res = {
        "metric": "dp_step_ms", "model": args.model, "n_gpus": world, "engine": args.engine,
        "params": sum(numel(s) for _, s in shapes), "grad_bytes": nbytes, "buckets": len(reducer.buckets),
        "tokens": args.tokens, "bucket_mib": args.bucket_mib, "sync": args.sync, "event_scope": args.event_scope,
        "comm_grid": args.comm_grid, "step_overlap_ms": round(t_overlap, 3), "step_serial_ms": round(t_serial, 3),
        "compute_ms": round(t_compute, 3), "comm_ms": round(t_comm, 3),
        "exposed_comm_ms": round(t_overlap - t_compute, 3),
        "overlap_efficiency": round((t_serial - t_overlap) / max(min(t_comm, t_compute), 1e-9), 3),
        "comm_algbw_GBps": round(nbytes / (t_comm / 1e3) / 1e9, 2),
        "backward_tflops": round(bwd.flops() / (t_compute / 1e3) / 1e12, 1),
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
