#!/usr/bin/env python3
"""Data-parallel training of a small causal transformer LM with the framework's bucketed
gradient allreduce, one process per GPU.

The reference allreduces one flat vector per round, taken from a `dataSource` and handed to
a `dataSink` (AllreduceWorker.scala:171-192). In training, that vector is the gradient set,
and `BucketedGradReducer` makes the gradients themselves the flat vectors. Each bucket is one
HBM buffer that the parameters' `.grad` tensors view. Full buckets are allreduced on a side
stream while backward still runs.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_dp.py --steps 200
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/train_dp.py --cpu --steps 20   # gloo

Straggler-tolerant steps use the reference's thresholds (GPU):
    ... examples/train_dp.py --th 0.875     # a chunk missing up to 1/8 of the ranks is rescaled

Each rank draws its own synthetic token batches. A rank's batch repeats a short random
pattern, so the loss falls quickly. At the end every rank checks that its parameters equal
rank 0's, bit for bit.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.parallel import BucketedGradReducer, TorchDistComm, XgmiCommunicator  # noqa: E402
from akka_allreduce_1_amd.parallel.comm import init_distributed  # noqa: E402


class Block(nn.Module):
    def __init__(self, d: int, heads: int):
        super().__init__()
        self.ln1, self.ln2 = nn.LayerNorm(d), nn.LayerNorm(d)
        self.attn = nn.MultiheadAttention(d, heads, batch_first=True)
        self.mlp = nn.Sequential(nn.Linear(d, 4 * d), nn.GELU(), nn.Linear(4 * d, d))

    def forward(self, x, mask):
        h = self.ln1(x)
        x = x + self.attn(h, h, h, attn_mask=mask, need_weights=False)[0]
        return x + self.mlp(self.ln2(x))


class TinyLM(nn.Module):
    def __init__(self, vocab: int, d: int, layers: int, heads: int, ctx: int):
        super().__init__()
        self.tok = nn.Embedding(vocab, d)
        self.pos = nn.Parameter(torch.zeros(ctx, d))
        self.blocks = nn.ModuleList(Block(d, heads) for _ in range(layers))
        self.ln = nn.LayerNorm(d)
        self.head = nn.Linear(d, vocab, bias=False)

    def forward(self, idx):
        T = idx.shape[1]
        mask = torch.triu(torch.full((T, T), float("-inf"), device=idx.device), 1)
        x = self.tok(idx) + self.pos[:T]
        for b in self.blocks:
            x = b(x, mask)
        return self.head(self.ln(x))


def batch(gen, bsz, ctx, vocab, dev):
    """Sequences that repeat a random 8-token pattern: learnable, different on every rank."""
    pat = torch.randint(0, vocab, (bsz, 8), generator=gen)
    seq = pat.repeat(1, ctx // 8 + 2)[:, : ctx + 1]
    return seq[:, :-1].to(dev), seq[:, 1:].to(dev)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--ctx", type=int, default=64)
    ap.add_argument("--vocab", type=int, default=256)
    ap.add_argument("--width", type=int, default=128)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--lr", type=float, default=3e-3)
    ap.add_argument("--bucket-mib", type=int, default=4)
    ap.add_argument("--th", type=float, default=1.0, help="thReduce = thComplete of every bucket (GPU, < 1: straggler-tolerant)")
    ap.add_argument("--cpu", action="store_true", help="gloo on the CPU (TorchDistComm)")
    ap.add_argument("--overlap", choices=["on", "off", "auto"], default="on",
                    help="buckets beside backward, after it, or measured in the first steps (GPU)")
    args = ap.parse_args()

    rank, world, local = init_distributed("gloo" if args.cpu else "nccl")
    dev = torch.device("cpu") if args.cpu else torch.device("cuda", local)
    torch.manual_seed(0)  # identical initial replicas
    model = TinyLM(args.vocab, args.width, args.layers, 4, args.ctx).to(dev)
    if args.cpu:
        comm = TorchDistComm()
    else:
        comm = XgmiCommunicator(device=dev, max_lag=1 if args.th < 1.0 else None)
    kw = dict(th_reduce=args.th, th_complete=args.th, rescale=True) if args.th < 1.0 else {}
    overlap = {"on": True, "off": False, "auto": "auto"}[args.overlap]
    reducer = BucketedGradReducer(model, comm, bucket_bytes=args.bucket_mib << 20, op="avg", overlap=overlap, **kw)
    opt = torch.optim.AdamW(model.parameters(), lr=args.lr)
    gen = torch.Generator().manual_seed(1000 + rank)
    t0 = time.perf_counter()
    first = last = None
    for step in range(args.steps):
        x, y = batch(gen, args.batch, args.ctx, args.vocab, dev)
        loss = F.cross_entropy(model(x).flatten(0, 1), y.flatten())
        loss.backward()          # the reducer's hooks launch full buckets during backward
        reducer.wait()           # the mean gradient is in every .grad
        opt.step()
        reducer.zero_grad()      # keep .grad as views of the buckets
        lv = float(loss.detach())
        first = lv if first is None else first
        last = lv
        if rank == 0 and (step % max(1, args.steps // 10) == 0 or step == args.steps - 1):
            print(f"step {step:4d} loss {lv:.4f}", flush=True)
    if not args.cpu:
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    # every replica must hold rank 0's parameters (exact allreduce: bit-identical updates)
    import torch.distributed as dist

    flat = torch.cat([p.detach().float().flatten() for p in model.parameters()])
    ref = flat.clone()
    dist.broadcast(ref, 0)
    diff = torch.tensor([float((flat - ref).abs().max())], device=flat.device)
    dist.all_reduce(diff, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(f"done: {args.steps} steps in {dt:.2f} s, loss {first:.3f} -> {last:.3f}, "
              f"replica max diff {diff.item():.3g}, schedule {reducer.stats.get('schedule', reducer.schedule)}",
              flush=True)
    ok = last < first and (diff.item() == 0.0 or args.th < 1.0)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
