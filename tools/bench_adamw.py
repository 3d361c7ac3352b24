#!/usr/bin/env python3
"""Fused sharded-DP step vs its unfused pipeline, P logical ranks on one MI355X.

unfused (what ShardedDataParallel does with a torch optimizer, bf16 params + fp32 master):
    reduce_scatter (xGMI, mean) -> cast shard grad to fp32 -> torch AdamW(fused=True) on the
    fp32 master shard -> cast master to the bf16 param shard -> all_gather (xGMI)
fused (csrc/hip/xgmi_adam.hip): one launch doing all of it.

    python tools/bench_adamw.py --ranks 2 8 --mib 64
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.ops import dtype_code, fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402
from akka_allreduce_1_amd.utils.timing import percentile  # noqa: E402


def timeit(fn, iters: int) -> float:
    for _ in range(3):
        fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return percentile([a.elapsed_time(b) for a, b in evs], 50)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 8])
    ap.add_argument("--mib", type=int, default=64, help="bf16 parameter bytes per rank")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--fused-only", action="store_true", help="time the fused launch only (PMC runs)")
    ap.add_argument("--grid", type=int, default=512)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    n = (args.mib << 20) // 2
    hp = dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    for P in args.ranks:
        cl = LocalCluster(P, slot_bytes=-(-(args.mib << 20) // P) + (1 << 20), grid=args.grid, timeout_s=20.0)
        b = cl.comms[0].block_elems(n, dtype_code(dt))
        grads = [fill_uniform(torch.empty(n, dtype=dt, device=dev), seed=k) for k in range(P)]
        params = [fill_uniform(torch.empty(n, dtype=dt, device=dev), seed=99) for _ in range(P)]
        states = [{"master": params[k][k * b:(k + 1) * b].float().contiguous(),
                   "exp_avg": torch.zeros(b, device=dev), "exp_avg_sq": torch.zeros(b, device=dev)}
                  for k in range(P)]
        t = {"step": 0}

        def fused():
            t["step"] += 1
            cl.step_adamw(grads, params, states, step=t["step"], **hp)

        # unfused pipeline with the same buffers
        shard_g = [torch.empty(b, dtype=dt, device=dev) for _ in range(P)]
        masters = [torch.nn.Parameter(states[k]["master"].clone()) for k in range(P)]
        opts = [torch.optim.AdamW([masters[k]], fused=True, **hp) for k in range(P)]
        shard_p = [torch.empty(b, dtype=dt, device=dev) for _ in range(P)]

        def unfused():
            cl.collective("reduce_scatter", grads, shard_g, scale=1.0 / P)
            for k in range(P):
                masters[k].grad = shard_g[k].float()
                opts[k].step()
                shard_p[k].copy_(masters[k].detach())
            cl.collective("all_gather", shard_p, params)

        row = {"P": P, "grid": args.grid, "param_MiB_per_rank": args.mib, "fused_ms": round(timeit(fused, args.iters), 4)}
        if P == 1:  # bytes per param: bf16 grad in + bf16 param out + fp32 master / m / v in and out
            row["hbm_TBps"] = round(28 * n / (row["fused_ms"] / 1e3) / 1e12, 3)
        if not args.fused_only:
            row["unfused_ms"] = round(timeit(unfused, args.iters), 3)
            row["speedup"] = round(row["unfused_ms"] / row["fused_ms"], 2)
        cl.check()
        print(json.dumps(row), flush=True)
        del cl, grads, params, states, shard_g, masters, opts, shard_p
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
