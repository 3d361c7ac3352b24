#!/usr/bin/env python3
"""Single-GPU analysis bench: P logical ranks of the fused allreduce on ONE MI355X.

All ranks' traffic lands in one GPU's HBM (no xGMI hop), so this measures the kernel's
own costs - fences, flag hand-offs, unit geometry, HBM efficiency - not link bandwidth.
HBM bytes per rank for a two-shot of S bytes (bf16): read S + write S(P-1)/P (scatter),
read S + write S (reduce + broadcast), read S(P-1)/P + write S(P-1)/P (gather).

    python tools/bench_local.py --ranks 2 4 8 --sizes 1M 16M 256M --fence 3 0
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402
from akka_allreduce_1_amd.utils.timing import hbm_bytes, percentile  # noqa: E402


def parse_size(s: str) -> int:
    m = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * m[s[-1].upper()]) if s[-1].upper() in m else int(s)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--sizes", nargs="+", default=["64K", "1M", "16M", "64M", "256M"])
    ap.add_argument("--algos", nargs="+", default=["twoshot", "oneshot"])
    ap.add_argument("--fence", type=int, nargs="+", default=[3])
    ap.add_argument("--ring-depth", type=int, nargs="+", default=[0],
                    help="ring chunks per workgroup to sweep (0 = the communicator's default)")
    ap.add_argument("--grid", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    rows = []
    # reference: device copy bandwidth
    x = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    copy_ms = e0.elapsed_time(e1) / 10
    print(json.dumps({"copy_256MiB_ms": round(copy_ms, 4), "copy_TBps": round(2 * x.numel() / copy_ms / 1e9, 2)}))
    del x, y
    for P in args.ranks:
        max_sz = max(parse_size(s) for s in args.sizes)
        slot = max(1 << 20, -(-max_sz // P) + (1 << 16))
        cl = LocalCluster(P, slot_bytes=slot, grid=args.grid, timeout_s=10.0,
                          max_lag=1 if "threshold" in args.algos else None)
        for sz_s in args.sizes:
            S = parse_size(sz_s)
            n = S // es
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=k) for k in range(P)]
            ys = [torch.empty_like(t) for t in xs]
            ref = torch.zeros(n, device=dev)
            for t in xs:
                ref += t.float()
            for algo in args.algos:
                if (algo == "oneshot" and S > slot) or (algo == "ll" and S > cl.comms[0].ll_max_bytes):
                    continue
                variants = [(f, d) for f in args.fence for d in (args.ring_depth if algo.startswith("ring") else [0])]
                for fence, depth in variants:
                    for c in cl.comms:
                        c.fence = fence
                        if depth:
                            c.ring_depth = depth
                    if algo in ("all_to_all", "reduce_scatter", "all_gather"):
                        ins = [t[:n // P].contiguous() for t in xs] if algo == "all_gather" else xs
                        outs = [torch.empty(n // P if algo == "reduce_scatter" else n, dtype=dtype, device=dev)
                                for _ in range(P)]

                        def fn(ins=ins, outs=outs, algo=algo):
                            cl.collective(algo, ins, outs)
                        err = 0.0
                    elif algo == "threshold":  # the round engine's kernel at th = 1 (same bytes as two-shot)
                        def fn():
                            cl.allreduce_threshold(xs, ys)
                        fn()
                        cl.check()
                        err = max((t.float() - ref).abs().max().item() for t in ys)
                    else:
                        def fn(algo=algo):
                            cl.allreduce(xs, ys, algo=algo)
                        fn()
                        cl.check()
                        err = max((t.float() - ref).abs().max().item() for t in ys)
                    for _ in range(3):
                        fn()
                    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                          for _ in range(args.iters)]
                    for a, b in ev:
                        a.record()
                        fn()
                        b.record()
                    cl.check()
                    ts = [a.elapsed_time(b) for a, b in ev]
                    p50 = percentile(ts, 50)
                    row = {"P": P, "bytes": S, "algo": algo, "fence": fence, "p50_us": round(p50 * 1e3, 1),
                           "min_us": round(min(ts) * 1e3, 1),
                           "hbm_TBps": round(hbm_bytes(S, P, algo, es) / p50 / 1e9, 2), "max_err": err}
                    if depth:
                        row["ring_depth"] = depth
                    rows.append(row)
                    print(json.dumps(row), flush=True)
            del xs, ys, ref
        del cl
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"copy_ms": copy_ms, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
