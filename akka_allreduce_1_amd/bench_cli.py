"""mxar-bench: allreduce algbw / busbw / p50 sweep over tensor sizes.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m akka_allreduce_1_amd bench
    python -m akka_allreduce_1_amd bench --local 8 --algos twoshot ring   # 8 ranks on ONE GPU
    python -m akka_allreduce_1_amd bench --backend gloo --algos torch     # CPU plumbing

Per (size, algo): p50 and mean over `--iters` event-timed calls after `--warmup`; the
slowest rank's numbers are reported (all-reduce MAX). algbw = bytes / p50, busbw =
algbw * 2(P-1)/P (nccl-tests convention). Engines:
  twoshot / oneshot / ring  fused xGMI kernels (csrc/hip/xgmi_comm.hip)
  ll                        low-latency one-shot, flags inside the data (csrc/hip/xgmi_ll.hip)
  all_to_all / all_gather / reduce_scatter   xGMI collectives (csrc/hip/xgmi_coll.hip); SIZE =
                            the full [world x m] buffer (all_gather: its output)
  threshold                 straggler-tolerant kernel at th = 1 (csrc/hip/xgmi_threshold.hip)
  rccl                      torch.distributed all_reduce on the nccl (= RCCL) backend
  torch                     torch.distributed all_reduce on whatever backend (gloo on CPU)
Rank 0 prints a table to stderr and one JSON line per row to stdout (or --json FILE).
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch


def _sizes(spec: list[str]) -> list[int]:
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}

    def one(s: str) -> int:
        s = s.strip().upper().rstrip("B").rstrip("I")
        return int(float(s[:-1]) * mult[s[-1]]) if s and s[-1] in mult else int(s)

    if len(spec) == 1 and ".." in spec[0]:  # geometric range lo..hi (x4)
        lo, hi = (one(x) for x in spec[0].split(".."))
        out, v = [], lo
        while v < hi:
            out.append(v)
            v *= 4
        return out + [hi]
    return [one(s) for s in spec]


def _time(fn, iters: int, warmup: int, sync) -> tuple[float, float]:
    from .utils.timing import percentile

    for _ in range(warmup):
        fn()
    sync()
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for a, b in evs:
            a.record()
            fn()
            b.record()
        sync()
        ts = [a.elapsed_time(b) for a, b in evs]
    else:
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            sync()
            ts.append((time.perf_counter() - t0) * 1e3)
    return percentile(ts, 50), sum(ts) / len(ts)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="mxar-bench", description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--sizes", nargs="+", default=["4K..256M"], help="sizes (4K 1M ...) or a range lo..hi (x4 steps)")
    ap.add_argument("--algos", nargs="+", default=["ll", "oneshot", "twoshot", "ring", "rccl"])
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--op", choices=["sum", "avg"], default="sum")
    ap.add_argument("--local", type=int, default=0, help="P logical ranks on one GPU (no torch.distributed)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (gloo: CPU tensors, algo 'torch')")
    ap.add_argument("--json", default=None, help="write the JSON rows here instead of stdout")
    args = ap.parse_args(argv)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    sizes = _sizes(args.sizes)
    rows: list[dict] = []

    if args.local:
        from .ops import fill_uniform
        from .parallel import LocalCluster

        P = args.local
        cl = LocalCluster(P, slot_bytes=max(16 << 20, -(-max(sizes) // P) + (1 << 20)), grid=512,  # workgroup budget of the device, shared by the P ranks
                          max_lag=0 if "threshold" in args.algos else None)
        dev = cl.devices[0]
        xs = [fill_uniform(torch.empty(max(sizes) // es, dtype=dtype, device=dev), seed=k) for k in range(P)]
        ys = [torch.empty_like(x) for x in xs]
        for size in sizes:
            n = size // es
            for algo in args.algos:
                if algo in ("rccl", "torch") or (algo == "oneshot" and size > cl.comms[0].slot_bytes) or (
                        algo == "ll" and size > cl.comms[0].ll_max_bytes):
                    continue
                if algo == "threshold":
                    def fn():
                        cl.allreduce_threshold([x[:n] for x in xs], [y[:n] for y in ys])
                elif algo in ("all_to_all", "all_gather", "reduce_scatter"):
                    m = n // P // 8 * 8
                    if m == 0:
                        continue
                    ins = [x[:m] for x in xs] if algo == "all_gather" else [x[:P * m] for x in xs]
                    outs = [y[:m] for y in ys] if algo == "reduce_scatter" else [y[:P * m] for y in ys]

                    def fn(algo=algo, ins=ins, outs=outs):
                        cl.collective(algo, ins, outs)
                else:
                    def fn():
                        cl.allreduce([x[:n] for x in xs], [y[:n] for y in ys], algo=algo, op=args.op)
                p50, mean = _time(fn, args.iters, args.warmup, lambda: torch.cuda.synchronize(dev))
                cl.check()
                rows.append({"P": P, "mode": "local", "bytes": size, "algo": algo, "p50_us": round(p50 * 1e3, 2),
                             "mean_us": round(mean * 1e3, 2)})
        rank = 0
    else:
        import torch.distributed as dist

        from .parallel.comm import init_distributed

        rank, P, local = init_distributed(args.backend)
        on_gpu = args.backend == "nccl"
        dev = torch.device("cuda", local) if on_gpu else torch.device("cpu")
        comm = None
        if on_gpu and any(a in ("ll", "oneshot", "twoshot", "ring", "threshold") + ("all_to_all", "all_gather", "reduce_scatter") for a in args.algos):
            from .parallel import XgmiCommunicator

            comm = XgmiCommunicator(slot_bytes=max(64 << 20, -(-max(sizes) // P) + (1 << 20)),
                                    max_lag=0 if "threshold" in args.algos else None)
        x = torch.empty(max(sizes) // es, dtype=dtype, device=dev).uniform_(-1, 1)
        y = torch.empty_like(x)
        sync = (lambda: torch.cuda.synchronize(dev)) if on_gpu else (lambda: None)
        for size in sizes:
            n = size // es
            for algo in args.algos:
                if algo in ("ll", "oneshot", "twoshot", "ring"):
                    if comm is None or (algo == "oneshot" and size > comm.slot_bytes) or (
                            algo == "ll" and size > comm.native.ll_max_bytes):
                        continue
                    fn = lambda: comm.allreduce(x[:n], y[:n], algo=algo, op=args.op)  # noqa: E731
                elif algo == "threshold":
                    if comm is None:
                        continue
                    fn = lambda: comm.allreduce_threshold(x[:n], y[:n])  # noqa: E731
                elif algo in ("all_to_all", "all_gather", "reduce_scatter"):
                    if comm is None:
                        continue
                    m = n // P // 8 * 8
                    if m == 0:
                        continue
                    if algo == "all_gather":
                        fn = lambda m=m: comm.all_gather(x[:m], y[:P * m])  # noqa: E731
                    elif algo == "all_to_all":
                        fn = lambda m=m: comm.all_to_all(x[:P * m], y[:P * m])  # noqa: E731
                    else:
                        fn = lambda m=m: comm.reduce_scatter(x[:P * m], y[:m])  # noqa: E731
                elif algo in ("rccl", "torch"):
                    if algo == "rccl" and not on_gpu:
                        continue

                    def fn():
                        y[:n].copy_(x[:n])
                        dist.all_reduce(y[:n])
                else:
                    raise SystemExit(f"unknown algo {algo}")
                p50, mean = _time(fn, args.iters, args.warmup, sync)
                t = torch.tensor([p50, mean], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                rows.append({"P": P, "mode": "dist", "backend": args.backend, "bytes": size, "algo": algo,
                             "p50_us": round(t[0].item() * 1e3, 2), "mean_us": round(t[1].item() * 1e3, 2)})
        if comm is not None:
            comm.check()
    for r in rows:
        alg = r["bytes"] / (r["p50_us"] / 1e6) / 1e9
        r["algbw_GBps"] = round(alg, 2)
        r["busbw_GBps"] = round(alg * 2 * (r["P"] - 1) / r["P"], 2)
        r["dtype"] = args.dtype
    if rank == 0:
        print(f"{'bytes':>12} {'algo':>8} {'p50 us':>10} {'algbw GB/s':>11} {'busbw GB/s':>11}", file=sys.stderr)
        for r in rows:
            print(f"{r['bytes']:>12} {r['algo']:>8} {r['p50_us']:>10.2f} {r['algbw_GBps']:>11.2f} {r['busbw_GBps']:>11.2f}",
                  file=sys.stderr)
        lines = "\n".join(json.dumps(r) for r in rows) + "\n"
        if args.json:
            with open(args.json, "w") as f:
                f.write(lines)
        else:
            sys.stdout.write(lines)
    if not args.local:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
