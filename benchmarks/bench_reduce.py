#!/usr/bin/env python3
"""BASELINE config 2: single-GPU in-place reduce of a 1 GiB fp32 buffer (kernel only,
world_size = 1) - the worker's `reduce` (AllreduceWorker.scala:240-251, K1 of SURVEY §2.4)
as the `reduce_slots` HIP kernel.

`slots` is [P, n]; the in-place form accumulates into row 0 (out = slots[0]), which is how
a receive buffer is reduced in place. Reported per case: time (median of --iters event-timed
launches), algbw = buffer bytes / time, HBM traffic rate = (P reads + 1 write) x bytes / time,
and that rate as a fraction of the device-copy roofline measured in the same process (our
copy kernel, read + write). PyTorch's own kernels on the same tensors are timed for
comparison (`add_` for P = 2, `sum(dim=0)` otherwise).

    python benchmarks/bench_reduce.py                      # 1 GiB fp32, P = 2, 4, 8
    python benchmarks/bench_reduce.py --mib 256 --dtype bf16
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform, reduce_slots  # noqa: E402
from akka_allreduce_1_amd.utils.timing import percentile  # noqa: E402


def time_ms(fn, iters: int, warmup: int = 3) -> float:
    for _ in range(warmup):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return percentile([a.elapsed_time(b) for a, b in ev], 50)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024, help="buffer size per slot")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--slots", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", type=int, nargs="*", default=[],
                    help="also time these reduce_slots kernel variants (kernels.hip launch_reduce_typed)")
    ap.add_argument("--pad-kib", type=int, default=0,
                    help="pad every slot row by this much (slot stride not a power of two)")
    args = ap.parse_args()
    dt = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    es = 4 if dt == torch.float32 else 2
    nbytes = args.mib << 20
    n = nbytes // es
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.current_stream().cuda_stream

    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    t_copy = time_ms(lambda: C.hip.copy(src.data_ptr(), dst.data_ptr(), nbytes, s), args.iters)
    copy_rate = 2 * nbytes / (t_copy / 1e3) / 1e12
    del src, dst
    rows = []
    for P in args.slots:
        pad = (args.pad_kib << 10) // es
        slots = torch.empty(P, n + pad, dtype=dt, device=dev)[:, :n]
        for p in range(P):
            fill_uniform(slots[p], seed=p)
        # correctness: one in-place launch vs an fp32 torch reference
        ref = slots.float().sum(0)
        work = slots.contiguous().clone()
        reduce_slots(work, out=work[0])
        err = (work[0].float() - ref).abs().max().item()
        del work, ref
        out = torch.empty(n, dtype=dt, device=dev)
        cases = {
            "mxar_inplace": lambda: reduce_slots(slots, out=slots[0]),
            "mxar_outofplace": lambda: reduce_slots(slots, out=out),
            "torch": (lambda: slots[0].add_(slots[1])) if P == 2 else (lambda: torch.sum(slots, 0, out=out)),
        }
        for v in args.variants:
            def run_v(v=v):
                C.hip.set_reduce_variant(v)
                reduce_slots(slots, out=out)
            cases[f"variant{v}_outofplace"] = run_v

            def run_vi(v=v):
                C.hip.set_reduce_variant(v)
                reduce_slots(slots, out=slots[0])
            cases[f"variant{v}_inplace"] = run_vi
        for name, fn in cases.items():
            t = time_ms(fn, args.iters)
            hbm = (P + 1) * nbytes / (t / 1e3) / 1e12
            rows.append({"case": name, "P": P, "pad_kib": args.pad_kib, "dtype": args.dtype, "bytes_per_slot": nbytes, "ms": round(t, 4),
                         "algbw_GBps": round(nbytes / (t / 1e3) / 1e9, 1), "hbm_TBps": round(hbm, 3),
                         "frac_of_copy_roofline": round(hbm / copy_rate, 3),
                         **({"max_abs_err_vs_fp32": err} if name == "mxar_inplace" else {})})
        C.hip.set_reduce_variant(-1)
        del slots, out
        torch.cuda.empty_cache()
    print(json.dumps({"metric": "reduce_kernel", "copy_roofline_TBps": round(copy_rate, 3), "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
