#!/usr/bin/env python3
"""Host-side cost of one XgmiCommunicator.allreduce call (N=1, torchrun-less): wall time per
call for a tiny tensor (GPU work ~ nothing) vs the same call captured in a hipGraph and
replayed, plus the raw launch path without the Python checks."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akka_allreduce_1_amd.parallel.comm import XgmiCommunicator, init_distributed  # noqa: E402


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


def main():
    init_distributed("nccl")
    comm = XgmiCommunicator()
    for size in (4096, 256 << 20):
        x = torch.ones(size // 2, dtype=torch.bfloat16, device="cuda")
        y = torch.empty_like(x)
        host, wall = per_call(lambda: comm.allreduce(x, y), 2000 if size < 1 << 20 else 200)
        s = torch.cuda.current_stream().cuda_stream
        c = comm._c
        code = torch.bfloat16
        from akka_allreduce_1_amd.parallel.comm import ALGOS, _dtype_code

        dc = _dtype_code(code)
        algo = ALGOS["auto"]
        raw_host, raw_wall = per_call(lambda: c.allreduce(x.data_ptr(), y.data_ptr(), x.numel(), dc, s, algo, 1.0),
                                      2000 if size < 1 << 20 else 200)
        copy_host, copy_wall = per_call(lambda: y.copy_(x), 2000 if size < 1 << 20 else 200)
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            comm.allreduce(x, y)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            comm.allreduce(x, y)
        gh, gw = per_call(g.replay, 2000 if size < 1 << 20 else 200)
        print(f"bytes={size}: python call host {host:.1f} us wall {wall:.1f} us | raw binding host {raw_host:.1f} "
              f"wall {raw_wall:.1f} | torch copy_ host {copy_host:.1f} wall {copy_wall:.1f} | graph replay host "
              f"{gh:.1f} wall {gw:.1f}", flush=True)


if __name__ == "__main__":
    main()
