#!/usr/bin/env python3
"""A/B of the fused AdamW state placement (1 logical rank, 134 M bf16 params, the bench's
fused_adamw_step shape): master / exp_avg / exp_avg_sq as three separate 512 MiB
allocations ("separate", what adamw_state() does) vs views of one allocation offset by
1 MiB + 4 KiB ("offset"), so the three streams do not share the same address bits.

    python tools/adam_state_ab.py [separate|offset|both] [iters]
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.ops import dtype_code, fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402
from akka_allreduce_1_amd.utils.timing import percentile  # noqa: E402

N = 134_217_728
PAD = ((1 << 20) + 4096) // 4


def states(kind: str, b: int, dev) -> dict:
    if kind == "separate":
        return {k: torch.zeros(b, device=dev) for k in ("master", "exp_avg", "exp_avg_sq")}
    big = torch.zeros(3 * (b + PAD), device=dev)
    return {k: big[i * (b + PAD): i * (b + PAD) + b] for i, k in enumerate(("master", "exp_avg", "exp_avg_sq"))}


def main() -> None:
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cl = LocalCluster(1, slot_bytes=(N * 2) + (1 << 20), grid=512, timeout_s=10.0)
    b = cl.comms[0].block_elems(N, dtype_code(torch.bfloat16))
    g = fill_uniform(torch.empty(N, dtype=torch.bfloat16, device=dev), seed=1)
    p = fill_uniform(torch.empty(N, dtype=torch.bfloat16, device=dev), seed=2)
    hp = dict(lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for kind in (("separate", "offset") if which == "both" else (which,)):
        st = states(kind, b, dev)
        for t in range(1, 4):
            cl.step_adamw([g], [p], [st], step=t, **hp)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for i, (e0, e1) in enumerate(evs):
            e0.record()
            cl.step_adamw([g], [p], [st], step=4 + i, **hp)
            e1.record()
        torch.cuda.synchronize()
        cl.check()
        ms = percentile([e0.elapsed_time(e1) for e0, e1 in evs], 50)
        print(json.dumps({"state": kind, "params": N, "ms": round(ms, 4), "TBps": round(28 * N / ms / 1e9, 2)}),
              flush=True)
        del st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
