#!/usr/bin/env python3
"""Soak test of the xGMI engine: a long random mix of collectives on P processes, every
result checked against an fp32 reference.

Every rank draws the same sequence of (operation, algorithm, dtype, size, in-place) from a
shared seed, so the ranks issue identical collective sequences, and every rank generates all
P inputs from per-(step, rank) seeds, so it can check its own output. What this exercises that
the unit tests do not: thousands of launches that switch algorithm, dtype and size between
calls on the same slabs and epoch counters (what `tune()` and a training step do), for minutes.

    # P processes on ONE GPU (rehearsal; gloo for the CPU group):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/soak.py \
        --share-device --seconds 240
    # one process per GPU (rank k on local device k, cross-GPU stores over xGMI):
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/soak.py --seconds 600
    # an explicit rank -> device map (rank k on devices[k % len]), e.g. 4 ranks on 2 GPUs:
    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 tools/soak.py --devices 0,1

The control plane (stop flags, error counts, the communicator's handle exchange) is a gloo
group in every mode, so the soak needs nothing from RCCL and the data moves only through
the engine's kernels.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import random
import sys
import time

if "--share-device" in sys.argv:  # see bench.py: one hardware queue per process on a shared GPU
    os.environ["GPU_MAX_HW_QUEUES"] = "1"

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel.comm import CommError, XgmiCommunicator, init_distributed  # noqa: E402

OPS = ["ll", "oneshot", "twoshot", "ring", "ring_native", "threshold", "auto", "all_gather", "reduce_scatter",
       "all_to_all"]
DTYPES = {"fp32": (torch.float32, 1e-5), "bf16": (torch.bfloat16, 2.0 ** -7), "fp16": (torch.float16, 2.0 ** -10)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--max-mib", type=float, default=32.0, help="largest tensor per rank")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--share-device", action="store_true", help="every rank on cuda:0")
    ap.add_argument("--devices", default="",
                    help="comma-separated device ids, rank k runs on devices[k %% len] (default: local rank)")
    args = ap.parse_args()
    rank, world, local = init_distributed("gloo")
    devices = [int(d) for d in args.devices.split(",") if d.strip()] if args.devices else []
    if args.share_device:
        devices = [0]
    local = devices[rank % len(devices)] if devices else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # ranks sharing a GPU split its workgroups so every persistent kernel stays resident
    share = sum(1 for r in range(world) if (devices[r % len(devices)] if devices else r) == local)
    max_bytes = int(args.max_mib * (1 << 20))
    comm = XgmiCommunicator(device=local, slot_bytes=-(-max_bytes // world) + (1 << 20),
                            grid=max(8, 512 // share) if share > 1 else 0, timeout_s=30.0, max_lag=1)
    rng = random.Random(args.seed)  # same stream on every rank
    counts: dict[str, int] = {}
    errors: list[str] = []
    t0 = last = time.time()
    step = 0
    flags = torch.zeros(2)
    while True:
        # [time is up on rank 0, errors anywhere]: every rank leaves at the same step
        flags[0] = 1.0 if (rank == 0 and time.time() - t0 >= args.seconds) else 0.0
        flags[1] = float(len(errors))
        dist.all_reduce(flags, op=dist.ReduceOp.MAX)
        if flags[0] > 0 or flags[1] > 0:
            break
        op = rng.choice(OPS)
        dname = rng.choice(list(DTYPES))
        dt, rtol = DTYPES[dname]
        es = torch.empty(0, dtype=dt).element_size()
        unit = world * 8  # every block 16-byte sized for every dtype
        n = max(unit, int(math.exp(rng.uniform(math.log(unit), math.log(max_bytes // es)))) // unit * unit)
        inplace = rng.random() < 0.5 and op not in ("all_gather", "reduce_scatter", "all_to_all")
        xs = [fill_uniform(torch.empty(n, dtype=dt, device=dev), seed=(step * 977 + k) % (1 << 30))
              for k in range(world)]
        x = xs[rank]
        tag = f"{op}/{dname}/{n * es}B" + ("/inplace" if inplace else "")
        try:
            if op in ("all_gather",):
                m = n // world
                out = comm.all_gather(x[:m].clone())
                ref = torch.cat([xk[:m] for xk in xs])
                ok = torch.equal(out, ref)
            elif op == "all_to_all":
                out = comm.all_to_all(x)
                m = n // world
                ref = torch.cat([xk[rank * m:(rank + 1) * m] for xk in xs])
                ok = torch.equal(out, ref)
            else:
                ref = torch.stack([xk.float() for xk in xs]).sum(0)
                if op == "reduce_scatter":
                    m = n // world
                    out = comm.reduce_scatter(x, op="sum").float()
                    ref = ref[rank * m:(rank + 1) * m]
                elif op == "threshold":
                    out = comm.allreduce_threshold(x, x if inplace else None).float()
                else:
                    out = comm.allreduce(x, x if inplace else None, op="sum", algo=op).float()
                # the element-type-wire ring rounds the partial sum to the wire dtype at each of its
                # P-2 intermediate hops: each rounding <= rtol/2 * sum_k |x_k| (the exact-wire ring and
                # `auto` keep the bound too, as they did when the ring's partials were element-typed)
                tol = 1e-4 * world + rtol * ref.abs()
                if op in ("ring", "ring_native", "auto"):
                    tol = tol + 0.5 * rtol * max(world - 2, 0) * torch.stack([xk.float().abs() for xk in xs]).sum(0)
                err = (out - ref).abs()
                ok = bool((err <= tol).all())
                if not ok:
                    tag += f" max_err {err.max().item():.3g} bad {(err > tol).sum().item()}/{err.numel()}"
            comm.check()
        except CommError as e:  # a peer missed a deadline: stop everyone at the next step
            errors.append(f"step {step} {tag}: {e}")
            ok = True
        counts[op] = counts.get(op, 0) + 1
        if not ok:
            errors.append(f"step {step} {tag}: mismatch")
        step += 1
        if rank == 0 and time.time() - last >= 20.0:
            last = time.time()
            print(f"[soak] {last - t0:.0f}s step {step} errors {len(errors)}", flush=True)
    bad = torch.tensor([float(len(errors))])
    dist.all_reduce(bad)
    if bad.item() > 0:  # every rank's control words next to the error: epoch agreement across ranks
        words = [None] * world
        try:
            mine = list(comm.native.ctl_words())
        except Exception as e:  # noqa: BLE001
            mine = [repr(e)]
        dist.all_gather_object(words, mine)
        if rank == 0:
            print(f"[soak] ctl words per rank ([0] launch epoch, [2] error, [4] threshold epoch): {words}",
                  file=sys.stderr, flush=True)
    if errors:
        print(f"[soak rank {rank}] " + "; ".join(errors[:5]), file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps({"metric": "soak", "world": world, "devices": devices or list(range(world)),
                          "seconds": round(time.time() - t0, 1), "steps": step,
                          "errors_all_ranks": int(bad.item()), "ops": counts, "max_bytes": max_bytes}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if bad.item() > 0 else 0)


if __name__ == "__main__":
    main()
