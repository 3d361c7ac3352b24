#!/usr/bin/env python3
"""Headline benchmark: allreduce algbw (GB/s) + p50 latency of a 256 MiB bf16 gradient
buffer per GPU (BASELINE.json metric; config "Ring allreduce of 256 MiB bf16 gradient
buffer across 8xMI355X over xGMI"), one process per GPU.

    python bench.py                                    # 1 GPU, defaults
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --steps 20 --warmup 5

One "step" = one out-of-place allreduce of the buffer through the framework's engine
(the fused xGMI two-shot kernel, csrc/hip/xgmi_comm.hip). The result is validated against
an fp32 reference before timing. RCCL (`torch.distributed` nccl backend) is timed on the
same buffer for comparison. Rank 0 prints ONE JSON line. `value` = algbw = buffer bytes / time
of the slowest rank (nccl-tests convention: the job reduces S bytes per step, whatever N), the
figure RCCL's algbw column and BASELINE's metric use; `algbw_sum_over_ranks` = N x algbw is
kept under its own key. At N=1 an allreduce is an out-of-place copy, so the N=1 point is an
HBM copy rate, not a communication rate (`algo` says "copy (world=1)" and the tuner is
skipped); the `local_ranks` section then times the allreduce kernels themselves with 8
logical ranks in one launch on the GPU. Data: synthetic uniform(-1, 1) gradients.

Before anything is timed, every algorithm a section may pick (ll, one-shot, two-shot, ring,
threshold, all-to-all, all-gather, reduce-scatter) is checked against fp32 (`validated`),
and rank 0 records the peer-access / link-type / hop matrix (`topology`).

After the headline, side sections on the same engine (in the JSON, not in `value`): the
tuner's size sweep vs RCCL, the straggler-tolerant kernel, all-to-all / all-gather /
reduce-scatter, the fused sharded AdamW step, and `dp` = BASELINE configs 4 and 5 (one
data-parallel step of the ResNet-50 and full Llama-3-8B gradient sets with a GEMM-backed
synthetic backward overlapped with the bucketed reducer).

At N = 1 straggler tolerance is timed (`stragglers`, benchmarks/stragglers.py): the
reference's default job at its own thresholds (in process and native), and P = 4 workers with
one dataSource delayed 0 / 0.2 / 2 ms per round at th 0.75, maxLag 1 / 2, 40 B / 1 MiB / 64 MiB
(fast workers' round period vs no straggler, forced / cold rounds, counts, validated outputs).

At N = 1 the metric's size axis is timed too (benchmarks/sections.py): `latency_vs_size`
(p50 latency + algbw of every kernel and of `auto`, 8 / 4 / 2 logical ranks in one launch,
4 KiB .. 256 MiB, each cell validated to one rounding first), `reduce_kernel` (BASELINE
config 2: 1 GiB fp32 reduce of 2 / 4 / 8 slots vs the copy roofline), `protocol.sizes` (the
reference's round protocol on the GPU at 40 B / 1 MiB / 64 MiB) and `dp.overlap_rehearsal`
(config 5 with real 2-rank comm kernels beside the GEMMs, swept over the reducer grid).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import statistics
import threading
import time

if "--share-device" in sys.argv:
    # Rehearsal with every rank on one GPU: each process's HIP queues are hardware queue
    # slots on the same device; with 8 processes x 4 queues the command processor runs out
    # of slots and time-slices the queues, so the ranks' spinning kernels are no longer
    # co-resident (measured: 46.7 ms vs 3.1 ms per 256 MiB step at 8 ranks). One queue per
    # process keeps every rank's kernel on the device at once. Set before HIP initialises.
    os.environ["GPU_MAX_HW_QUEUES"] = "1"
# (The N = 1 protocol section hosts two plane workers in this process: their rounds share one
# group kernel, csrc/hip/xgmi_plane.cc PlaneGroup - no queue-count setting.)

# Library banners (RCCL's version block, gloo's "connected to N peer ranks") are written to
# fd 1 from native code; keep stdout for the ONE result line: fd 1 -> stderr for the whole
# run, the result goes to a private copy of the original stdout.
sys.stdout.flush()
_RESULT_FD = os.dup(1)
os.dup2(2, 1)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel.comm import LOSSY_ALGOS, CommError, XgmiCommunicator, init_distributed  # noqa: E402
from benchmarks.summary import headline_guard  # noqa: E402
from akka_allreduce_1_amd.utils.timing import busbw, percentile  # noqa: E402

BASELINE_VALUE = None  # the reference publishes no numbers


def log(rank: int, msg: str) -> None:
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def timed(fn, steps: int, dev) -> float:
    """Wall time of `steps` back-to-back calls, barrier + sync on both sides. Nothing else
    is enqueued in between (an event record per step would add a cache flush per step).
    The clock stops once this rank's device has drained; the closing barrier runs after
    it, and the caller takes the MAX over ranks, so the slowest rank decides."""
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    dist.barrier()
    torch.cuda.synchronize(dev)
    return t1 - t0


def event_times(fn, iters: int, dev) -> list[float]:
    """Per-call device times (ms) from event pairs - a separate, untimed pass for p50."""
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
    torch.cuda.synchronize(dev)
    for i in range(iters):
        starts[i].record()
        fn()
        ends[i].record()
    torch.cuda.synchronize(dev)
    return [a.elapsed_time(b) for a, b in zip(starts, ends)]


def max_over_ranks(x: float, dev) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def tolerance(dtype: torch.dtype, world: int, algo: str = "") -> float:
    """Max abs error vs the fp32 sum of `world` uniform(-1, 1) inputs: one rounding of the sum
    (|sum| <= world); the element-type-wire ring rounds each of its P - 1 partials once more."""
    if dtype == torch.float32:
        return 1e-5 * world
    if algo.startswith("ring_native"):
        return 1e-2 * world * world
    return 2e-2 * world


def validate(comm: XgmiCommunicator, n: int, dtype: torch.dtype, dev, rank: int, world: int,
             algo: str = "auto") -> tuple[bool, float]:
    """Engine result vs an fp32 reference sum (computed with RCCL on fp32 copies)."""
    x = torch.empty(n, dtype=dtype, device=dev)
    fill_uniform(x, seed=1000 + rank)
    ref = x.float()
    dist.all_reduce(ref)
    try:  # a timed-out wait must still reach the flag all-reduce below (no rank left blocked)
        y = comm.allreduce(x, algo=algo)
        comm.check()
        err = (y.float() - ref).abs().max().item()
    except CommError:
        err = float("inf")
    ok = err <= tolerance(dtype, world, algo if algo != "auto" else comm._pick(n * x.element_size()))
    flag = torch.tensor([0 if ok else 1], device=dev)
    dist.all_reduce(flag)
    return flag.item() == 0, err


_LINK_NAMES = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}


def topology(world: int) -> dict:
    """Peer access, link type and hop count of every pair of visible devices (rank 0's view):
    the first multi-GPU run records what its cross-GPU stores actually went over."""
    from akka_allreduce_1_amd._native import C

    n = C.hip.device_count()
    peer, link, hops = [], [], []
    for a in range(n):
        pr, lr, hr = [], [], []
        for b in range(n):
            can, t, h = C.hip.link_info(a, b)
            pr.append(int(can))
            lr.append("self" if a == b else _LINK_NAMES.get(t, str(t)))
            hr.append(0 if a == b else h)
        peer.append(pr)
        link.append(lr)
        hops.append(hr)
    return {"devices_visible": n, "ranks": world, "peer_access": peer, "link_type": link, "hops": hops}


def validate_algos(comm: XgmiCommunicator, dtype: torch.dtype, dev, rank: int, world: int) -> dict:
    """Every algorithm the tuner or a section may pick, checked against an fp32 reference
    BEFORE anything is timed, so a first-run failure on new hardware is loud and attributed.
    Every rank regenerates all ranks' inputs from their seeds: the reference needs no
    collective of its own."""
    out: dict = {}

    def inputs(n, seed):
        return [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=seed + k) for k in range(world)]

    cases = [("ll", 100_003), ("oneshot", 300_007), ("twoshot", 5_000_011), ("ring", 5_000_011),
             ("ring_native", 5_000_011)]
    if world > 1 and comm._c.threshold_rows > 0:
        cases.append(("threshold", 2_000_003))
    for algo, n in cases:
        if algo == "ll" and n * torch.empty(0, dtype=dtype).element_size() > comm._c.ll_max_bytes:
            n = comm._c.ll_max_bytes // torch.empty(0, dtype=dtype).element_size() - 5
        xs = inputs(n, 7000 + len(out) * 31)
        ref = torch.zeros(n, device=dev)
        for t in xs:
            ref += t.float()
        try:
            if algo == "threshold":
                y = comm.allreduce_threshold(xs[rank])
            else:
                y = comm.allreduce(xs[rank], algo=algo)
            comm.check()
            err = (y.float() - ref).abs().max().item()
            out[algo] = {"ok": err <= tolerance(dtype, world, algo), "max_abs_err": err, "n": n}
        except Exception as e:  # noqa: BLE001 - reported per algorithm
            out[algo] = {"ok": False, "error": repr(e)}
    m = 65_536
    for name in ("all_to_all", "all_gather", "reduce_scatter"):
        try:
            if name == "all_gather":
                xs = inputs(m, 8100)
                y = comm.all_gather(xs[rank])
                ref = torch.cat([t.float() for t in xs])
            else:
                xs = inputs(world * m, 8200 if name == "all_to_all" else 8300)
                if name == "all_to_all":
                    y = comm.all_to_all(xs[rank])
                    ref = torch.cat([t[rank * m:(rank + 1) * m].float() for t in xs])
                else:
                    y = comm.reduce_scatter(xs[rank])
                    ref = sum(t[rank * m:(rank + 1) * m].float() for t in xs)
            comm.check()
            err = (y.float() - ref).abs().max().item()
            out[name] = {"ok": err <= tolerance(dtype, world), "max_abs_err": err}
        except Exception as e:  # noqa: BLE001
            out[name] = {"ok": False, "error": repr(e)}
    flags = torch.tensor([1 if out[k]["ok"] else 0 for k in out], device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    for k, f in zip(out, flags.tolist()):
        out[k]["validated"] = bool(f)
    return out


def local_ranks(dev, args, P: int = 8) -> dict:
    """P logical ranks in ONE launch on this GPU (LocalCluster), the bench buffer per rank:
    the allreduce kernels themselves at N = 1, where the one-rank headline is only a copy.
    All traffic lands in one HBM, so the yardstick is the copy roofline measured in this
    process: hbm_TBps = protocol bytes (utils.timing.hbm_bytes, PMC-checked) / time."""
    from akka_allreduce_1_amd._native import C
    from akka_allreduce_1_amd.parallel import LocalCluster
    from akka_allreduce_1_amd.utils.timing import hbm_bytes

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    S = args.size_mib << 20
    n = S // es
    row: dict = {"ranks": P, "bytes_per_rank": S, "dtype": args.dtype}
    cl = xs = ys = ref = a = b = None
    try:
        # copy roofline: the engine's own copy kernel, 2 x 256 MiB of traffic per call
        a = torch.empty(S, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        stream = torch.cuda.current_stream(dev).cuda_stream

        def cp():
            C.hip.copy(a.data_ptr(), b.data_ptr(), S, stream)

        for _ in range(args.warmup):
            cp()
        cms = percentile(event_times(cp, args.steps, dev), 50)
        copy_tbps = 2 * S / (cms / 1e3) / 1e12
        row["copy_roofline_TBps"] = round(copy_tbps, 3)
        del a, b
        a = b = None
        # slots of 2 blocks: the exact-wire ring's fp32 partials of a bf16 block fit one launch
        # placement: up to 6 slab placements, timed on buffers of the rank buffers' size (torch's
        # cache hands the same pages to the xs / ys below), the fastest kept
        cl = LocalCluster(P, slot_bytes=2 * -(-S // P) + (1 << 20), grid=512, timeout_s=10.0, placement_tries=6,
                          placement_bytes=S, placement_dtype=dtype)
        row["placement"] = cl.placement
        xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=500 + k) for k in range(P)]
        ys = [torch.empty_like(t) for t in xs]
        ref = torch.zeros(n, device=dev)
        for t in xs:
            ref += t.float()
        for algo in ("twoshot", "ring", "ring_native"):
            def fn(algo=algo):
                cl.allreduce(xs, ys, algo=algo)

            fn()
            cl.check()
            err = max((t.float() - ref).abs().max().item() for t in ys)
            for _ in range(args.warmup):
                fn()
            wall = timed_local(fn, args.steps, dev) / args.steps * 1e3
            p50 = percentile(event_times(fn, args.steps, dev), 50)
            cl.check()
            tbps = hbm_bytes(S, P, algo, es) / (p50 / 1e3) / 1e12
            row[algo] = {"p50_ms": round(p50, 4), "ms_per_step": round(wall, 4), "max_abs_err": err,
                         "validated": err <= tolerance(dtype, P, algo),
                         "hbm_bytes": int(hbm_bytes(S, P, algo, es)), "hbm_TBps": round(tbps, 3),
                         "frac_copy_roofline": round(tbps / copy_tbps, 3)}
            if algo.startswith("ring"):  # per rank per hop, [reduce-scatter, all-gather] (xGMI: link bytes)
                B = S // P
                row[algo]["wire_bytes_per_hop"] = [B * (4 // es if algo == "ring" else 1), B]
    except Exception as e:  # noqa: BLE001 - reported, never loses the headline
        row["error"] = repr(e)
    finally:
        del cl, xs, ys, ref, a, b
        torch.cuda.empty_cache()
    return row


def resolve_auto(comm: XgmiCommunicator, n: int, dtype: torch.dtype) -> str:
    """Name of the kernel the native size policy (Algo.Auto) runs for n elements."""
    from akka_allreduce_1_amd._native import C

    names = {int(C.hip.Algo.TwoShot): "twoshot", int(C.hip.Algo.OneShot): "oneshot",
             int(C.hip.Algo.Ring): "ring", int(C.hip.Algo.LL): "ll", int(C.hip.Algo.RingNative): "ring_native"}
    from akka_allreduce_1_amd.parallel.comm import _KERNEL_DTYPES

    try:
        return names.get(int(comm._c.resolve(n, _KERNEL_DTYPES[dtype], C.hip.Algo.Auto, 1)), "auto")
    except Exception:  # noqa: BLE001 - the label only
        return "auto"


def timed_local(fn, steps: int, dev) -> float:
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0


def collectives(comm: XgmiCommunicator, x: torch.Tensor, world: int, args, dev) -> dict:
    """ms per call of the xGMI all_to_all / all_gather / reduce_scatter vs RCCL on the bench
    buffer (all_gather gathers 1/world of it per rank, so every op moves the same bytes)."""
    n = x.numel()
    m = n // world
    a2a_out = torch.empty_like(x)
    shard = x[:m].contiguous()
    rs_out = torch.empty(m, dtype=x.dtype, device=dev)
    ops = {
        "all_to_all": (lambda: comm.all_to_all(x, a2a_out), lambda: dist.all_to_all_single(a2a_out, x)),
        "all_gather": (lambda: comm.all_gather(shard, a2a_out), lambda: dist.all_gather_into_tensor(a2a_out, shard)),
        "reduce_scatter": (lambda: comm.reduce_scatter(x, rs_out), lambda: dist.reduce_scatter_tensor(rs_out, x)),
    }
    out = {}
    for name, (ours, rccl) in ops.items():
        row = {}
        try:
            for label, fn in (("xgmi", ours), ("rccl", rccl)):
                if label == "rccl" and args.no_rccl:
                    continue
                for _ in range(args.warmup):
                    fn()
                ms = max_over_ranks(timed(fn, args.steps, dev), dev) / args.steps * 1e3
                row[f"{label}_ms"] = round(ms, 4)
                row[f"{label}_algbw"] = round(x.numel() * x.element_size() / (ms / 1e3) / 1e9, 2)
            comm.check()
            if "rccl_ms" in row:
                row["speedup_vs_rccl"] = round(row["rccl_ms"] / row["xgmi_ms"], 3)
        except Exception as e:  # noqa: BLE001 - reported, never loses the headline
            row["error"] = repr(e)
        out[name] = row
    return out


def fused_step(comm: XgmiCommunicator, grads: torch.Tensor, params: torch.Tensor, world: int, rank: int, args,
               dev) -> dict:
    """Sharded-DP optimizer step on the bench buffer (bf16 params, fp32 AdamW shard state):
    the fused launch (csrc/hip/xgmi_adam.hip) vs reduce-scatter + torch fused AdamW + casts +
    all-gather."""
    row = {}
    try:
        hp = dict(lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
        st = comm.adamw_state(params)
        t = {"step": 0}

        def fused():
            t["step"] += 1
            comm.step_adamw(grads, params, st, step=t["step"], **hp)

        b = comm.shard_len(params.numel(), params.dtype)
        shard = torch.empty(b, dtype=params.dtype, device=dev)
        pshard = torch.empty(b, dtype=params.dtype, device=dev)
        master = torch.nn.Parameter(st["master"].clone())
        opt = torch.optim.AdamW([master], fused=True, **hp)

        def unfused():
            comm.reduce_scatter(grads, shard, op="avg")
            master.grad = shard.float()
            opt.step()
            pshard.copy_(master.detach())
            comm.all_gather(pshard, params)

        for label, fn in (("fused", fused), ("unfused", unfused)):
            for _ in range(args.warmup):
                fn()
            row[f"{label}_ms"] = round(max_over_ranks(timed(fn, args.steps, dev), dev) / args.steps * 1e3, 4)
        comm.check()
        row["speedup"] = round(row["unfused_ms"] / row["fused_ms"], 3)
        row["params"] = params.numel()
        if world == 1:  # bytes per param: bf16 grad in + bf16 param out + fp32 master/m/v in and out
            row["hbm_TBps"] = round(28 * params.numel() / (row["fused_ms"] / 1e3) / 1e12, 3)
    except Exception as e:  # noqa: BLE001 - reported, never loses the headline
        row["error"] = repr(e)
    return row


def dp_step(comm: XgmiCommunicator, model: str, dev) -> dict:
    """BASELINE configs 4 / 5 on the same engine: one data-parallel step of a gradient set
    (ResNet-50: 25.6 M params in 161 tensors; Llama-3-8B: 8.03 B params, 16.06 GB bf16),
    every gradient produced by a real GEMM in autograd order while the bucketed reducer
    allreduces full buckets on its own stream, then an SGD update (benchmarks/bench_dp.py has
    the full breakdown). exposed = step - compute-only step; comm_only = every bucket's
    allreduce back to back."""
    from akka_allreduce_1_amd.models.grad_sets import gradient_shapes, numel
    from akka_allreduce_1_amd.parallel import BucketedGradReducer
    from benchmarks.bench_dp import SyntheticBackward

    row: dict = {}
    params = reducer = bwd = grads = None
    try:
        shapes = gradient_shapes(model)
        params = [torch.nn.Parameter(torch.zeros(sh, dtype=torch.bfloat16, device=dev)) for _, sh in shapes]
        big = model == "llama3_8b"
        # Llama-3-8B (16 GB): size-graded buckets - a 64 MiB first bucket starts the overlap
        # early, 1 GiB buckets after it keep the per-bucket hand-off count low (each costs a
        # few us of host time and a compute-stream drain: 163 x 64 MiB buckets exposed 1.1 ms
        # at N = 1, 66 x 256 MiB 0.57 ms). The tail bucket is the 1.05 GB embedding whatever
        # the cap (the last gradient backward produces). ResNet-50: torch DDP's 25 MiB.
        if big:
            reducer = BucketedGradReducer(params, comm, bucket_bytes=1 << 30, first_bucket_bytes=64 << 20,
                                          op="avg")
        else:
            reducer = BucketedGradReducer(params, comm, bucket_bytes=25 << 20, op="avg")
        reducer.remove_hooks()  # the synthetic backward calls the hook itself
        bwd = SyntheticBackward(params, 1024, torch.bfloat16, dev)
        grads = [q.grad for q in params]
        steps, warm = (6, 1) if big else (20, 3)

        def overlap():
            bwd.run(reducer)
            reducer.wait()
            torch._foreach_add_(params, grads, alpha=-1e-3)

        def compute():
            bwd.run(None)
            torch._foreach_add_(params, grads, alpha=-1e-3)

        def comm_only():
            for b in reducer.buckets:
                comm.allreduce_(b.buffer, op="avg")

        with torch.no_grad():
            t = {}
            for fn in (overlap, compute, comm_only):
                for _ in range(warm):
                    fn()
            # step and compute-only alternate one step at a time and each takes its median:
            # the exposed time is a ~1 % difference of two 30 ms steps, which clock drift
            # between two back-to-back blocks of steps swamps (tools/reducer_overhead.py)
            per = {"step": [], "compute": []}
            for _ in range(steps):
                per["step"].append(timed(overlap, 1, dev))
                per["compute"].append(timed(compute, 1, dev))
            for name, v in per.items():
                t[name] = max_over_ranks(statistics.median(v), dev) * 1e3
            t["comm"] = max_over_ranks(timed(comm_only, steps, dev), dev) / steps * 1e3
            if comm.world > 1:
                # the same step with the bucket launches capped at 128 workgroups: a reduce
                # running beside backward's GEMMs competes for CUs (ddp.py `algo`)
                reducer.algo = "twoshot@128"
                for _ in range(warm):
                    overlap()
                t["step_g128"] = max_over_ranks(timed(overlap, steps, dev), dev) / steps * 1e3
                # the copy-engine allreduce (parallel/sdma.py): xGMI transfers off the CUs
                try:
                    reducer.algo = "sdma"
                    for _ in range(warm):
                        overlap()
                    t["step_sdma"] = max_over_ranks(timed(overlap, steps, dev), dev) / steps * 1e3
                except Exception as e:  # noqa: BLE001 - recorded, the other schedules still run
                    t["sdma_error"] = repr(e)
                reducer.algo = "auto"
                # every bucket after backward (no overlap)
                reducer.overlap = False
                for _ in range(warm):
                    overlap()
                t["step_serial"] = max_over_ranks(timed(overlap, steps, dev), dev) / steps * 1e3
                reducer.overlap = True
                # the reducer's own choice: one tuning step per candidate schedule, agreed
                # over the ranks, then the kept schedule timed (ddp.py overlap="auto")
                reducer.tune_schedule(tune_steps=1)
                for _ in range(len(reducer._cands)):
                    overlap()
                for _ in range(warm):
                    overlap()
                t["step_auto"] = max_over_ranks(timed(overlap, steps, dev), dev) / steps * 1e3
        comm.check()
        nbytes = sum(b.nbytes for b in reducer.buckets)
        row = {"params": sum(numel(sh) for _, sh in shapes), "grad_bytes": nbytes, "buckets": len(reducer.buckets),
               "bucket_bytes": [reducer.buckets[0].nbytes, max(b.nbytes for b in reducer.buckets)],
               "step_ms": round(t["step"], 3), "compute_ms": round(t["compute"], 3),
               "exposed_comm_ms": round(t["step"] - t["compute"], 3), "steps": steps}
        if comm.world > 1:
            row["comm_only_ms"] = round(t["comm"], 3)
            row["comm_algbw_per_rank"] = round(nbytes / (t["comm"] / 1e3) / 1e9, 2)
        else:  # an average over one rank is the identity: no kernel runs, nothing to rate
            row["note"] = ("world=1: the allreduce is the identity (no launch), so exposed_comm_ms is the "
                           "reducer's host overhead; comm-only time / bandwidth are not measured")
        if "step_sdma" in t:
            row["step_ms_sdma"] = round(t["step_sdma"], 3)
        if "sdma_error" in t:
            row["sdma_error"] = t["sdma_error"][:200]
        if "step_g128" in t:
            row["step_ms_twoshot_128wg"] = round(t["step_g128"], 3)
            row["step_ms_serial"] = round(t["step_serial"], 3)
            row["step_ms_auto_schedule"] = round(t["step_auto"], 3)
            row["auto_schedule"] = reducer.stats.get("schedule")
            row["auto_schedule_tuning_ms"] = reducer.stats.get("schedule_ms")
    except Exception as e:  # noqa: BLE001 - reported, never loses the headline
        row["error"] = repr(e)
    finally:
        del params, reducer, bwd, grads
        torch.cuda.empty_cache()
    return row


def bridge_driven_rounds(P, n, chunk, dtype, rounds, warm, xs, ref) -> dict:
    """The same job with the rounds driven from OUTSIDE the engine: a control-bridge client
    (docs/BRIDGE.md, JSON lines over TCP, the way a JVM Akka client would) sends each
    StartAllreduce, pipelined (the next start queued while a round runs); timed by the
    client's RoundComplete arrivals."""
    from akka_allreduce_1_amd.bridge import BridgeClient
    from akka_allreduce_1_amd.engine import PlaneJob

    row: dict = {"driver": "control-bridge client, pipelined StartAllreduce (JSON lines over TCP)"}
    job = PlaneJob(P, n, max_chunk_size=chunk, dtype=dtype, max_round=rounds - 1, sources=xs,
                   keep_outputs=False, keep_last=True, timeout_s=20.0, bridge_port=0, external_rounds=True)
    try:
        job.start()
        stamps = []
        with BridgeClient("127.0.0.1", job.bridge_port, timeout=60) as b:
            b.wait_for("InitWorkers")
            b.start(0)
            for r in range(rounds):
                if r + 1 < rounds:
                    b.start(r + 1)
                b.wait_for("RoundComplete", round=r)
                stamps.append(time.perf_counter())
        if not job.finished.wait(30):
            raise TimeoutError("bridge-driven job did not finish")
        for p in job.planes:
            p.drain()
        o = job.last_output(0)
        row["validated"] = bool(o is not None and o.iteration == rounds - 1 and torch.equal(o.data, ref))
        per = (stamps[-1] - stamps[warm - 1]) / (len(stamps) - warm)
        row["ms_per_round"] = round(per * 1e3, 4)
        row["rounds_per_s"] = round(1.0 / per, 2)
    except Exception as e:  # noqa: BLE001 - reported, never loses the protocol row
        row["error"] = repr(e)
    finally:
        job.shutdown()
    return row


def protocol_rounds(args, rank: int, world: int, dev) -> dict:
    """The reference's protocol driving the GPU engine: the master's
    StartAllreduce(r) becomes one threshold-kernel round per worker on the xGMI round plane
    (csrc/runtime/plane_worker.h, csrc/hip/xgmi_plane.h), CompleteAllreduce goes back, the
    master starts r + 1 at the barrier - the bench buffer per worker, th = 1, maxLag 1.
    N = 1: two workers in this process share the GPU (all traffic in one HBM). N > 1: one
    worker per GPU process, master on rank 0, control over TCP, data over xGMI.
    rounds_per_s / ms_per_round come from the master's round-barrier stamps after the
    warm-up rounds; algbw = buffer bytes / ms_per_round."""
    from akka_allreduce_1_amd.engine import PlaneJob, distributed_plane_job

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    nbytes = args.size_mib << 20
    n = nbytes // es
    warm = max(1, args.warmup)
    rounds = warm + max(args.steps, 10)
    P = 2 if world == 1 else world
    block = -(-n // P)
    chunk = max(1024, -(-block // 256))  # ~256 reduce units per worker: one per workgroup pair of CUs
    row: dict = {"workers": P, "bytes_per_worker": nbytes, "dtype": args.dtype, "rounds": rounds,
                 "warmup_rounds": warm, "th_reduce": 1.0, "th_complete": 1.0, "max_lag": 1,
                 "max_chunk_size": chunk, "engine": "PlaneWorkerActor + XgmiRoundPlane (threshold kernel)",
                 "io": "tensor dataSource + native keep-last dataSink (no Python per round)"}
    try:
        if world == 1:
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=700 + k) for k in range(P)]
            last = {}
            log(rank, f"protocol: {P} plane workers on this GPU, {rounds} rounds of {args.size_mib} MiB")
            # the gradient buffers themselves are the dataSources and a native sink keeps the
            # newest output: no Python (GIL) on the round path (engine.PlaneJob)
            job = PlaneJob(P, n, max_chunk_size=chunk, dtype=dtype, max_round=rounds - 1, sources=xs,
                           keep_outputs=False, keep_last=True, timeout_s=20.0)
            try:
                job.run(timeout=300)
                stamps = job.stamps
                lat = job.system.plane_worker_state(job.workers[0])["round_latency"]
                o = job.last_output(0)
                if o is not None and o.iteration == rounds - 1:
                    last["y"] = o.data.clone()
                row["note"] = "N=1: 2 workers share one GPU (one HBM, no xGMI)"
            finally:
                job.shutdown()
            ref = (xs[0].float() + xs[1].float()).to(dtype)
            row["validated"] = bool(torch.equal(last["y"], ref))
            row["bridge"] = bridge_driven_rounds(P, n, chunk, dtype, rounds, warm, xs, ref)
        else:
            x = fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=700 + rank)
            last = {}
            # ranks sharing one GPU (rehearsal): separate kernels, one per process, together two
            # workgroups per CU (profiles/round5/rehearsal_grid.jsonl: 8 processes x 32 lose to x 64)
            grid = (args.plane_grid or max(8, 512 // world)) if args.share_device else 0
            log(rank, f"protocol: one plane worker per rank, {rounds} rounds of {args.size_mib} MiB")
            # one GPU per rank: host threads poll through the rounds (--spin-us 500 of the native
            # executables); ranks sharing one GPU (rehearsal) share the box's few CPUs: no polling
            spin = None if args.share_device else 500
            res = distributed_plane_job(n, x, max_chunk_size=chunk, dtype=dtype, rounds=rounds,
                                        grid=grid, keep_last=True, timeout_s=120.0, host_spin_us=spin)
            if res["last"] is not None and res["last"].iteration == rounds - 1:
                last["y"] = res["last"].data.clone()
            stamps = res["stamps"]
            lat = res["state"]["round_latency"]
            # the kernel sums in WORKER-id order (ids are dense in the master's join order, not
            # torch ranks): the fp32 reference must add the ranks' inputs in that order
            ids = [None] * world
            dist.all_gather_object(ids, res["state"]["id"])
            ref = torch.zeros(n, device=dev)
            for k in sorted(range(world), key=lambda q: ids[q]):
                ref += fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=700 + k).float()
            row["worker_ids"] = ids
            st = res["state"]["stats"]
            mine = {"rank": rank, "output": "y" in last, "plane_errors": st["plane_errors"],
                    "forced": st["forced_completions"], "cold": st["cold_rounds"]}
            if "y" in last:
                diff = (last["y"].float() - ref.to(dtype).float()).abs()
                mine["bad"] = int((diff > 0).sum().item())
                mine["max_abs_err"] = float(diff.max().item())
                if mine["bad"]:  # the first few mismatches with every rank's input (bf16 bits as floats)
                    idx = torch.nonzero(diff > 0).flatten()[:3].tolist()
                    xs_all = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=700 + k) for k in range(world)]
                    mine["first_bad"] = [{"i": i, "got": float(last["y"][i].float()), "ref_f32": float(ref[i]),
                                          "inputs": [float(xk[i].float()) for xk in xs_all]} for i in idx]
                    del xs_all
            good = torch.tensor([1 if (mine.get("bad", 1) == 0 and not mine["plane_errors"]) else 0], device=dev)
            dist.all_reduce(good, op=dist.ReduceOp.MIN)
            row["validated"] = bool(good.item())
            if not row["validated"]:  # which rank, how many elements, kernel error words
                detail = [None] * world
                dist.all_gather_object(detail, mine)
                row["validation_detail"] = detail
            row["note"] = "one worker per GPU process; master on rank 0; control over TCP, data over xGMI"
            if row["validated"]:  # the same job with rounds driven by a control-bridge client on rank 0
                b: dict = {"driver": "control-bridge client on rank 0, pipelined StartAllreduce (JSON lines over TCP)"}
                res2 = distributed_plane_job(n, x, max_chunk_size=chunk, dtype=dtype, rounds=rounds, grid=grid,
                                             keep_last=True, timeout_s=45.0, external_client=True,
                                             host_spin_us=spin)
                ids2 = [None] * world
                dist.all_gather_object(ids2, res2["state"]["id"])
                ref2 = torch.zeros(n, device=dev)
                for k in sorted(range(world), key=lambda q: ids2[q]):
                    ref2 += fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=700 + k).float()
                y2 = res2["last"]
                ok2 = bool(res2["ok"] and y2 is not None and y2.iteration == rounds - 1
                           and torch.equal(y2.data, ref2.to(dtype)))
                del ref2
                good2 = torch.tensor([1 if ok2 else 0], device=dev)
                dist.all_reduce(good2, op=dist.ReduceOp.MIN)
                b["validated"] = bool(good2.item())
                st2 = res2["stamps"]
                if len(st2) > warm + 1:
                    per2 = (st2[-1] - st2[warm - 1]) / (len(st2) - warm)
                    b["ms_per_round"] = round(per2 * 1e3, 4)
                    b["rounds_per_s"] = round(1.0 / per2, 2)
                row["bridge"] = b
        if len(stamps) > warm + 1:
            per = (stamps[-1] - stamps[warm - 1]) / (len(stamps) - warm)
            row["ms_per_round"] = round(per * 1e3, 4)
            row["rounds_per_s"] = round(1.0 / per, 2)
            row["algbw_per_worker"] = round(nbytes / per / 1e9, 2)
        row["worker_round_latency_p50_ms"] = round(lat["p50_ms"], 4)
        row["worker_round_latency_p99_ms"] = round(lat["p99_ms"], 4)
    except Exception as e:  # noqa: BLE001 - reported, never loses the headline
        row["error"] = repr(e)
    return row


_EMIT_LOCK = threading.Lock()
_EMITTED = [False]


_DETAIL = {"path": None}


def write_detail(result: dict) -> str | None:
    """The full result dict (every section, size and candidate) goes to a side file; the
    stdout line carries compact summaries and names this file (benchmarks/summary.py)."""
    path = _DETAIL["path"]
    if not path:
        return None
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(result, f, indent=1)
        return path
    except OSError as e:
        log(0, f"could not write {path}: {e}")
        return None


def result_line(result: dict) -> str:
    """ONE JSON line <= summary.LINE_BUDGET bytes, the full dict written to the detail file."""
    from benchmarks.summary import line

    return line(result, write_detail(result)) + "\n"


def emit(rank: int, result: dict) -> bool:
    """Write the ONE result line (rank 0), at most once per process: the dp watchdog and the
    main path may both get here. Returns True for the caller that wrote it."""
    with _EMIT_LOCK:
        if _EMITTED[0]:
            return False
        _EMITTED[0] = True
        if rank == 0:
            text = result_line(result)
            sys.stdout.flush()
            with os.fdopen(_RESULT_FD, "w") as out:
                out.write(text)
        return True


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--algo", choices=["auto", "twoshot", "oneshot", "ll", "ring", "ring_native", "threshold", "rccl",
                                       "rsag", "p2p"],
                    default="auto")
    ap.add_argument("--no-rccl", action="store_true", help="skip the RCCL comparison timing")
    ap.add_argument("--no-tune", action="store_true", help="skip the size sweep / algorithm tuner")
    ap.add_argument("--sweep-steps", type=int, default=10)
    ap.add_argument("--no-threshold", action="store_true", help="skip the straggler-tolerant kernel timing")
    ap.add_argument("--no-collectives", action="store_true", help="skip the all-to-all / all-gather / reduce-scatter timing")
    ap.add_argument("--no-fused-step", action="store_true", help="skip the fused reduce-scatter + AdamW + all-gather timing")
    ap.add_argument("--no-dp", action="store_true", help="skip the ResNet-50 / Llama-3-8B DP-step sections")
    ap.add_argument("--no-local", action="store_true", help="skip the 8-logical-rank section at N = 1")
    ap.add_argument("--no-links", action="store_true", help="skip the xGMI bring-up probes at N > 1")
    ap.add_argument("--no-sdma", action="store_true", help="skip the copy-engine allreduce section at N > 1")
    ap.add_argument("--no-protocol", action="store_true", help="skip the master/worker protocol-engine section")
    ap.add_argument("--no-native", action="store_true",
                    help="skip the native-deployment protocol rounds (child mxar processes; e.g. under a profiler)")
    ap.add_argument("--no-sizes", action="store_true",
                    help="skip the N = 1 size-axis sections (latency_vs_size, reduce_kernel, protocol sizes)")
    ap.add_argument("--no-stragglers", action="store_true",
                    help="skip the straggler-tolerance section at N = 1 (benchmarks/stragglers.py)")
    ap.add_argument("--stragglers-budget", type=float, default=90.0, help="seconds for the straggler section")
    ap.add_argument("--protocol-timeout", type=float, default=240.0,
                    help="native watchdog over the protocol section (s); the result line is written either way")
    ap.add_argument("--dp-rehearsal", action="store_true", help="with --share-device: run the ResNet-50 DP step too")
    ap.add_argument("--dp-timeout", type=float, default=240.0,
                    help="seconds for the DP-step sections; past it the result line is written without them")
    ap.add_argument("--detail-out", default=None,
                    help="side file for the full result dict (default gpurun_out/bench_detail_n<N>.json; '' = none)")
    ap.add_argument("--plane-grid", type=int, default=0,
                    help="with --share-device: workgroups per protocol worker (0: 512 / ranks)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal: every rank on cuda:0 over gloo (RCCL refuses two ranks on one GPU), "
                         "workgroup budget split between the ranks so all spinning workgroups stay resident")
    args = ap.parse_args()

    rank, world, local = init_distributed("gloo" if args.share_device else "nccl")
    if rank == 0:
        _DETAIL["path"] = (os.path.join("gpurun_out", f"bench_detail_n{world}.json") if args.detail_out is None
                           else args.detail_out or None)
    if world != args.gpus:
        log(rank, f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}")
    grid = 0
    if args.share_device:
        local, args.no_rccl = 0, True
        torch.cuda.set_device(0)
        grid = max(8, 512 // world)
    dev = torch.device("cuda", local)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    es = 2 if dtype == torch.bfloat16 else 4
    nbytes = args.size_mib << 20
    n = nbytes // es
    slot = max(64 << 20, -(-nbytes // world) + (1 << 20))

    # ---- engine bring-up + validation; any failure degrades to RCCL (recorded) instead of
    # losing the run
    comm, reason, err = None, "", float("nan")
    t_setup = time.perf_counter()
    log(rank, f"bring-up: world={world} slot={slot >> 20} MiB")
    try:
        # max_lag=1: a lag ring for the straggler-tolerant kernel, timed after the headline
        # (the lock-step kernels use slab row 0 only; the extra rows cost HBM, not time)
        comm = XgmiCommunicator(slot_bytes=slot, grid=grid, max_lag=1 if world > 1 else None)
        log(rank, f"{comm}  tensor={args.size_mib} MiB {args.dtype}  (setup {time.perf_counter() - t_setup:.1f} s)")
        ok, err = validate(comm, n, dtype, dev, rank, world)
        ok_small, err_small = validate(comm, 12345, dtype, dev, rank, world)
        if not (ok and ok_small):
            reason = f"validation failed (max err {err:.3g} / {err_small:.3g})"
    except Exception as e:  # noqa: BLE001 - reported in the JSON
        reason = f"engine unavailable: {e!r}"
    healthy = torch.tensor([0 if reason else 1], device=dev)
    dist.all_reduce(healthy, op=dist.ReduceOp.MIN)
    if healthy.item() == 0 and not reason:
        reason = "engine failed on another rank"
    engine_ok = healthy.item() == 1
    if not engine_ok:
        log(rank, f"ENGINE DISABLED: {reason}; timing RCCL")

    x = torch.empty(n, dtype=dtype, device=dev)
    fill_uniform(x, seed=rank)
    y = torch.empty_like(x)

    def step_rccl():
        y.copy_(x)
        dist.all_reduce(y)

    validated = None
    if engine_ok:
        log(rank, "validating every algorithm against fp32")
        # every algorithm a section or the tuner may pick, against fp32, before any timing
        validated = validate_algos(comm, dtype, dev, rank, world)
        bad = [k for k, v in validated.items() if not v["validated"]]
        if bad:
            log(rank, f"VALIDATION FAILED for {bad}: {[validated[k] for k in bad]}")
            # a timed-out wait poisons the communicator: every rank saw the same `bad` list
            # (the flags were all-reduced), so all of them take part in the collective reset
            try:
                comm.reset()
            except Exception as e:  # noqa: BLE001 - recorded, the run degrades to RCCL
                engine_ok, reason = False, f"reset after failed validation: {e!r}"
    ok_algos = {k for k, v in (validated or {}).items() if v["validated"]}
    links = None
    if engine_ok and world > 1 and not args.no_links:
        # the xGMI bring-up pack, before anything else is timed: per-link push rate, all-peer
        # fan-out rate and flag hand-off latency on the engine's own store path
        # (akka_allreduce_1_amd/utils/links.py), so a slow first multi-GPU run is attributable
        from akka_allreduce_1_amd.utils.links import probe_links

        log(rank, "xgmi_links: per-link push rates, fan-out, flag latency")
        try:
            links = probe_links(comm, nbytes=min(nbytes, 64 << 20))
        except Exception as e:  # noqa: BLE001 - recorded, never loses the headline
            links = {"error": repr(e)}
            try:
                comm.reset()
            except Exception as e2:  # noqa: BLE001
                engine_ok, reason = False, f"reset after link probe failure: {e2!r}"
    sweep = None
    if engine_ok and not args.no_tune and world > 1:  # at world = 1 every candidate is the same copy
        # RCCL / RS+AG are timed as comparison columns (rccl_p50_us, speedup_vs_rccl per size):
        # tune() never adopts a library path, so the headline is always this engine's kernel
        lib = () if args.no_rccl else ("rccl", "rsag")
        cands = tuple(c for c in ("ll", "oneshot", "twoshot", "ring", "ring_native", "threshold") if c in ok_algos) + lib
        sweep = comm.tune(max_bytes=nbytes, dtype=dtype, iters=args.sweep_steps, candidates=cands,
                          grids=(128, 256))
    status = "ok"
    if engine_ok and args.algo != "rccl":
        algo = args.algo
        chosen = comm._pick(nbytes) if algo == "auto" else algo
        if world > 1 and chosen == "auto":  # the built-in size policy: name the kernel it runs
            chosen = resolve_auto(comm, n, dtype)
        # never time an unvalidated kernel ("auto" without a tuned table is the size-default
        # dispatch, checked by validate() above); a failure is reported as such, never
        # replaced by the library's number
        # a per-hop-rounded kernel or a library path is never the automatic headline (lower
        # precision than the reference's fp32 sums / not this engine): tune(exact_only=True)
        # never adopts one, a hand-set table entry is replaced here and said so
        guarded, note = headline_guard(chosen, args.algo, world)
        if note:
            log(rank, note)
            status, algo, chosen = note, guarded, guarded
        if world > 1 and chosen.split("@")[0].split("~")[0] not in ok_algos | {"auto"}:
            log(rank, f"headline algorithm {chosen} failed validation")
            status = f"headline kernel {chosen} failed validation"
        elif world > 1 and sweep is not None:
            # the tuned headline configuration (algorithm, grid, geometry) at the full size
            ok_tuned, err_tuned = validate(comm, n, dtype, dev, rank, world, algo=chosen)
            if not ok_tuned:
                log(rank, f"tuned headline {chosen} failed validation (max err {err_tuned:.3g})")
                comm.reset()
                status = f"tuned headline {chosen} failed validation"
                algo = chosen = "twoshot"
        if world == 1:  # XgmiComm::run: a 1-rank sum is an out-of-place copy, whatever the algorithm
            chosen = "copy (world=1)"

        def step():
            comm.allreduce(x, y, algo=algo)
    else:
        chosen = "rccl (--algo rccl)" if engine_ok else "rccl-fallback"
        status = "ok" if engine_ok else "engine_failed: value is RCCL's, not this framework's"
        step = step_rccl

    log(rank, f"headline: {chosen}, {args.warmup} + {args.steps} steps")
    for _ in range(args.warmup):
        step()
    wall = timed(step, args.steps, dev)
    per = event_times(step, args.steps, dev)
    if engine_ok:
        try:
            comm.check()
        except CommError as e:
            log(rank, f"engine error during timing: {e}")
            chosen += " (ERROR during timing)"
    wall = max_over_ranks(wall, dev)
    ms = wall / args.steps * 1e3
    algbw = nbytes / (ms / 1e3) / 1e9
    p50 = max_over_ranks(percentile(per, 50), dev)

    result = {
        "metric": "allreduce_algbw",
        "value": round(algbw, 2),
        "value_note": ("nccl-tests algbw = buffer bytes / time of the slowest rank (the job reduces S bytes per "
                       "step); algbw_sum_over_ranks = n_gpus x algbw"),
        "algbw_per_rank": round(algbw, 2),
        "algbw_sum_over_ranks": round(algbw * world, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None if BASELINE_VALUE is None else round(algbw / BASELINE_VALUE, 3),
        "dtype": args.dtype,
        "data": "synthetic uniform(-1,1) gradient buffer per rank",
        "config": {
            "model": f"flat {args.size_mib} MiB {args.dtype} gradient buffer (BASELINE config 3)",
            "global_batch": world,
            "seq_len": None,
            "parallelism": f"dp{world}" + (" (rehearsal: all ranks on one GPU)" if args.share_device else ""),
            "tensor_bytes": nbytes,
            "algo": chosen,
            "wire": ("element type per hop (rounded P-1 times)" if chosen.split("@")[0] in LOSSY_ALGOS
                     else "fp32 accumulation, rounded once" if args.dtype == "bf16" else "fp32"),
        },
        "p50_ms": round(p50, 4),
        "busbw": round(busbw(algbw, world), 2),
        "validated_max_abs_err": err,
        "engine_ok": engine_ok,
        "status": status,
    }
    if world == 1:
        result["value_note"] += ("; world=1: the allreduce is an out-of-place HBM copy (no communication) - "
                                 "see local_ranks for the allreduce kernels on this GPU")
    if validated is not None:
        result["validated"] = {k: v["validated"] for k, v in validated.items()}
        result["validation"] = validated
    if rank == 0:
        try:
            result["topology"] = topology(world)
        except Exception as e:  # noqa: BLE001
            result["topology"] = {"error": repr(e)}
    if reason:
        result["engine_note"] = reason
    if links is not None:
        result["xgmi_links"] = links

    if engine_ok and not chosen.startswith("twoshot") and world > 1:
        for _ in range(args.warmup):
            comm.allreduce(x, y, algo="twoshot")
        twall = timed(lambda: comm.allreduce(x, y, algo="twoshot"), args.steps, dev)
        tms = max_over_ranks(twall, dev) / args.steps * 1e3
        result["xgmi_twoshot"] = {"algbw": round(nbytes / (tms / 1e3) / 1e9, 2), "ms_per_step": round(tms, 4)}
    if not args.no_rccl and not chosen.startswith("rccl") and world > 1:
        # (at world = 1 RCCL's allreduce is a no-op after a copy: nothing to compare)
        for _ in range(args.warmup):
            step_rccl()
        rwall = timed(step_rccl, args.steps, dev)
        rper = event_times(step_rccl, args.steps, dev)
        rms = max_over_ranks(rwall, dev) / args.steps * 1e3
        r_alg = nbytes / (rms / 1e3) / 1e9
        result["rccl"] = {"algbw": round(r_alg, 2), "ms_per_step": round(rms, 4),
                          "p50_ms": round(max_over_ranks(percentile(rper, 50), dev), 4),
                          "note": "copy + in-place dist.all_reduce (nccl backend = RCCL)"}
        result["speedup_vs_rccl"] = round(algbw / r_alg, 3)
    # the optional sections below only run on a healthy engine (every rank's error word 0),
    # so one timed-out launch can never cascade into a chain of 20-s device deadlines
    if engine_ok:
        e = torch.tensor([1 if comm.error() == 0 else 0], device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MIN)
        if e.item() == 0:
            log(rank, "engine error word set: optional sections skipped")
            engine_ok = False
    if engine_ok and world > 1 and not args.no_threshold:
        # the reference's round semantics (thReduce / thComplete / maxLag) on the same buffer,
        # at th = 1 so every rank must still deliver: the cost of straggler tolerance itself
        try:
            def step_th():
                comm.allreduce_threshold(x, y, th_reduce=1.0, th_complete=1.0)

            for _ in range(args.warmup):
                step_th()
            thw = max_over_ranks(timed(step_th, args.steps, dev), dev) / args.steps * 1e3
            comm.check()
            ref = x.float()
            dist.all_reduce(ref)
            step_th()
            terr = max_over_ranks((y.float() - ref).abs().max().item(), dev)
            result["xgmi_threshold"] = {"algbw": round(nbytes / (thw / 1e3) / 1e9, 2), "ms_per_step": round(thw, 4),
                                        "max_abs_err": terr, "th_reduce": 1.0, "th_complete": 1.0, "max_lag": 1}
        except Exception as e:  # noqa: BLE001 - reported, never loses the headline
            result["xgmi_threshold"] = {"error": repr(e)}
    if engine_ok and world > 1 and not args.no_collectives:
        # the allreduce's two halves and the all-to-all as collectives of their own
        # (csrc/hip/xgmi_coll.hip) on the same bytes, next to RCCL's equivalents
        log(rank, "collectives")
        result["collectives"] = collectives(comm, x, world, args, dev)
    if engine_ok and not args.no_fused_step:
        log(rank, "fused AdamW step")
        result["fused_adamw_step"] = fused_step(comm, x, y, world, rank, args, dev)
    if engine_ok and world > 1 and not args.no_sdma and args.share_device and 2 * world > 12:
        # every rank's child would open the one shared GPU too: 2 x world processes on it,
        # past what a rehearsal box admits (16) - on a node it is 2 per GPU
        result["sdma"] = {"skipped": "share-device rehearsal with more than 6 ranks (2 processes per rank on one GPU)"}
    elif engine_ok and world > 1 and not args.no_sdma:
        # the copy-engine allreduce across the GPUs, first in child processes (a fault there
        # cannot cost this line); validated on every rank -> the DP tuner may use it too
        from akka_allreduce_1_amd.parallel.comm import free_port
        from akka_allreduce_1_amd.parallel.sdma import mark_xdev_validated
        from benchmarks.sdma_xdev import run_children

        log(rank, "sdma: copy-engine allreduce across the ranks (child processes)")
        port = [free_port() if rank == 0 else 0]
        dist.broadcast_object_list(port, src=0)
        torch.cuda.synchronize(dev)
        mine = run_children(rank, world, local, port[0], mib=args.size_mib)
        rows = [None] * world
        dist.all_gather_object(rows, mine)
        ok = all(r.get("validated") for r in rows)
        p50 = [r.get("p50_ms") for r in rows if r.get("p50_ms") is not None]
        result["sdma"] = {"validated": ok, "cross_gpu": bool(rows[0].get("cross_gpu")),
                          "p50_ms": max(p50) if len(p50) == world else None,
                          "algbw": round(nbytes / (max(p50) / 1e3) / 1e9, 2) if len(p50) == world else None,
                          "max_abs_err": max((r.get("max_abs_err") or 0.0) for r in rows),
                          "errors": [r.get("error") for r in rows if r.get("error")][:2]}
        if ok:
            mark_xdev_validated()
    if sweep is not None:
        result["sweep"] = sweep
    if engine_ok and world == 1 and not args.share_device and not args.no_local:
        # the allreduce kernels at N = 1: 8 logical ranks in one launch on this GPU
        log(rank, "local_ranks: 8 logical ranks in one launch")
        result["local_ranks"] = local_ranks(dev, args, P=8)
        if not args.no_sizes:
            from benchmarks.sections import latency_vs_size, reduce_kernel

            # the headline metric's size axis: p50 latency + algbw per kernel, 4 KiB .. 256 MiB
            log(rank, "latency_vs_size: 8 and 2 logical ranks, 4 KiB .. 256 MiB")
            result["latency_vs_size"] = latency_vs_size(dev, dtype, max_bytes=nbytes)
            log(rank, "reduce_kernel: BASELINE config 2 (1 GiB fp32, P = 2 / 4 / 8)")
            result["reduce_kernel"] = reduce_kernel(dev)
            from benchmarks.sections import sdma_local

            log(rank, "sdma_local: the copy-engine allreduce, 2 / 8 logical ranks")
            result["sdma_local"] = sdma_local(dev, dtype, nbytes)
    if engine_ok and not args.no_protocol:
        # the reference's master/worker round protocol driving the GPU engine, under the same
        # native watchdog as the dp section: a stuck round never costs the result line
        from akka_allreduce_1_amd._native import C

        timed_out = dict(result, protocol={"error": f"timed out after {args.protocol_timeout:g} s"},
                         status="protocol_timeout")
        sys.stdout.flush()
        cancel = C.watchdog_arm(args.protocol_timeout, _RESULT_FD if rank == 0 else -1,
                                result_line(timed_out) if rank == 0 else "\n", 3)
        prot = protocol_rounds(args, rank, world, dev)
        if world == 1 and not args.no_sizes:
            from benchmarks.sections import protocol_sizes

            log(rank, "protocol: 40 B / 1 MiB / 64 MiB rounds")
            prot["sizes"] = protocol_sizes(dev)
            if not args.no_native:
                from benchmarks.sections import native_deployment

                log(rank, "protocol: native deployment (mxar master + 2 mxar-gpu processes)")
                prot["native"] = native_deployment()
        if not cancel():  # the watchdog fired and wrote the line; the process is exiting
            return
        result["protocol"] = prot
    if engine_ok and world == 1 and not args.share_device and not args.no_stragglers:
        # straggler tolerance, timed (the reference's thresholds / maxLag with one slow worker),
        # under its own native watchdog: a stuck round never costs the result line
        from akka_allreduce_1_amd._native import C
        from benchmarks.stragglers import section as straggler_section

        timed_out = dict(result, stragglers={"error": f"timed out after {2 * args.stragglers_budget:g} s"},
                         status="stragglers_timeout")
        sys.stdout.flush()
        cancel = C.watchdog_arm(2 * args.stragglers_budget + 60, _RESULT_FD if rank == 0 else -1,
                                result_line(timed_out) if rank == 0 else "\n", 3)
        log(rank, "stragglers: reference default job, P = 4 straggler sweep, native 2-process shape")
        strag = straggler_section(dev, budget_s=args.stragglers_budget)
        if not cancel():
            return
        result["stragglers"] = strag
    if engine_ok and not args.no_dp and (not args.share_device or args.dp_rehearsal):
        # configs 4 / 5 (full Llama-3-8B: 32 GB of params + grads per rank). Not in the
        # one-GPU rehearsal: there every rank's spinning comm kernel shares the device with the
        # other ranks' GEMMs (8 ranks: 953 ms per overlapped ResNet-50 step vs 5.9 ms compute +
        # 0.8 ms comm), which says nothing about one GPU per rank. A watchdog keeps a stuck
        # section from costing the result line.
        # The watchdog is native: it writes the prepared line (explicit status "dp_timeout")
        # and exits even while this thread is blocked in a C call holding the GIL - a
        # Python Timer could not run then (seen in the 8-process one-GPU rehearsal). It
        # exits at once because a persistent kernel of the stuck section may still spin.
        from akka_allreduce_1_amd._native import C

        timed_out = dict(result, dp={"error": f"timed out after {args.dp_timeout:g} s"}, status="dp_timeout")
        sys.stdout.flush()
        cancel = C.watchdog_arm(args.dp_timeout, _RESULT_FD if rank == 0 else -1,
                                result_line(timed_out) if rank == 0 else "\n", 3)
        log(rank, "dp: ResNet-50 / Llama-3-8B data-parallel steps")
        dp = {m: dp_step(comm, m, dev) for m in (("resnet50",) if args.share_device else ("resnet50", "llama3_8b"))}
        if world == 1 and not args.share_device and not args.no_sizes:
            # the same steps with REAL comm kernels beside the GEMMs (one rank of an 8-GPU
            # two-shot per bucket, run alone: a real rank's per-GPU HBM bytes), serial vs
            # overlapped vs CU slices vs paced grids
            from benchmarks.sections import dp_overlap

            log(rank, "dp.overlap_rehearsal: one rank of an 8-GPU two-shot per bucket beside backward")
            dp["overlap_rehearsal"] = dp_overlap(dev)
        if not cancel():  # the watchdog fired and wrote the line; the process is exiting
            return
        result["dp"] = dp

    emit(rank, result)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
