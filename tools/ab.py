#!/usr/bin/env python3
"""One driver for same-box A/B measurements. Each experiment prints one JSON line per
measurement; settings come from the environment, so an A/B is the same experiment run
interleaved under different settings (study knobs need MXAR_STUDY=1, docs/TUNING.md):

    MXAR_STUDY=1 MXAR_TH_ONESHOT_MAX=0 python tools/ab.py threshold --tag twoshot-body
    python tools/ab.py threshold --tag oneshot-body
    python tools/ab.py --env MXAR_PLANE_RESIDENT=0 protocol --tag launched
    PYTHONPATH=abtree/old python tools/ab.py ring --tag old      # an older build's package

experiments (every cell validated against an fp32 sum before it is timed):
  threshold  p50 device time of the threshold kernel next to the two-shot and the LL one-shot,
             P logical ranks in one launch (--ranks, --kib)
  protocol   the reference's round protocol: in-process PlaneJob rounds (40 B, 1 MiB) and the
             native deployment (mxar master + 2 mxar-gpu), us per round
  ring       8 logical ranks x 256 MiB: fp32-wire ring, element-type ring, two-shot, p50 and
             fraction of the same process's copy roofline
  sdma       the copy-engine allreduce at several reduce grids (--grids)
  sdma-remap the copy-engine allreduce before / after its input (x), output (y) or both
             were freed, the cache emptied and re-allocated at the same addresses, and with
             the input staged through a buffer allocated first (--mode x|y|both)
  grid       protocol rounds (2 workers, th = 1) at several per-worker workgroup budgets
  coll-grid  all-gather / reduce-scatter / all-to-all over device workgroup budgets

(Replaces thr_ab.py, proto_ab.py, resident_ab.py, ring_ab.py, sdma_ab.py, plane_grid_sweep.py
and coll_grid_sweep.py, whose records are cited in profiles/round4-5 - git history.)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(env: list[str]) -> None:
    for kv in env:  # before anything reads them (study knobs are read at construction)
        k, _, v = kv.partition("=")
        os.environ[k] = v
    if not os.environ.get("PYTHONPATH"):  # PYTHONPATH=<tree>: that tree's package
        sys.path.insert(0, _ROOT)
    sys.path.append(_ROOT)


def _emit(row: dict) -> None:
    print(json.dumps(row), flush=True)


def exp_threshold(a) -> None:
    import torch

    import akka_allreduce_1_amd
    from akka_allreduce_1_amd.ops import fill_uniform
    from akka_allreduce_1_amd.parallel import LocalCluster
    from akka_allreduce_1_amd.utils.timing import percentile
    from benchmarks.sections import device_times, rounding_check

    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16
    for P in [int(x) for x in a.ranks.split(",")]:
        sizes = [int(x) << 10 for x in a.kib.split(",")]
        cl = LocalCluster(P, slot_bytes=-(-max(sizes) // P) + (1 << 20), grid=512, timeout_s=10.0, max_lag=1)
        for size in sizes:
            n = size // 2
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=900 + k) for k in range(P)]
            ys = [torch.empty_like(t) for t in xs]
            ref = torch.zeros(n, device=dev)
            for t in xs:
                ref += t.float()
            row = {"exp": "threshold", "tag": a.tag, "P": P, "bytes": size,
                   "pkg": os.path.dirname(akka_allreduce_1_amd.__file__)}
            for algo in a.algos.split(","):
                if algo == "threshold":
                    fn = lambda: cl.allreduce_threshold(xs, ys, counts=False)  # noqa: E731
                else:
                    fn = lambda algo=algo: cl.allreduce(xs, ys, algo=algo)  # noqa: E731
                fn()
                cl.check()
                ok, err, _ = rounding_check(ys, ref, dtype, P)
                for _ in range(5):
                    fn()
                t = device_times(fn, a.iters, dev)
                cl.check()
                row[algo] = round(percentile(t, 50) * 1e3, 2) if ok else f"INVALID {err}"
            _emit(row)
        del cl
        torch.cuda.empty_cache()


def exp_protocol(a) -> None:
    import torch

    from benchmarks.sections import native_deployment, protocol_sizes

    dev = torch.device("cuda", 0)
    for rep in range(a.reps):
        p = protocol_sizes(dev, cases=((40, torch.float32, 2, 2000), (1 << 20, torch.bfloat16, 0, 2000)))
        import akka_allreduce_1_amd

        row = {"exp": "protocol", "tag": a.tag, "rep": rep, "pkg": os.path.dirname(akka_allreduce_1_amd.__file__),
               "inproc_us": {k: v.get("us_per_round") for k, v in p.items() if isinstance(v, dict) and "us_per_round" in v},
               "inproc_ok": all(v.get("validated") for v in p.values() if isinstance(v, dict) and "validated" in v)}
        if a.native:
            nat = native_deployment(cases=((10, 2, 400), (262144, 1024, 400)), budget_s=60.0)
            row["native_us"] = {k: v.get("us_per_round") for k, v in nat.items() if isinstance(v, dict) and "us_per_round" in v}
            row["native_ok"] = all(v.get("validated") for v in nat.values() if isinstance(v, dict) and "validated" in v)
        _emit(row)


def exp_ring(a) -> None:
    import torch

    from akka_allreduce_1_amd._native import C
    from akka_allreduce_1_amd.ops import fill_uniform
    from akka_allreduce_1_amd.parallel import LocalCluster
    from akka_allreduce_1_amd.utils.timing import hbm_bytes, percentile
    from benchmarks.sections import device_times

    dev = torch.device("cuda", 0)
    P, S = a.P, a.mib << 20
    n = S // 2
    st = torch.cuda.current_stream(dev).cuda_stream
    x = torch.empty(S, dtype=torch.uint8, device=dev)
    y = torch.empty_like(x)
    for _ in range(3):
        C.hip.copy(x.data_ptr(), y.data_ptr(), S, st)
    cms = percentile(device_times(lambda: C.hip.copy(x.data_ptr(), y.data_ptr(), S, st), a.iters, dev), 50)
    copy_tbps = 2 * S / (cms / 1e3) / 1e12
    del x, y
    cl = LocalCluster(P, slot_bytes=2 * -(-S // P) + (1 << 20), grid=512, timeout_s=10.0)
    xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=500 + k) for k in range(P)]
    ys = [torch.empty_like(t) for t in xs]
    ref = torch.zeros(n, device=dev)
    for t in xs:
        ref += t.float()
    row = {"exp": "ring", "tag": a.tag, "P": P, "mib": a.mib, "copy_TBps": round(copy_tbps, 3)}
    for algo in a.algos.split(","):
        fn = lambda algo=algo: cl.allreduce(xs, ys, algo=algo)  # noqa: E731
        fn()
        cl.check()
        err = max((t.float() - ref).abs().max().item() for t in ys)
        for _ in range(3):
            fn()
        p50 = percentile(device_times(fn, a.iters, dev), 50)
        cl.check()
        tb = hbm_bytes(S, P, algo, 2) / (p50 / 1e3) / 1e12
        row[algo] = [round(p50, 4), round(tb / copy_tbps, 3), round(err, 4)]
    _emit(row)


def exp_sdma(a) -> None:
    import torch

    from akka_allreduce_1_amd.ops import fill_uniform
    from akka_allreduce_1_amd.parallel import LocalSdmaCluster
    from akka_allreduce_1_amd.utils.timing import percentile
    from benchmarks.sections import device_times, rounding_check

    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16
    P, nbytes = a.P, a.mib << 20
    n = nbytes // 2
    xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=900 + k) for k in range(P)]
    ys = [torch.empty_like(x) for x in xs]
    ref = torch.zeros(n, device=dev)
    for x in xs:
        ref += x.float()
    for rep in range(a.reps):
        for g in [int(x) for x in a.grids.split(",")]:
            cl = LocalSdmaCluster(P, slot_bytes=-(-nbytes // P) + (1 << 20), grid=g, timeout_s=20.0)
            for k in [int(x) for x in a.pieces.split(",")]:
                for c in cl.comms:
                    c.pieces = k
                for y in ys:
                    y.fill_(float("nan"))
                cl.allreduce(xs, ys)
                torch.cuda.synchronize(dev)
                cl.check()
                ok, err, _ = rounding_check(ys, ref, dtype, P)
                p50 = percentile(device_times(lambda: cl.allreduce(xs, ys), a.iters, dev), 50)
                cl.check()
                _emit({"exp": "sdma", "tag": a.tag, "rep": rep, "P": P, "mib": a.mib, "grid": g, "pieces": k,
                       "engines": cl.comms[0].engines, "engines_per_peer": cl.comms[0].engines_per_peer,
                       "validated": ok, "max_abs_err": err, "p50_ms": round(p50, 4),
                       "algbw_GBps": round(nbytes / (p50 / 1e3) / 1e9, 1)})
            del cl
            torch.cuda.empty_cache()


def exp_sdma_remap(a) -> None:
    import torch

    from akka_allreduce_1_amd.ops import fill_uniform
    from akka_allreduce_1_amd.parallel import LocalSdmaCluster
    from akka_allreduce_1_amd.utils.timing import percentile
    from benchmarks.sections import device_times

    dev = torch.device("cuda", 0)
    P, nbytes = a.P, a.mib << 20
    n = nbytes // 2

    def bufs(seed):
        xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=seed + k) for k in range(P)]
        return xs, [torch.empty_like(x) for x in xs]

    cl = LocalSdmaCluster(P, slot_bytes=-(-nbytes // P) + (1 << 20), grid=128, timeout_s=20.0)
    stage = [torch.empty(n, dtype=torch.bfloat16, device=dev) for _ in range(P)]

    def t(fn, tag, xs):
        for _ in range(3):
            fn()
        ts = device_times(fn, a.iters, dev)
        cl.check()
        _emit({"exp": "sdma-remap", "tag": a.tag, "mode": a.mode, "P": P, "case": tag,
               "x": hex(xs[0].data_ptr()), "p50_ms": round(percentile(ts, 50), 4)})

    xs, ys = bufs(0)
    t(lambda: cl.allreduce(xs, ys), "first", xs)
    if a.mode in ("x", "both"):
        del xs
        torch.cuda.empty_cache()
        xs, _ = bufs(10)
    if a.mode in ("y", "both"):
        del ys
        torch.cuda.empty_cache()
        ys = [torch.empty_like(x) for x in xs]
    t(lambda: cl.allreduce(xs, ys), "remapped", xs)

    def staged():
        for s_, x in zip(stage, xs):
            s_.copy_(x)
        cl.allreduce(stage, ys)

    t(staged, "staged_input", xs)


def exp_grid(a) -> None:
    import torch

    from akka_allreduce_1_amd.engine import PlaneJob
    from akka_allreduce_1_amd.ops import fill_uniform

    dev = torch.device("cuda", 0)
    P = 2
    for nbytes, rounds in ((1 << 20, 1000), (16 << 20, 400), (64 << 20, 200), (256 << 20, 100)):
        n = nbytes // 2
        xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
        for grid in [int(x) for x in a.grids.split(",")]:
            block = -(-n // P)
            job = PlaneJob(P, n, max_chunk_size=max(1024, -(-block // 256)), dtype=torch.bfloat16, max_round=rounds - 1,
                           sources=xs, keep_outputs=False, keep_last=True, timeout_s=20.0, grid=grid)
            try:
                job.run(timeout=120)
                st = job.stamps
                per = (st[-1] - st[9]) / (len(st) - 10)
                _emit({"exp": "grid", "tag": a.tag, "bytes": nbytes, "grid_per_worker": grid,
                       "us_per_round": round(per * 1e6, 1)})
            finally:
                job.shutdown()


def exp_coll_grid(a) -> None:
    import torch

    from akka_allreduce_1_amd._native import C

    H = C.hip
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ops = {"all_to_all": H.Coll.AllToAll, "all_gather": H.Coll.AllGather, "reduce_scatter": H.Coll.ReduceScatter}
    for P in (8, 2):
        comms = [H.XgmiComm(k, P, 0, 16 << 20, 512, 10.0, 0) for k in range(P)]
        for c in comms:
            c.connect_local(comms)
        for blk in (128 << 10, 512 << 10, 2 << 20, 8 << 20):
            m = blk // 2
            for name, op in ops.items():
                ins = [torch.randn((1 if name == "all_gather" else P) * m, device=dev).to(torch.bfloat16) for _ in range(P)]
                outs = [torch.empty((1 if name == "reduce_scatter" else P) * m, dtype=torch.bfloat16, device=dev)
                        for _ in range(P)]
                for g in [int(x) for x in a.grids.split(",")]:
                    for c in comms:
                        c.grid = g
                    call = lambda: H.XgmiComm.collective_local(comms, op, [x.data_ptr() for x in ins],  # noqa: E731
                                                               [y.data_ptr() for y in outs], m, H.DType.BF16,
                                                               torch.cuda.current_stream().cuda_stream, 1.0)
                    for _ in range(3):
                        call()
                    ts = []
                    for _ in range(20):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        call()
                        e1.record()
                        e1.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    _emit({"exp": "coll-grid", "tag": a.tag, "P": P, "op": name, "block_bytes": blk, "grid": g,
                           "p50_us": round(statistics.median(ts), 2), "error": max(c.error() for c in comms)})
        del comms
        torch.cuda.synchronize()


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE set before anything is imported")
    sub = ap.add_subparsers(dest="exp", required=True)
    p = sub.add_parser("threshold")
    p.add_argument("--ranks", default="8,2")
    p.add_argument("--kib", default="4,64,1024")
    p.add_argument("--algos", default="ll,twoshot,threshold")
    p.add_argument("--iters", type=int, default=50)
    p = sub.add_parser("protocol")
    p.add_argument("--reps", type=int, default=1)
    p.add_argument("--native", type=int, default=1)
    p = sub.add_parser("ring")
    p.add_argument("--P", type=int, default=8)
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--algos", default="ring,ring_native,twoshot")
    p.add_argument("--iters", type=int, default=10)
    p = sub.add_parser("sdma")
    p.add_argument("--P", type=int, default=2)
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--grids", default="32,128,256,512")
    p.add_argument("--pieces", default="0", help="pipeline pieces per block (0 = by size)")
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--iters", type=int, default=10)
    p = sub.add_parser("sdma-remap")
    p.add_argument("--P", type=int, default=2)
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--mode", default="both", choices=["x", "y", "both"])
    p.add_argument("--iters", type=int, default=10)
    p = sub.add_parser("grid")
    p.add_argument("--grids", default="64,128,256")
    p = sub.add_parser("coll-grid")
    p.add_argument("--grids", default="64,128,256,512")
    for s in sub.choices.values():
        s.add_argument("--tag", default="")
    a = ap.parse_args()
    _setup(a.env)
    {"threshold": exp_threshold, "protocol": exp_protocol, "ring": exp_ring, "sdma": exp_sdma, "sdma-remap": exp_sdma_remap, "grid": exp_grid,
     "coll-grid": exp_coll_grid}[a.exp](a)


if __name__ == "__main__":
    main()
