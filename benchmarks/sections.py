"""Side sections of the N = 1 bench line (bench.py) that put the headline metric's SIZE axis in
front of the driver: "allreduce algbw + p50 latency vs tensor size" (BASELINE.json).

At N = 1 the one-rank allreduce is a copy, so the allreduce kernels themselves are timed with
P logical ranks in ONE launch on the GPU (LocalCluster: every rank's traffic lands in the
same HBM, no xGMI):

  latency_vs_size  P = 8 and P = 2, 4 KiB .. 256 MiB per rank in x4 steps; every cell holds
                   p50 device latency and algbw of ll / oneshot / twoshot / ring / threshold
                   and of `auto` (plus the kernel auto resolves to), each cell validated
                   against an fp32 reference (rounded once: within 1 bf16 ulp) BEFORE it is
                   timed. `auto_vs_best` = auto's p50 / the best kernel's p50 per size.
  reduce_kernel    BASELINE config 2: the reduce_slots kernel over P = 2 / 4 / 8 slots of a
                   1 GiB fp32 buffer (the worker's `reduce`, AllreduceWorker.scala:240-251),
                   TB/s of HBM traffic and the fraction of the same-run copy roofline.
  dp_overlap       BASELINE config 5's overlap on one GPU with REAL communication: every
                   bucket goes through ONE rank of an 8-GPU two-shot run alone (peers' flags
                   pre-armed; the same per-GPU HBM bytes as a real rank) on the comm stream
                   while the synthetic backward's GEMMs run; serial vs overlapped vs CU
                   slices vs paced (small-grid) comm, the GEMMs' slowdown and the exposed time.
  protocol_sizes   the reference's master / worker round protocol driving the GPU round
                   engine (PlaneJob: StartAllreduce -> one threshold-kernel launch per worker)
                   at 40 B (the reference's default job: 10 floats, maxChunkSize 2 -
                   AllreduceMaster.scala:105-114), 1 MiB and 64 MiB per worker; 2000 / 2000 /
                   200 rounds, mean and median round interval.

Latency method: the host is put ahead of the GPU (a sleep kernel first), then every call is
bracketed by device events - so p50 is the device time of one call (kernel launch to kernel
end, as seen by the GPU's command processor), not the Python enqueue rate; the host-bound
rate of back-to-back calls is reported next to it (`wall_us`).
"""
from __future__ import annotations

import contextlib
import statistics
import sys
import time

import torch

from akka_allreduce_1_amd._native import C
from akka_allreduce_1_amd.ops import fill_uniform
from akka_allreduce_1_amd.utils.timing import percentile

_SLEEP_CYCLES_PER_MS: list[float] = []


def _sleep_cycles_per_ms(dev) -> float:
    """torch.cuda._sleep spins on the shader clock: calibrate cycles per ms once."""
    if not _SLEEP_CYCLES_PER_MS:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        a.record()
        torch.cuda._sleep(1_000_000)
        b.record()
        torch.cuda.synchronize(dev)
        _SLEEP_CYCLES_PER_MS.append(1_000_000 / max(a.elapsed_time(b), 1e-3))
    return _SLEEP_CYCLES_PER_MS[0]


def device_times(fn, iters: int, dev, lead_ms: float = 4.0) -> list[float]:
    """Per-call device time (ms) of `fn` with the host AHEAD of the GPU: a sleep kernel of
    `lead_ms` is queued first, so the calls behind it run back to back on the device and each
    event pair brackets exactly one call's device work."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    cyc = _sleep_cycles_per_ms(dev)
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(cyc * lead_ms))
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize(dev)
    return [a.elapsed_time(b) for a, b in ev]


def wall_per_call(fn, iters: int, dev) -> float:
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / iters


def _bf16_ulp(x: torch.Tensor) -> torch.Tensor:
    _, e = torch.frexp(x.abs().clamp_min(1e-30))
    return torch.ldexp(torch.ones_like(x), e - 8)


def rounding_check(ys, ref: torch.Tensor, dtype: torch.dtype, P: int) -> tuple[bool, float, float]:
    """(ok, max_abs_err, max_err_in_ulps): every output within ONE ulp of the fp32 reference
    (bf16: the fp32 sum rounded once; the ordering of fp32 additions may move a value across a
    rounding boundary, never further), plus an absolute slack for fp32 reassociation."""
    worst_abs, worst_ulp, ok = 0.0, 0.0, True
    slack = 4e-7 * P
    for y in ys:
        d = (y.float() - ref).abs()
        worst_abs = max(worst_abs, d.max().item())
        if dtype == torch.bfloat16:
            u = _bf16_ulp(ref)
            worst_ulp = max(worst_ulp, (d / (u + slack)).max().item())
            ok = ok and bool((d <= u + slack).all().item())
        else:
            ok = ok and bool((d <= 1e-6 * P * ref.abs().clamp_min(1.0)).all().item())
    return ok, worst_abs, worst_ulp


def _sizes(lo: int, hi: int) -> list[int]:
    out, s = [], lo
    while s <= hi:
        out.append(s)
        s *= 4
    return out


def latency_vs_size(dev, dtype: torch.dtype = torch.bfloat16, ranks=(8, 4, 2), min_bytes: int = 4 << 10,
                    max_bytes: int = 256 << 20, iters: int = 20, warmup: int = 3) -> dict:
    from akka_allreduce_1_amd.parallel import LocalCluster

    es = torch.empty(0, dtype=dtype).element_size()
    out: dict = {"dtype": str(dtype).replace("torch.", ""), "method": "p50 of per-call device time (host ahead "
                 "of the GPU), P logical ranks in one launch on one GPU; algbw = bytes per rank / p50",
                 "sizes": _sizes(min_bytes, max_bytes)}
    names = {0: "auto", 1: "twoshot", 2: "oneshot", 3: "ring", 4: "ll"}
    for P in ranks:
        rows = []
        cl = xs = ys = None
        try:
            slot = -(-max_bytes // P) + (1 << 20)
            cl = LocalCluster(P, slot_bytes=slot, grid=512, timeout_s=10.0, max_lag=1)
            n_max = max_bytes // es
            xs = [fill_uniform(torch.empty(n_max, dtype=dtype, device=dev), seed=900 + k) for k in range(P)]
            ys = [torch.empty_like(t) for t in xs]
            ll_max = cl.comms[0].ll_max_bytes
            for size in out["sizes"]:
                n = size // es
                xv = [t[:n] for t in xs]
                yv = [t[:n] for t in ys]
                ref = torch.zeros(n, device=dev)
                for t in xv:
                    ref += t.float()
                row: dict = {"bytes": size}
                algos = ["ll", "oneshot", "twoshot", "ring", "threshold", "auto"]
                for algo in algos:
                    if algo == "ll" and size > 4 * ll_max:
                        continue
                    if algo == "oneshot" and size > min(slot - (1 << 20), 64 << 20):
                        continue
                    if algo == "threshold":
                        def fn(xv=xv, yv=yv):
                            cl.allreduce_threshold(xv, yv, counts=False)
                    else:
                        def fn(xv=xv, yv=yv, algo=algo):
                            cl.allreduce(xv, yv, algo=algo)
                    cell: dict = {}
                    try:
                        for y in yv:
                            y.fill_(float("nan"))  # a kernel that writes nothing cannot pass
                        fn()
                        cl.check()
                        ok, err, ulps = rounding_check(yv, ref, dtype, P)
                        cell.update(validated=ok, max_abs_err=err, max_err_ulp=round(ulps, 3))
                        if not ok:
                            row[algo] = cell
                            continue
                        for _ in range(warmup):
                            fn()
                        t = device_times(fn, iters, dev)
                        p50 = percentile(t, 50)
                        cell.update(p50_us=round(p50 * 1e3, 2), algbw_GBps=round(size / (p50 / 1e3) / 1e9, 2),
                                    wall_us=round(wall_per_call(fn, iters, dev) * 1e6, 2))
                        cl.check()
                    except Exception as e:  # noqa: BLE001 - reported per cell
                        cell["error"] = repr(e)
                    row[algo] = cell
                code = _H_dtype(dtype)
                row["auto_picks"] = names[int(cl.comms[0].resolve(n, code, C.hip.Algo.Auto, P))]
                timed_ = {a: c["p50_us"] for a, c in row.items() if isinstance(c, dict) and "p50_us" in c
                          and a != "auto"}
                if timed_:
                    best = min(timed_, key=timed_.get)
                    row["best"] = best
                    if "p50_us" in row.get("auto", {}):
                        row["auto_vs_best"] = round(row["auto"]["p50_us"] / timed_[best], 3)
                rows.append(row)
                del ref
        except Exception as e:  # noqa: BLE001 - reported, never loses the headline
            out[f"P{P}_error"] = repr(e)
        finally:
            del cl, xs, ys
            torch.cuda.empty_cache()
        out[f"P{P}"] = rows
        ratios = [r["auto_vs_best"] for r in rows if "auto_vs_best" in r]
        if ratios:
            out[f"P{P}_auto_worst_vs_best"] = max(ratios)
        out[f"P{P}_all_validated"] = all(c.get("validated", False) for r in rows for c in r.values()
                                         if isinstance(c, dict))
    return out


def _H_dtype(dtype: torch.dtype):
    return {torch.float32: C.hip.DType.F32, torch.bfloat16: C.hip.DType.BF16, torch.float16: C.hip.DType.F16}[dtype]


def reduce_kernel(dev, mib: int = 1024, slots=(2, 4, 8), iters: int = 10) -> dict:
    """BASELINE config 2: in-place-style reduce of P fp32 slots of `mib` MiB each into an
    output (out = sum of slots, fp32), the reduce_slots HIP kernel (csrc/hip/kernels.hip)."""
    from akka_allreduce_1_amd.ops import reduce_slots

    nbytes = mib << 20
    n = nbytes // 4
    res: dict = {"bytes_per_slot": nbytes, "dtype": "fp32"}
    s = torch.cuda.current_stream(dev).cuda_stream
    try:
        a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        for _ in range(3):
            C.hip.copy(a.data_ptr(), b.data_ptr(), nbytes, s)
        tc = percentile(device_times(lambda: C.hip.copy(a.data_ptr(), b.data_ptr(), nbytes, s), iters, dev), 50)
        roof = 2 * nbytes / (tc / 1e3) / 1e12
        res["copy_roofline_TBps"] = round(roof, 3)
        del a, b
        for P in slots:
            row: dict = {}
            sl = out = ref = None
            try:
                sl = torch.empty(P, n, device=dev)
                for p in range(P):
                    fill_uniform(sl[p], seed=40 + p)
                out = torch.empty(n, device=dev)
                reduce_slots(sl, out=out)
                ref = sl[0].clone()
                for p in range(1, P):
                    ref += sl[p]
                err = (out - ref).abs().max().item()
                row["max_abs_err"] = err
                row["validated"] = err <= 1e-6 * P
                del ref
                ref = None
                for _ in range(3):
                    reduce_slots(sl, out=out)
                t = percentile(device_times(lambda: reduce_slots(sl, out=out), iters, dev), 50)
                tb = (P + 1) * nbytes / (t / 1e3) / 1e12
                row.update(ms=round(t, 4), hbm_TBps=round(tb, 3), frac_copy_roofline=round(tb / roof, 3),
                           algbw_GBps=round(nbytes / (t / 1e3) / 1e9, 1))
            except Exception as e:  # noqa: BLE001
                row["error"] = repr(e)
            finally:
                del sl, out, ref
                torch.cuda.empty_cache()
            res[f"P{P}"] = row
    except Exception as e:  # noqa: BLE001
        res["error"] = repr(e)
    return res


def protocol_sizes(dev, cases=((40, torch.float32, 2, 2000), (1 << 20, torch.bfloat16, 0, 2000),
                               (64 << 20, torch.bfloat16, 0, 200))) -> dict:
    """The master / worker protocol on the GPU round engine at several per-worker sizes, two
    workers sharing the GPU (th = 1, maxLag 1). chunk 0 = the bench geometry (about 256 reduce
    units per worker). ms_per_round from the master's native round-barrier stamps after 10
    warm-up rounds; validated = the last round's output equals the fp32-ordered sum."""
    from akka_allreduce_1_amd.engine import PlaneJob

    res: dict = {"workers": 2, "th_reduce": 1.0, "th_complete": 1.0, "max_lag": 1,
                 "note": "2 plane workers share one GPU; StartAllreduce -> one threshold-kernel launch per worker"}
    P = 2
    for nbytes, dtype, chunk, rounds in cases:
        es = torch.empty(0, dtype=dtype).element_size()
        n = max(1, nbytes // es)
        if chunk <= 0:
            block = -(-n // P)
            chunk = max(1024, -(-block // 256))
        row: dict = {"bytes": nbytes, "dtype": str(dtype).replace("torch.", ""), "max_chunk_size": chunk,
                     "rounds": rounds}
        job = None
        try:
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=70 + k) for k in range(P)]
            ref = (xs[0].float() + xs[1].float()).to(dtype)
            job = PlaneJob(P, n, max_chunk_size=chunk, dtype=dtype, max_round=rounds - 1, sources=xs,
                           keep_outputs=False, keep_last=True, timeout_s=20.0)
            job.run(timeout=120)
            st = job.stamps
            warm = 10
            if len(st) > warm + 1:
                per = (st[-1] - st[warm - 1]) / (len(st) - warm)
                row["ms_per_round"] = round(per * 1e3, 4)
                row["us_per_round"] = round(per * 1e6, 1)
                row["rounds_per_s"] = round(1.0 / per, 1)
                row["algbw_per_worker_GBps"] = round(nbytes / per / 1e9, 3)
                gaps = sorted(st[i + 1] - st[i] for i in range(warm - 1, len(st) - 1))
                row["round_interval_p50_us"] = round(gaps[len(gaps) // 2] * 1e6, 1)
                row["round_interval_p99_us"] = round(gaps[int(0.99 * (len(gaps) - 1))] * 1e6, 1)
            lat = job.system.plane_worker_state(job.workers[0])["round_latency"]
            row["worker_round_latency_p50_us"] = round(lat["p50_ms"] * 1e3, 1)
            o = job.last_output(0)
            row["validated"] = bool(o is not None and o.iteration == rounds - 1 and torch.equal(o.data, ref))
        except Exception as e:  # noqa: BLE001
            row["error"] = repr(e)
        finally:
            if job is not None:
                job.shutdown()
        res[f"{nbytes}B"] = row
    return res


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _native_job(n: int, chunk: int, rounds: int, quiet: bool, timeout: float = 60.0) -> tuple[dict | None, list[str]]:
    """One run of the reference's deployment shape: `mxar master` + 2 `mxar-gpu worker`
    processes on GPU 0 (static source data[i] = i, 256 workgroups each - separate kernels:
    profiles/round5/native_grid_ab.jsonl, 128 each is no faster - host threads polling
    through the round: --spin-us 500). Returns the master's steady-rate line and the workers'
    stdout lines."""
    import json as _json
    import os
    import subprocess

    import akka_allreduce_1_amd

    exe = os.path.dirname(os.path.abspath(akka_allreduce_1_amd.__file__))  # the imported package's executables
    port = _free_port()
    seeds = ["--seeds", f"mxar.tcp://ClusterSystem@127.0.0.1:{port}", "--loglevel", "ERROR"]
    wargs = [os.path.join(exe, "mxar-gpu"), "worker", "0", str(n), "--device", "0", "--max-peers", "2",
             "--plane-timeout", "20", "--grid", "256", "--source", "static"] + seeds + (["--quiet"] if quiet else [])
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    workers = [subprocess.Popen(wargs, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
               for _ in range(2)]
    master = None
    try:
        master = subprocess.run([os.path.join(exe, "mxar"), "master", str(port), "2", str(n), str(chunk),
                                 "--th-reduce", "1", "--th-complete", "1", "--max-lag", "1", "--max-round",
                                 str(rounds - 1), "--spin-us", "500"] + seeds + ["--quiet"],
                                capture_output=True, text=True, timeout=timeout, env=env)
        outs = [w.communicate(timeout=timeout)[0] for w in workers]
    finally:
        for w in workers:
            if w.poll() is None:
                w.kill()
                w.wait()
    line = next((ln for ln in master.stdout.splitlines() if "steady_rounds_per_s" in ln), None)
    return (_json.loads(line) if line else None), [ln for o in outs for ln in o.splitlines()]


def native_deployment(cases=((10, 2, 400), (262144, 1024, 400), (16777216, 32768, 400), (67108864, 131072, 200)),
                      budget_s: float = 90.0) -> dict:
    """The reference's deployment shape on the GPU round engine, Python-free: master + 2 worker
    PROCESSES sharing GPU 0, arenas IPC-mapped, control over TCP (mxar / mxar-gpu). Per size:
    a 3-round run printing every worker's output sum and head, checked against the exact f32
    sum 2 * float(i); then the timed run (mean round interval from the master's barrier
    stamps), whose own last round each worker checks the same way (`validated_timed`). (n, maxChunkSize) = (10, 2) is the reference's default job (AllreduceMaster.scala:
    111-114)."""
    import re

    import numpy as np

    res: dict = {"workers": 2, "dtype": "float32", "source": "static data[i] = i (mxar-gpu --source static)",
                 "host": "--spin-us 500", "grid_per_worker": 256}
    t_end = time.monotonic() + budget_s  # the whole section; a failed size ends it
    for n, chunk, rounds in cases:
        row: dict = {"n_f32": n, "bytes": 4 * n, "max_chunk_size": chunk, "rounds": rounds}
        left = t_end - time.monotonic()
        if left < 10:
            row["error"] = f"skipped: section budget {budget_s:g} s spent"
            res[f"{4 * n}B"] = row
            continue
        try:
            _, lines = _native_job(n, chunk, 3, quiet=False, timeout=min(30.0, left / 2))
            exp = float((np.arange(n, dtype=np.float32).astype(np.float64) * 2).sum())
            sums = [float(m.group(1)) for ln in lines if (m := re.search(r"round \d+ sum (\S+)", ln))]
            row["validated"] = len(sums) == 6 and all(x == exp for x in sums)
            if not row["validated"]:
                row["check"] = {"expected_sum": exp, "seen": sums[:6]}
            else:
                st, tl = _native_job(n, chunk, rounds, quiet=True, timeout=min(30.0, max(5.0, t_end - time.monotonic())))
                # the timed run itself: each worker keeps its newest output and checks its sum at exit
                last = [(int(m.group(1)), float(m.group(2))) for ln in tl
                        if (m := re.search(r"last round (\d+) sum (\S+)", ln))]
                row["validated_timed"] = len(last) == 2 and all(r == rounds - 1 and x == exp for r, x in last)
                row["validated"] = row["validated"] and row["validated_timed"]
                if not row["validated_timed"]:
                    row["check_timed"] = {"expected": [rounds - 1, exp], "seen": last}
                if st:
                    row["us_per_round"] = round(1e6 / st["steady_rounds_per_s"], 1)
                    row["round_interval_p50_us"] = st["round_interval_p50_us"]
                    row["round_interval_p99_us"] = st["round_interval_p99_us"]
        except Exception as e:  # noqa: BLE001
            row["error"] = repr(e)[:300]
            t_end = 0.0  # the shape does not run here (e.g. under a profiler): skip the rest
        res[f"{4 * n}B"] = row
    return res


def sdma_local(dev, dtype: torch.dtype = torch.bfloat16, nbytes: int = 256 << 20, ranks=(2, 8), iters: int = 10) -> dict:
    """The copy-engine allreduce (parallel/sdma.py) with P logical ranks on this GPU: p50 per
    call and algbw, validated against fp32 first. All transfers are same-device engine copies
    here (the engines' xGMI rate is unmeasured on one GPU)."""
    from akka_allreduce_1_amd.parallel import LocalSdmaCluster

    es = torch.empty(0, dtype=dtype).element_size()
    n = nbytes // es
    out: dict = {"bytes_per_rank": nbytes, "dtype": str(dtype).replace("torch.", "")}
    for P in ranks:
        row: dict = {}
        cl = xs = ys = None
        try:
            cl = LocalSdmaCluster(P, slot_bytes=-(-nbytes // P) + (1 << 20), grid=128, timeout_s=20.0)
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=900 + k) for k in range(P)]
            ys = [torch.empty_like(x) for x in xs]
            ref = torch.zeros(n, device=dev)
            for x in xs:
                ref += x.float()
            cl.allreduce(xs, ys)
            torch.cuda.synchronize(dev)
            cl.check()
            ok, err, _ = rounding_check(ys, ref, dtype, P)
            del ref
            row.update(validated=ok, max_abs_err=err, engines_per_peer=cl.comms[0].engines_per_peer,
                       engines_per_rank=cl.comms[0].engines)
            for _ in range(10):  # the engines' rate is bimodal run to run (profiles/round6 section 3): warm up
                cl.allreduce(xs, ys)
            ts = device_times(lambda: cl.allreduce(xs, ys), iters, dev)
            cl.check()
            p50 = percentile(ts, 50)
            row.update(p50_ms=round(p50, 4), min_ms=round(min(ts), 4), algbw_GBps=round(nbytes / (p50 / 1e3) / 1e9, 1))
        except Exception as e:  # noqa: BLE001
            row["error"] = repr(e)[:300]
        finally:
            del cl, xs, ys
            torch.cuda.empty_cache()
        out[f"P{P}"] = row
    return out


class SoloRehearsalComm:
    """ONE rank of an N-rank (default 8) direct two-shot, run alone on this GPU: the N - 1 peers
    are communicators whose slabs live here but which never launch, and this rank's slab has
    every flag a peer would write pre-armed (XgmiComm.arm_solo_rehearsal), so its kernel runs
    the real two-shot without waiting. It reads its input, pushes the N - 1 foreign blocks into
    the peers' S slots, reduces its own block from the input and its own S slots (the synthetic
    peers' contributions: zeros), pushes the sum into the peers' R slots and gathers its own R
    slots (never written: the other blocks of the output come back as zeros). Every byte lands in this GPU's HBM, and per bucket of S bytes it moves reads
    (1 + 2 (N - 1) / N) S and writes (1 + 2 (N - 1) / N) S: exactly the per-GPU HBM traffic of a
    real N-GPU two-shot, where the outgoing pushes land on the peers and the peers' pushes land
    here (`hbm_bytes`). What it cannot model is the xGMI time: the pushes run at HBM speed, so
    the small-grid variants of dp_overlap pace it towards the link-bound duration."""

    accepts_stream = True

    def __init__(self, buckets, world: int = 8, grid: int = 512):
        from akka_allreduce_1_amd._native import C

        self.H = C.hip
        big = max(b.nbytes for b in buckets)
        dev = torch.cuda.current_device()
        self.world = world
        slot = -(-big // world) + (1 << 20)
        self.comms = [self.H.XgmiComm(k, world, dev, slot, grid, 20.0, 0) for k in range(world)]
        for c in self.comms:
            c.connect_local(self.comms)
        self.comms[0].arm_solo_rehearsal()
        self.cl = self  # dp_overlap sets `cl.comms[*].grid`
        self.bytes_moved = 0

    @staticmethod
    def hbm_bytes(S: int, world: int = 8) -> int:
        """Per-GPU HBM bytes of one rank of a real `world`-GPU two-shot of S bytes: reads of
        the input, the S slots and the R slots; writes of the own output block, the peers'
        incoming S and R pushes and the gathered output."""
        return int(2 * (S + 2 * S * (world - 1) / world))

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum", algo: str = "auto", stream: int | None = None):
        from akka_allreduce_1_amd.parallel.comm import _dtype_code

        s = torch.cuda.current_stream(t.device).cuda_stream if stream is None else stream
        self.comms[0].allreduce(t.data_ptr(), t.data_ptr(), t.numel(), _dtype_code(t.dtype), s,
                                self.H.Algo.TwoShot, 1.0 / self.world if op == "avg" else 1.0)
        return t

    def check(self):
        torch.cuda.synchronize()
        e = self.comms[0].error()
        if e:
            raise RuntimeError(f"solo rehearsal: error word {e:#x}")


class PairRehearsalComm:
    """A 2-rank data-parallel communicator on ONE GPU for overlap rehearsals: every bucket
    allreduce runs the real 2-rank kernel (LocalCluster, both ranks in one launch) over the
    bucket and a synthetic peer gradient of the same size, on the stream the reducer passes.
    Both ranks' kernel traffic lands on this GPU, so it contends with compute at about twice
    one rank's HBM traffic of a real 2-GPU job (and none of it crosses xGMI): an upper bound
    on the CU / HBM contention a real rank sees."""

    accepts_stream = True
    world = 2

    def __init__(self, buckets, grid: int, algo: str = "twoshot"):
        from akka_allreduce_1_amd.parallel import LocalCluster

        big = max(b.nbytes for b in buckets)
        self.cl = LocalCluster(2, slot_bytes=-(-big // 2) + (1 << 20), grid=grid, timeout_s=20.0)
        self.algo = algo
        self.peer = {}
        for b in buckets:
            t = b.buffer
            self.peer[t.data_ptr()] = (fill_uniform(torch.empty_like(t), seed=3 + b.index), torch.empty_like(t))

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum", algo: str = "auto", stream: int | None = None):
        x1, y1 = self.peer[t.data_ptr()]
        self.cl.allreduce([t, x1], [t, y1], algo=self.algo if algo == "auto" else algo, op=op, stream=stream)
        return t

    def check(self):
        self.cl.check()


def dp_overlap(dev, models=("resnet50", "llama3_8b"), grids=(32, 64, 128, 256, 512), world: int = 8,
               link_GBps: float = 153.6) -> dict:
    """BASELINE config 5 (and 4) rehearsed on one GPU with a byte-faithful comm beside the
    GEMMs: every bucket allreduce is ONE rank of a `world`-GPU two-shot (SoloRehearsalComm),
    so the comm moves exactly one rank's per-GPU HBM bytes of the N = 8 job (reported as
    hbm_bytes_per_rank). Per variant: the step (backward + overlapped bucket allreduces + SGD
    update), the compute-only step, the backward's own time with the comm beside it vs without
    (gemm_slowdown) and the comm-only time. The comm pushes at HBM speed, not xGMI speed: the
    grid variants pace it (comm_GBps, against xgmi_floor_ms = the link-bound time of the same
    buckets at `link_GBps` per link and direction), serial runs every bucket after backward,
    and the cu / split variants confine the comm (and the backward) to CU slices."""
    from akka_allreduce_1_amd.models.grad_sets import gradient_shapes
    from akka_allreduce_1_amd.parallel import BucketedGradReducer
    from benchmarks.bench_dp import SyntheticBackward

    out: dict = {"method": f"one rank of a {world}-GPU two-shot per bucket, run alone (peers' flags pre-armed, "
                           "pushes into local peer slabs) on the reducer's comm stream; medians of interleaved steps",
                 "note": "per-GPU HBM bytes equal a real N-GPU rank's; the pushes run at HBM rather than xGMI speed "
                         "(grid variants pace them)"}
    for model in models:
        row: dict = {}
        params = bwd = reducer = comm = None
        try:
            shapes = gradient_shapes(model)
            params = [torch.nn.Parameter(torch.zeros(sh, dtype=torch.bfloat16, device=dev)) for _, sh in shapes]
            big = model == "llama3_8b"
            steps, warm = (5, 1) if big else (15, 3)
            kw = dict(bucket_bytes=1 << 30, first_bucket_bytes=64 << 20) if big else dict(bucket_bytes=25 << 20)
            reducer = BucketedGradReducer(params, _Placeholder(world), op="avg", **kw)
            reducer.remove_hooks()  # the synthetic backward calls the hook itself
            comm = SoloRehearsalComm(reducer.buckets, world, max(grids))
            reducer.comm = comm
            reducer._raw_ok = True
            sizes = [b.nbytes for b in reducer.buckets]
            row["hbm_bytes_per_rank"] = sum(SoloRehearsalComm.hbm_bytes(S, world) for S in sizes)
            row["xgmi_floor_ms"] = round(sum(2 * (S / world) / (link_GBps * 1e9) for S in sizes) * 1e3, 3)
            bwds = {1024: SyntheticBackward(params, 1024, torch.bfloat16, dev)}
            bwd = bwds[1024]
            grads = [q.grad for q in params]
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

            cstream = {"s": None}  # the masked compute stream of a CU-split variant

            def overlap():
                ctx = torch.cuda.stream(cstream["s"]) if cstream["s"] is not None else contextlib.nullcontext()
                with ctx:
                    ev[0].record()
                    bwd.run(reducer)
                    ev[1].record()
                    reducer.wait()
                    torch._foreach_add_(params, grads, alpha=-1e-3)
                if cstream["s"] is not None:
                    torch.cuda.current_stream(dev).wait_stream(cstream["s"])

            def compute():
                ev[0].record()
                bwd.run(None)
                ev[1].record()
                torch._foreach_add_(params, grads, alpha=-1e-3)

            def comm_only():
                for b in reducer.buckets:
                    comm.allreduce_(b.buffer, op="avg", stream=reducer._comm_raw)
                torch.cuda.current_stream(dev).wait_stream(reducer.stream)

            hi_stream, hi_raw = reducer.stream, reducer._comm_raw
            splits: dict = {}
            lo_stream = torch.cuda.Stream(device=dev, priority=0)
            variants = [(f"grid{g}", g, True, True, 1024) for g in grids]
            # every bucket after backward (no overlap), and the overlap on a normal-priority
            # comm stream (the GEMMs' dispatches are not pre-empted by the comm queue)
            variants += [("serial_grid512", 512, False, True, 1024), ("grid128_normal_prio", 128, True, False, 1024)]
            # CU-sliced comm streams (hipExtStreamCreateWithCUMask; ddp.py "cuN:" schedules): the
            # bucket kernels may use only N of the 256 CUs, two workgroups per CU of the slice
            variants += [("cu16_grid32", 32, True, True, 1024), ("cu32_grid64", 64, True, True, 1024),
                         ("cu64_grid128", 128, True, True, 1024)]
            # and the complete split: backward on every OTHER CU (ddp.compute_stream_excluding),
            # so no GEMM tile shares a CU with a spinning comm workgroup
            variants += [("split32_grid64", 64, True, True, 1024), ("split64_grid128", 128, True, True, 1024)]
            if big:
                # 1024 tokens make the weight-gradient GEMMs (K = tokens) nearly bandwidth bound,
                # so a bandwidth-bound allreduce beside them slows them; at a training-size
                # 8192 tokens per GPU they are compute bound, and a small comm grid stretches
                # the allreduces over the backward instead of contending at full bandwidth
                variants += [("tokens8192_grid256", 256, True, True, 8192), ("tokens8192_serial", 512, False, True, 8192),
                             ("tokens8192_grid32", 32, True, True, 8192), ("tokens8192_grid64", 64, True, True, 8192),
                             ("tokens8192_grid128", 128, True, True, 8192),
                             ("split16_tokens8192", 32, True, True, 8192), ("split32_tokens8192", 64, True, True, 8192),
                             ("split64_tokens8192", 128, True, True, 8192)]
            # ResNet-50's steps are ~2 ms: a clock or power excursion during one variant's
            # window moves its step AND compute medians (a 4.7 ms serial step beside 2.3 ms
            # ones, BENCH of round 6), so every variant runs twice and keeps the pass with the
            # lower compute median; Llama-3-8B's 30-160 ms steps average such excursions out
            passes = 1 if big else 2
            for name, grid, ov, hi, tokens in [v for v in variants for _ in range(passes)]:
                cell: dict = {"tokens": tokens}
                print(f"[dp_overlap] {model} {name}", file=sys.stderr, flush=True)  # progress (a long section)
                try:
                    if tokens not in bwds:
                        bwds[tokens] = SyntheticBackward(params, tokens, torch.bfloat16, dev)
                    bwd = bwds[tokens]
                    for c in comm.cl.comms:
                        c.grid = grid
                    reducer.overlap = ov
                    reducer.stream = hi_stream if hi else lo_stream
                    reducer._comm_raw = hi_raw if hi else lo_stream.cuda_stream
                    reducer._cus = 0
                    cstream["s"] = None
                    if name.startswith("cu") or name.startswith("split"):
                        ncu = int(name.split("_")[0].replace("split", "").replace("cu", ""))
                        reducer._cus = -1  # force the switch onto the masked stream
                        reducer._set_algo(f"cu{ncu}:auto")
                        cell["cus"] = reducer._cus
                        if name.startswith("split"):
                            if ncu not in splits:
                                from akka_allreduce_1_amd.parallel import compute_stream_excluding

                                splits[ncu] = compute_stream_excluding(dev, ncu)
                            cstream["s"] = splits[ncu]
                    with torch.no_grad():
                        for fn in (overlap, compute, comm_only):
                            for _ in range(warm):
                                fn()
                        per = {"step": [], "compute": [], "bwd_with_comm": [], "bwd_alone": []}
                        for _ in range(steps):  # interleaved: clock drift hits both alike
                            for key, fn, bkey in (("step", overlap, "bwd_with_comm"), ("compute", compute, "bwd_alone")):
                                torch.cuda.synchronize(dev)
                                t0 = time.perf_counter()
                                fn()
                                torch.cuda.synchronize(dev)
                                per[key].append((time.perf_counter() - t0) * 1e3)
                                per[bkey].append(ev[0].elapsed_time(ev[1]))
                        torch.cuda.synchronize(dev)
                        t0 = time.perf_counter()
                        for _ in range(steps):
                            comm_only()
                        torch.cuda.synchronize(dev)
                        comm_ms = (time.perf_counter() - t0) / steps * 1e3
                    comm.check()
                    med = {k: statistics.median(v) for k, v in per.items()}
                    exposed = med["step"] - med["compute"]
                    cell = {"tokens": tokens, "step_ms": round(med["step"], 3), "compute_ms": round(med["compute"], 3),
                            "exposed_comm_ms": round(exposed, 3), "comm_only_ms": round(comm_ms, 3),
                            "bwd_ms_with_comm": round(med["bwd_with_comm"], 3),
                            "bwd_ms_alone": round(med["bwd_alone"], 3),
                            "gemm_slowdown": round(med["bwd_with_comm"] / med["bwd_alone"], 3),
                            "hidden_frac": round(max(0.0, 1 - exposed / comm_ms), 3),
                            "comm_GBps": round(row["hbm_bytes_per_rank"] / (comm_ms * 1e6), 1)}
                except Exception as e:  # noqa: BLE001
                    cell["error"] = repr(e)
                prev = row.get(name)
                if prev is None or "step_ms" not in prev or ("step_ms" in cell and cell["compute_ms"] < prev["compute_ms"]):
                    row[name] = cell
            reducer.overlap, reducer.stream, reducer._comm_raw, reducer._cus = True, hi_stream, hi_raw, 0
            reducer.algo = "auto"
            cstream["s"] = None
            ok = {g: c for g, c in row.items() if isinstance(c, dict) and "step_ms" in c}
            if ok:
                row["best"] = min(ok, key=lambda g: ok[g]["step_ms"])
            cu = {g: c for g, c in ok.items() if g.startswith("cu") or g.startswith("split")}
            if cu:  # the CU-sliced candidate's best cell
                g = min(cu, key=lambda k: cu[k]["step_ms"])
                row["cu_slice"] = dict(cu[g], variant=g)
            ser = {g: c for g, c in ok.items() if "serial" in g}
            for tag, pre in (("tokens1024", "grid"), ("tokens8192", "tokens8192_grid")):
                s_ = [c for g, c in ser.items() if (c["tokens"] == 8192) == (tag == "tokens8192")]
                ov_ = {g: c for g, c in ok.items() if g.startswith(pre) or (g.startswith("split") and
                                                                            (c["tokens"] == 8192) == (tag == "tokens8192"))}
                if s_ and ov_:  # the best overlapped cell against serial, per token count
                    g = min(ov_, key=lambda k: ov_[k]["step_ms"])
                    row[f"overlap_vs_serial_{tag}"] = [g, round(ov_[g]["step_ms"] / s_[0]["step_ms"], 3)]
            row["buckets"] = f"{len(reducer.buckets)} ({'64 MiB first, 1 GiB after' if big else '25 MiB'})"
        except Exception as e:  # noqa: BLE001
            row["error"] = repr(e)
        finally:
            del params, bwd, reducer, comm
            bwds = None
            torch.cuda.empty_cache()
        out[model] = row
    return out


class _Placeholder:
    """Stands in for the communicator while the reducer lays out its buckets (the rehearsal
    communicator needs the bucket buffers to size its slabs)."""

    accepts_stream = True

    def __init__(self, world: int = 2):
        self.world = world
