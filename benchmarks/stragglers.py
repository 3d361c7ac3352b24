"""Straggler tolerance, timed: the reference's reason to exist.

The reference's thresholds let fast workers keep going while one is slow: a chunk is reduced
once thReduce of the contributions are in, a round completes once thComplete of the reduced
chunks are in (DataBuffer.scala:28-33,69-75), the master advances on thAllreduce of the
workers (AllreduceMaster.scala:58-67), and a worker more than maxLag rounds behind is
force-completed (AllreduceWorker.scala:91-102; AllreduceSpec.scala:535-584). This section
times that on the GPU round engine (PlaneWorkerActor + XgmiRoundPlane):

* `reference_default`: the reference's own default job - 2 workers, 10 floats, maxChunkSize
  2, thReduce 0.9, thComplete 0.8, thAllreduce 1, maxLag 1, 101 rounds
  (AllreduceMaster.scala:105-114) - in process and as the native deployment (mxar master +
  2 mxar-gpu processes). It runs the threshold kernel's general (non-FULL) body.
* `sweep`: P = 4 co-located workers (one group kernel), thReduce = thComplete = thAllreduce
  = 0.75, maxLag 1 and 2, one worker's dataSource delayed by 0 / 0.2 / 2 ms per round
  (native tensor source, csrc/hip/hip_bind.cc tensor_source(delay_us)), rounds of 40 B /
  1 MiB / 64 MiB per worker. Lag skip on: a fast round waits at most lag_wait_us at its lag
  gate for the straggler, then runs without it and forces it (xgmi_threshold.hip; sticky while
  it lags). One 2 ms case with the waiting gate shows what bounded buffers cost without it.
* `native`: the deployment shape, 2 worker processes (P = 2: thReduce 0.75 -> 1 of 2,
  thComplete and thAllreduce 0.5, so the fast worker can finish on its own block), one of
  them delayed.

Per case: the fast workers' round period (p50 / p99 / mean of the intervals between their
sink calls, native stamps) against the same case without a straggler, forced completions,
cold rounds and coalesced starts, the fast workers' mean per-chunk count, the straggler's lag
behind the fast workers (sampled), and `validated`: every worker's source holds a distinct
power of two, so each output chunk must hold ONE integer whose set bits are its contributors,
with popcount = the chunk's reported count (the last output of every worker is checked; the
GPU test tests/test_stragglers_gpu.py checks every round of one case).
"""
from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys
import time

import torch

from akka_allreduce_1_amd._native import C


def pow2_check(data: torch.Tensor, counts, P: int, n: int, chunk: int) -> bool:
    """One output against its counts, sources 2^k (see the module docstring)."""
    lay = C.BlockLayout(n, P, chunk)
    nch = len(counts) // P
    lens, cnts = [], []
    for j in range(P):
        for c in range(nch):
            lo = lay.start[j] + c * chunk
            hi = min(lay.end[j], lo + chunk)
            if lo < hi:
                lens.append(hi - lo)
                cnts.append(counts[j * nch + c])
    if sum(lens) != n:
        return False
    dev = data.device
    L = torch.tensor(lens, device=dev)
    v = data.float()
    first = torch.repeat_interleave(v[torch.cumsum(L, 0) - L], L)
    cnt = torch.repeat_interleave(torch.tensor(cnts, device=dev, dtype=torch.int32), L)
    if not (torch.equal(v, first) and bool((v >= 0).all()) and bool((v == v.floor()).all())
            and bool((v < float(1 << P)).all())):
        return False
    vi = v.to(torch.int32)
    pc = torch.zeros_like(vi)
    for b in range(P):
        pc += (vi >> b) & 1
    return bool(torch.equal(pc, cnt))


def _period(stamps: list, warm: int) -> list[float]:
    """Intervals (us) between consecutive sink calls after `warm` rounds."""
    t = sorted(s for r, s in stamps if r >= warm)
    return [(b - a) * 1e6 for a, b in zip(t, t[1:])]


def _q(xs: list[float], p: float) -> float | None:
    if not xs:
        return None
    s = sorted(xs)
    return round(s[min(len(s) - 1, int(p * (len(s) - 1) + 0.5))], 2)


def inproc_case(dev, P: int, nbytes: int, dtype, chunk: int, max_lag: int, delay_us: float, rounds: int,
                lag_wait_us: float | None = 0.0, th: float = 0.75, th_all: float = 0.75, slow: int = 1,
                check: bool = True) -> dict:
    """P co-located plane workers, worker `slow`'s dataSource delayed by delay_us per round."""
    from akka_allreduce_1_amd.engine import PlaneJob

    es = torch.empty(0, dtype=dtype).element_size()
    n = max(1, nbytes // es)
    bufs = [torch.full((n,), float(1 << k), dtype=dtype, device=dev) for k in range(P)]
    srcs = [C.hip.tensor_source(b, delay_us=delay_us if k == slow else 0.0) for k, b in enumerate(bufs)]
    torch.cuda.synchronize(dev)
    row: dict = {"delay_us": delay_us, "max_lag": max_lag, "rounds": rounds, "lag_wait_us": lag_wait_us}
    job = PlaneJob(P, n, max_chunk_size=chunk, th_allreduce=th_all, th_reduce=th, th_complete=th, max_lag=max_lag,
                   max_round=rounds - 1, dtype=dtype, sources=srcs, keep_outputs=False, keep_last=True, record=True,
                   timeout_s=8.0, lag_wait_us=lag_wait_us)
    fast = [k for k in range(P) if k != slow]
    strag = slow if 0 <= slow < P else None
    try:
        t0 = time.perf_counter()
        job.start()
        lags = []
        while not job.finished.wait(0.002):
            if time.perf_counter() - t0 > 120:
                raise TimeoutError(f"straggler case did not finish: {job.state()}")
            try:  # ints only: no lock on the actors' round path
                if strag is not None:
                    rs = [job.system.plane_worker_rounds(w) for w in job.workers]
                    lags.append(max(rs[k][0] for k in fast) - rs[strag][0])
            except Exception:  # noqa: BLE001 - a sample, not the result
                pass
        wall = time.perf_counter() - t0
        st = job.state()
        warm = max(10, rounds // 10)
        iv = [x for k in fast for x in _period(job.sink_stamps(k), warm)]
        # where the long fast periods are: (worker, round ending it, us) for the 4 longest
        # above 4 x the median (a stall's position says what it waited for)
        med = statistics.median(iv) if iv else 0.0
        longest = []
        for k in fast:
            st_k = sorted((r, t) for r, t in job.sink_stamps(k) if r >= warm)
            longest += [(k, b[0], round((b[1] - a[1]) * 1e6, 1)) for a, b in zip(st_k, st_k[1:])
                        if (b[1] - a[1]) * 1e6 > 4 * med]
        if longest:
            row["long_periods"] = sorted(longest, key=lambda x: -x[2])[:4]
        ws = st["workers"]
        cs = [job.count_stats(k) for k in fast]
        row.update({
            "fast_period_p10_us": _q(iv, 0.1), "fast_period_p50_us": _q(iv, 0.5), "fast_period_p90_us": _q(iv, 0.9),
            "fast_period_p99_us": _q(iv, 0.99),
            "fast_period_mean_us": round(statistics.fmean(iv), 2) if iv else None,
            "master_rounds": st["master"].get("round"), "wall_s": round(wall, 3),
            "fast_count_mean": round(sum(c["sum"] for c in cs) / max(1, sum(c["n"] for c in cs)), 4),
            "forced": sum(w["stats"]["forced_completions"] for w in ws),
            "plane_errors": [w["stats"]["plane_errors"] for w in ws],
        })
        if strag is not None:
            sw = ws[strag]["stats"]
            row.update({"straggler_forced": sw["forced_completions"], "straggler_cold": sw["cold_rounds"],
                        "straggler_coalesced": sw["starts_coalesced"], "straggler_completed": sw["rounds_completed"],
                        "straggler_lag_p50": _q(lags, 0.5), "straggler_lag_max": max(lags) if lags else None})
        ok = all(ws[k]["stats"]["plane_errors"] == 0 for k in fast)
        if check:
            for k in range(P):
                o = job.last_output(k)
                if o is None:
                    ok = ok and k == strag  # a straggler may not have finished a round at all
                    continue
                ok = ok and pow2_check(o.data, list(o.count), P, n, chunk)
        row["validated"] = bool(ok)
    except Exception as e:  # noqa: BLE001 - reported per case
        row["error"] = repr(e)[:300]
    finally:
        job.shutdown()
        del bufs, srcs
    print(f"[stragglers] P={P} {nbytes} B lag={max_lag} delay={delay_us:g} us: "
          f"{row.get('fast_period_mean_us')} us/round validated={row.get('validated')}", file=sys.stderr, flush=True)
    return row


def _geometry(nbytes: int, dtype, P: int) -> tuple[int, int]:
    """(elements, maxChunkSize): the protocol bench's geometry (~256 chunks per block), the
    reference's 2-float chunk at 40 B."""
    es = torch.empty(0, dtype=dtype).element_size()
    n = max(1, nbytes // es)
    if nbytes <= 64:
        return n, 2
    block = -(-n // P)
    return n, max(1024, -(-block // 256))


SIZES = ((40, torch.float32, 1500), (1 << 20, torch.bfloat16, 1200), (64 << 20, torch.bfloat16, 150))


def sweep(dev, P: int = 4, lags=(1, 2), delays=(0.0, 200.0, 2000.0), sizes=SIZES, budget_s: float = 60.0) -> dict:
    """The straggler sweep (module docstring). ratio = fast period (mean) / no-straggler period.
    Lag-skip policy: a peer still short of the lag gate after lag_wait_us is skipped (sticky
    while it lags). The no-straggler case waits up to 5 ms (momentary lateness is waited
    for); the straggler cases use lag_wait = 2 x that case's mean round period (>= 100 us)."""
    out: dict = {"workers": P, "th": 0.75, "th_allreduce": 0.75, "straggler": 1,
                 "lag_wait_us": "d0: 5000; stragglers: max(100, 2 x the d0 mean period)",
                 "sources": "worker k: 2^k everywhere (tensor sources; the straggler's delayed natively)"}
    t_end = time.monotonic() + budget_s
    for nbytes, dtype, rounds in sizes:
        _, chunk = _geometry(nbytes, dtype, P)
        key = f"{nbytes}B"
        cell: dict = {"dtype": str(dtype).replace("torch.", ""), "max_chunk_size": chunk}
        for lag in lags:
            base = None
            for d in delays:
                if time.monotonic() > t_end:
                    cell[f"lag{lag}_d{int(d)}"] = {"error": f"skipped: section budget {budget_s:g} s spent"}
                    continue
                wait = 5000.0 if d == 0.0 else max(100.0, 2.0 * (base or 50.0))
                r = inproc_case(dev, P, nbytes, dtype, chunk, lag, d, rounds, lag_wait_us=round(wait, 1))
                if d == 0.0:
                    base = r.get("fast_period_mean_us")
                elif base and r.get("fast_period_mean_us"):
                    r["ratio_vs_no_straggler"] = round(r["fast_period_mean_us"] / base, 3)
                cell[f"lag{lag}_d{int(d)}"] = r
        out[key] = cell
    # the waiting lag gate (lag_wait_us None: bounded buffers) with the 2 ms straggler, 1 MiB
    if time.monotonic() < t_end:
        nb, dt, rounds = sizes[min(1, len(sizes) - 1)]
        _, chunk = _geometry(nb, dt, P)
        r = inproc_case(dev, P, nb, dt, chunk, 1, delays[-1], max(60, rounds // 20), lag_wait_us=None)
        r["policy"] = "waiting lag gate (no skip): bounded buffers hold the fast workers within maxLag + 1 rounds"
        base = ((out.get(f"{nb}B") or {}).get("lag1_d0") or {}).get("fast_period_mean_us")
        if base and r.get("fast_period_mean_us"):
            r["ratio_vs_no_straggler"] = round(r["fast_period_mean_us"] / base, 3)
        r["bytes"] = nb
        out["waiting_gate"] = r
    return out


def reference_default_inproc(dev, rounds: int = 101) -> dict:
    """The reference's default job in process: timed with native sinks, then the same job with
    every round's output kept and checked."""
    P, n, chunk = 2, 10, 2
    r = inproc_case(dev, P, 4 * n, torch.float32, chunk, 1, 0.0, rounds, lag_wait_us=None, th=0.9, th_all=1.0,
                    slow=-1)
    # a second run keeping every output: all rounds checked
    from akka_allreduce_1_amd.engine import PlaneJob

    bufs = [torch.full((n,), float(1 << k), device=dev) for k in range(P)]
    job = PlaneJob(P, n, max_chunk_size=chunk, th_allreduce=1.0, th_reduce=0.9, th_complete=0.8, max_lag=1,
                   max_round=rounds - 1, sources=bufs, timeout_s=20.0)
    try:
        job.run(timeout=60)
        ok = all(len(job.outputs[k]) == rounds and all(pow2_check(d, c, P, n, chunk)
                                                       for d, c in job.outputs[k].values()) for k in range(P))
        cnt = [sum(c) / len(c) for k in range(P) for _, c in job.outputs[k].values()]
        r["all_rounds_validated"] = bool(ok)
        r["count_mean_all_rounds"] = round(statistics.fmean(cnt), 4) if cnt else None
    except Exception as e:  # noqa: BLE001
        r["all_rounds_error"] = repr(e)[:200]
    finally:
        job.shutdown()
    r.update({"workers": P, "n": n, "max_chunk_size": chunk, "th_reduce": 0.9, "th_complete": 0.8,
              "th_allreduce": 1.0})
    r["period_note"] = "fast_period_* = every worker's period (no straggler here)"
    return r


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def native_job(n: int, chunk: int, rounds: int, *, th_reduce: float, th_complete: float, th_all: float,
               max_lag: int = 1, delay_us: float = 0.0, lag_wait_us: float | None = 0.0, grid: int = 256,
               timeout: float = 60.0) -> dict:
    """mxar master + 2 mxar-gpu workers on GPU 0 (sources 1 and 2; the second delayed by
    delay_us per round): the master's round intervals and each worker's summary line."""
    import akka_allreduce_1_amd

    exe = os.path.dirname(os.path.abspath(akka_allreduce_1_amd.__file__))
    port = _free_port()
    seeds = ["--seeds", f"mxar.tcp://ClusterSystem@127.0.0.1:{port}", "--loglevel", "ERROR"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    workers = []
    for k in range(2):
        a = [os.path.join(exe, "mxar-gpu"), "worker", "0", str(n), "--device", "0", "--max-peers", "2",
             "--plane-max-lag", str(max(1, max_lag)), "--plane-timeout", "20", "--grid", str(grid),
             "--source-value", str(float(1 << k)), "--check-chunk", str(chunk), "--quiet"] + seeds
        if k == 1 and delay_us > 0:
            a += ["--source-delay-us", str(delay_us)]
        if lag_wait_us is not None:
            a += ["--lag-wait-us", str(lag_wait_us)]
        workers.append(subprocess.Popen(a, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env))
        time.sleep(0.05)  # join order = worker id: the delayed one is id 1
    row: dict = {}
    try:
        m = subprocess.run([os.path.join(exe, "mxar"), "master", str(port), "2", str(n), str(chunk),
                            "--th-allreduce", str(th_all), "--th-reduce", str(th_reduce), "--th-complete",
                            str(th_complete), "--max-lag", str(max_lag), "--max-round", str(rounds - 1),
                            # both workers before the first init: below thAllreduce = 1 the
                            # reference starts with the first worker up and restarts the job at
                            # round 0 when the second joins (a lone-worker epoch, or a job that
                            # ends before the second worker ever joins)
                            "--init-workers", "2",
                            "--spin-us", "500"] + seeds + ["--quiet"],
                           capture_output=True, text=True, timeout=timeout, env=env)
        outs = []
        for k, w in enumerate(workers):
            try:
                outs.append(w.communicate(timeout=timeout)[0])
            except subprocess.TimeoutExpired:  # keep what it printed: the bench records why
                w.kill()
                tail = (w.communicate()[0] or "")[-600:]
                row["hung_worker"] = {"id": k, "output_tail": tail, "master_tail": (m.stdout or "")[-300:]}
                outs.append(tail)
    finally:
        for w in workers:
            if w.poll() is None:
                w.kill()
                w.wait()
    line = next((ln for ln in m.stdout.splitlines() if "steady_rounds_per_s" in ln), None)
    if line:
        s = json.loads(line)
        row["master_us_per_round"] = round(1e6 / s["steady_rounds_per_s"], 2)
        row["master_interval_p50_us"] = s["round_interval_p50_us"]
        row["master_interval_p99_us"] = s["round_interval_p99_us"]
    sums = []
    for o in outs:
        ln = next((x for x in o.splitlines() if x.startswith('{"worker_summary"')), None)
        sums.append(json.loads(ln)["worker_summary"] if ln else {"error": o[-300:]})
    row["workers"] = sums
    return row


def native_cases(delays=(0.0, 2000.0), sizes=((10, 2, 1500), (262144, 1024, 1200), (16777216, 32768, 200)),
                 budget_s: float = 60.0) -> dict:
    """The 2-process deployment with a straggler (module docstring): worker 0 fast, worker 1
    delayed; fp32 sources 1 / 2."""
    out: dict = {"workers": 2, "th_reduce": 0.75, "th_complete": 0.5, "th_allreduce": 0.5, "max_lag": 1,
                 "lag_wait_us": "d0: 5000; straggler: max(100, 2 x the d0 mean period)", "dtype": "float32"}
    t_end = time.monotonic() + budget_s
    for n, chunk, rounds in sizes:
        cell: dict = {"max_chunk_size": chunk}
        base = None
        for d in delays:
            if time.monotonic() > t_end:
                cell[f"d{int(d)}"] = {"error": "skipped: section budget spent"}
                continue
            try:
                wait = 5000.0 if d == 0.0 else max(100.0, 2.0 * (base or 50.0))
                r = native_job(n, chunk, rounds, th_reduce=0.75, th_complete=0.5, th_all=0.5, delay_us=d,
                               lag_wait_us=round(wait, 1), timeout=min(60.0, max(15.0, t_end - time.monotonic())))
                r["lag_wait_us"] = round(wait, 1)
                f = r["workers"][0] if r.get("workers") else {}
                r["fast_period_p50_us"] = f.get("period_p50_us")
                r["fast_period_mean_us"] = f.get("period_mean_us")
                r["validated"] = bool(r.get("workers")) and all(w.get("validated") is True and not w.get("plane_errors")
                                                                 for w in r["workers"][:1]) and \
                    all(w.get("validated") in (True, None) for w in r["workers"])
                if d == 0.0:
                    base = r["fast_period_mean_us"]
                elif base and r.get("fast_period_mean_us"):
                    r["ratio_vs_no_straggler"] = round(r["fast_period_mean_us"] / base, 3)
            except Exception as e:  # noqa: BLE001
                r = {"error": repr(e)[:300]}
            cell[f"d{int(d)}"] = r
        out[f"{4 * n}B"] = cell
    return out


def reference_default_native(rounds: int = 101) -> dict:
    """The reference's default job as its deployment: master + 2 worker processes."""
    try:
        r = native_job(10, 2, rounds, th_reduce=0.9, th_complete=0.8, th_all=1.0, lag_wait_us=None)
        r["validated"] = bool(r.get("workers")) and all(w.get("validated") is True and not w.get("plane_errors")
                                                         for w in r["workers"])
        return r
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)[:300]}


def section(dev, budget_s: float = 100.0) -> dict:
    """The bench section (bench.py `stragglers`)."""
    t0 = time.monotonic()
    out: dict = {}
    out["reference_default"] = {"inproc": reference_default_inproc(dev), "native": reference_default_native()}
    out["sweep"] = sweep(dev, budget_s=max(20.0, 0.6 * budget_s - (time.monotonic() - t0)))
    out["native"] = native_cases(budget_s=max(10.0, budget_s - (time.monotonic() - t0)))
    out["seconds"] = round(time.monotonic() - t0, 1)
    return out


def compact(s: dict) -> dict:
    """The bench line's summary: per size, [no-straggler mean us, ratio at 0.2 ms, ratio at
    2 ms, p99 us at 2 ms, straggler lag max at 2 ms] per maxLag; the reference default job's us
    per round in process / native; whether every case validated."""
    ok = []
    out: dict = {}
    rd = s.get("reference_default") or {}
    ip, nt = rd.get("inproc") or {}, rd.get("native") or {}
    out["ref_default_us"] = [ip.get("fast_period_mean_us"), nt.get("master_us_per_round")]
    ok += [ip.get("validated"), ip.get("all_rounds_validated"), nt.get("validated")]
    sw = s.get("sweep") or {}
    for key, cell in sw.items():
        if not isinstance(cell, dict) or not key.endswith("B") or key == "waiting_gate":
            continue
        row = {}
        for lag in (1, 2):
            c0, c1, c2 = (cell.get(f"lag{lag}_d{d}") or {} for d in (0, 200, 2000))
            if not c0:
                continue
            row[f"l{lag}"] = [c0.get("fast_period_mean_us"), c1.get("ratio_vs_no_straggler"),
                              c2.get("ratio_vs_no_straggler"), c2.get("fast_period_p99_us"), c2.get("straggler_lag_max")]
            ok += [c.get("validated") for c in (c0, c1, c2) if c]
        out[key] = row
    wg = sw.get("waiting_gate") or {}
    if wg:
        out["wait_gate_2ms_ratio"] = wg.get("ratio_vs_no_straggler")
    nat = s.get("native") or {}
    nrow = {}
    for key, cell in nat.items():
        if isinstance(cell, dict) and key.endswith("B"):
            a, b = cell.get("d0") or {}, cell.get("d2000") or {}
            nrow[key] = [a.get("fast_period_mean_us"), b.get("ratio_vs_no_straggler")]
            ok += [a.get("validated"), b.get("validated")]
    if nrow:
        out["native2"] = nrow
    out["validated"] = all(x is True for x in ok if x is not None) and any(x is not None for x in ok)
    return out


if __name__ == "__main__":
    # the section on its own: python -m benchmarks.stragglers [--budget S] > full.json
    import argparse
    import json

    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=100.0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = section(dev, a.budget)
    print(json.dumps(s), flush=True)
    print(json.dumps({"compact": compact(s)}), flush=True)
