#!/usr/bin/env python3
"""Randomised soak of the protocol round engine (PlaneJob: master + P plane workers on one GPU),
resident rounds included: every job draws P, size (both sides of the resident-round limit),
maxChunkSize, dtype, maxLag, round count and a source kind (per-round iota fill, a static
tensor, a slow source whose gaps make the resident kernel leave and come back), runs at
thresholds 1 and checks EVERY round's output of every worker against the exact sum. With
--threshold-frac a share of the jobs runs at thresholds < 1 with a straggler instead, each
chunk checked to be the sum of exactly `count` distinct workers (zeros at count 0). One JSON
line per job; the first failing job ends the soak (its line says why).

    python tools/plane_soak.py --seconds 240 --seed 1 > gpurun_out/plane_soak.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-jobs", type=int, default=10_000)
    ap.add_argument("--threshold-frac", type=float, default=0.0,
                    help="share of jobs at thresholds < 1 with a straggler (checked for consistency)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from akka_allreduce_1_amd.engine import PlaneJob, iota_source

    dev = torch.device("cuda", 0)
    rng = random.Random(args.seed)
    t_end = time.monotonic() + args.seconds
    totals = {"jobs": 0, "rounds": 0, "resident_rounds": 0, "resident_launches": 0}
    def subset_ok(v, lo, hi, it, cnt, P):
        """v[lo:hi] is the sum of `cnt` distinct workers' iota data of round `it`."""
        i = np.arange(lo, hi, dtype=np.float64)
        s_ = (v[lo:hi].astype(np.float64) - cnt * (i + it)) / 1000.0
        return bool(np.allclose(s_, s_[0], atol=1e-3)) and abs(s_[0] - round(s_[0])) <= 1e-3

    for j in range(args.max_jobs):
        if time.monotonic() > t_end:
            break
        if rng.random() < args.threshold_frac:
            # thresholds < 1 with a straggler: every chunk must be the sum of `count` distinct
            # workers (zeros at count 0) - the reference's partial rounds and catch-up
            P = rng.choice([3, 4])
            n = rng.choice([1000, 4096, 30000])
            chunk = rng.choice([64, 256, 1000])
            th = rng.choice([0.5, 2.0 / 3.0, 0.75])
            lag = rng.choice([1, 2])
            rounds = rng.randint(10, 40)
            slow_k, delay = rng.randrange(P), rng.uniform(0.001, 0.005)
            row = {"job": j, "P": P, "n": n, "chunk": chunk, "dtype": "float32", "max_lag": lag, "rounds": rounds,
                   "source": f"straggler {slow_k}", "th": round(th, 3), "resident_eligible": n * 4 <= 4 << 20}

            def src(k):
                base = iota_source(n, dev, torch.float32, 1000.0 * k)
                if k != slow_k:
                    return base

                def f(req):
                    time.sleep(delay)
                    return base(req)
                return f
            job = None
            t0 = time.perf_counter()
            try:
                job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=th, th_complete=th, max_lag=lag,
                               max_round=rounds - 1, timeout_s=20.0, sources=[src(k) for k in range(P)])
                job.run(timeout=120)
                step = -(-n // P)
                nch = -(-step // chunk)
                bad = None
                for k in range(P):
                    for it, (data, counts) in job.outputs[k].items():
                        v = data.float().cpu().numpy()
                        for jb in range(P):
                            for c in range(nch):
                                lo, hi = jb * step + c * chunk, min(n, jb * step + min(step, (c + 1) * chunk))
                                if lo >= hi:
                                    continue
                                cnt = counts[jb * nch + c]
                                ok = (0 <= cnt <= P) and ((cnt == 0 and not np.any(v[lo:hi])) or
                                                          (cnt > 0 and subset_ok(v, lo, hi, it, cnt, P)))
                                if not ok and bad is None:
                                    bad = {"worker": k, "round": it, "block": jb, "chunk": c, "count": cnt}
                errs = sum(job.system.plane_worker_state(w)["stats"]["plane_errors"] for w in job.workers)
                res = [(p.stats.resident_rounds, p.stats.resident_launches) for p in job.planes]
                row.update(ok=bad is None and errs == 0, plane_errors=errs, first_bad=bad,
                           resident_rounds=sum(r[0] for r in res), resident_launches=sum(r[1] for r in res),
                           wall_s=round(time.perf_counter() - t0, 3))
                totals["jobs"] += 1
                totals["rounds"] += sum(len(job.outputs[k]) for k in range(P))
                totals["resident_rounds"] += row["resident_rounds"]
                totals["resident_launches"] += row["resident_launches"]
                totals["threshold_jobs"] = totals.get("threshold_jobs", 0) + 1
            except Exception as e:  # noqa: BLE001
                row.update(ok=False, error=repr(e)[:600])
            finally:
                if job is not None:
                    job.shutdown()
            print(json.dumps(row), flush=True)
            job = None
            if not row.get("ok"):
                break
            continue
        P = rng.choice([2, 2, 3, 4])
        n = rng.choice([10, 37, 1000, 4096, 16384, 30000, 100_000, 300_000])
        chunk = max(1, rng.choice([2, 64, 512, 1024, 4096, n]))
        dtype = rng.choice([torch.float32, torch.float32, torch.bfloat16])
        lag = rng.choice([0, 1, 2])
        rounds = rng.randint(5, 60)
        kind = rng.choice(["iota", "iota", "static", "slow"])
        es = 4 if dtype == torch.float32 else 2
        cfg = {"job": j, "P": P, "n": n, "chunk": chunk, "dtype": str(dtype).replace("torch.", ""), "max_lag": lag,
               "rounds": rounds, "source": kind, "resident_eligible": n * es <= 4 << 20}
        if kind == "static":
            stat = [(torch.arange(n, dtype=torch.float64) + 1000.0 * k).to(dtype).to(dev) for k in range(P)]
            sources = stat
        elif kind == "slow":
            def slow(k, d=rng.uniform(0.0005, 0.003)):
                base = iota_source(n, dev, dtype, 1000.0 * k)

                def f(req):
                    time.sleep(d)
                    return base(req)
                return f
            sources = [slow(k) for k in range(P)]
        else:
            sources = [iota_source(n, dev, dtype, 1000.0 * k) for k in range(P)]
        row = dict(cfg)
        job = None
        t0 = time.perf_counter()
        try:
            job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=lag, max_round=rounds - 1, dtype=dtype, timeout_s=20.0,
                           sources=sources)
            job.run(timeout=120)
            ar = torch.arange(n, dtype=torch.float64)
            bad = None
            for it in range(rounds):
                if kind == "static":
                    parts = [(ar + 1000.0 * k).to(dtype).double() for k in range(P)]
                else:
                    parts = [(ar + it + 1000.0 * k).to(dtype).double() for k in range(P)]
                ref = sum(parts).numpy()
                for k in range(P):
                    data, counts = job.outputs[k][it]
                    got = data.double().cpu().numpy()
                    tol = 0.0 if dtype == torch.float32 else 2.0 ** -8
                    if not np.all(np.abs(got - ref) <= np.abs(ref) * tol) or any(c != P for c in counts):
                        bad = {"worker": k, "round": it, "max_err": float(np.max(np.abs(got - ref))),
                               "counts_ok": all(c == P for c in counts)}
                        break
                if bad:
                    break
            # plain ints: a stats object keeps its plane (and the plane's hardware queue) alive
            res = [(p.stats.resident_rounds, p.stats.resident_launches, p.stats.resident_parks) for p in job.planes]
            errs = sum(job.system.plane_worker_state(w)["stats"]["plane_errors"] for w in job.workers)
            row.update(ok=bad is None and errs == 0, plane_errors=errs, first_bad=bad,
                       resident_rounds=sum(r[0] for r in res), resident_launches=sum(r[1] for r in res),
                       resident_parks=sum(r[2] for r in res), wall_s=round(time.perf_counter() - t0, 3))
            totals["jobs"] += 1
            totals["rounds"] += rounds * P
            totals["resident_rounds"] += row["resident_rounds"]
            totals["resident_launches"] += row["resident_launches"]
        except Exception as e:  # noqa: BLE001
            row.update(ok=False, error=repr(e)[:600])
        finally:
            if job is not None:
                job.shutdown()
        print(json.dumps(row), flush=True)
        if not row.get("ok"):
            break
        job = None
        sources = None
    print(json.dumps({"summary": totals, "seed": args.seed}), flush=True)


if __name__ == "__main__":
    main()
