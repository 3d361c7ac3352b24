"""The ONE result line of bench.py, kept small enough for the driver to parse.

bench.py collects a large result dict (every section, every size, every candidate). The
driver reads only the last stdout line and truncates long lines, so the full dict goes to a
side file (`detail`), and the line holds the headline fields plus compact summaries:

  sweep          N > 1: per size class [bytes, chosen xGMI kernel, its p50 us, RCCL p50 us]
  local_ranks    N = 1: 8 logical ranks in one launch, two-shot / ring / element-type-wire
                 ring [p50 ms, fraction of the same run's copy roofline, (ring) reduce-scatter
                 wire bytes per rank per hop]
  lat_vs_size    N = 1: per P and size [bytes, best kernel, best p50 us, threshold p50 us]
  reduce_kernel  BASELINE config 2: fraction of the copy roofline per slot count
  protocol_us    the reference's round protocol, us per round per size (in-process, native
                 deployment, control-bridge), plus whether the timed rounds were validated
  stragglers     straggler tolerance (benchmarks/stragglers.py compact): the reference's default
                 job us per round [in process, native]; per size and maxLag [no-straggler period
                 us, ratio with a 0.2 ms straggler, ratio at 2 ms, p99 us at 2 ms, straggler lag];
                 the waiting gate's ratio at 2 ms; the 2-process native shape; validated
  adamw          fused reduce-scatter + AdamW + all-gather: ms and HBM TB/s
  dp             BASELINE configs 4 / 5: [step ms, compute-only ms, exposed ms]
  sdma           N > 1: the copy-engine allreduce across the GPUs, validated in child processes
                 first [ok, p50 ms, algbw GB/s] (benchmarks/sdma_xdev.py)
  xgmi_links     N > 1: the bring-up pack (akka_allreduce_1_amd/utils/links.py) - single-peer
                 push GB/s [min, median, max], all-peer push GB/s per rank [min, max], fan-out
                 ratio (all-peer / single-peer, 7 links ideal = 7), one-way flag hand-off us
                 [bare min, bare max, fenced max], coarse-grained push and pull [single-peer
                 median, all-peer min] GB/s; never dropped before the headline sections

`line()` guarantees the encoded line stays under LINE_BUDGET bytes: if a summary section
still overflows (e.g. a future section grows), sections are dropped in a fixed order and
their names listed under `dropped` (they remain in the side file).
"""
from __future__ import annotations

import json

LINE_BUDGET = 4000  # bytes, newline excluded; the driver contract is "one JSON line"

HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "p50_ms",
                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "algbw_per_rank",
                 "algbw_sum_over_ranks", "busbw", "engine_ok", "status")

# least important first: dropped in this order if the line is still over budget
_DROP_ORDER = ("lat_vs_size", "collectives", "sweep", "dp_overlap", "sdma_local", "sdma", "protocol_us", "dp",
               "stragglers",
               "reduce_kernel", "validation_failed", "engine_note", "adamw", "local_ranks", "threshold", "rccl",
               "xgmi_links")

from akka_allreduce_1_amd.algos import LIBRARY_ALGOS, LOSSY_ALGOS  # noqa: E402,F401 - one definition


def headline_guard(chosen: str, requested: str, world: int) -> tuple[str, str | None]:
    """The kernel the headline times: an automatic choice that is a library path or rounds
    per hop becomes the two-shot (with a status note); an explicit --algo is kept."""
    base = chosen.split("@")[0].split("~")[0]
    if world > 1 and requested == "auto" and (base in LOSSY_ALGOS or base in LIBRARY_ALGOS):
        return "twoshot", f"{chosen} is not a once-rounded engine kernel; headline is the two-shot"
    return chosen, None


def _r(x, nd=3):
    return None if x is None else round(float(x), nd)


def _sweep(rows: list) -> list:
    out = []
    for row in rows or []:
        ch = row.get("choice")
        out.append([row.get("bytes"), ch, row.get(f"{ch}_p50_us"), row.get("rccl_p50_us")])
    return out


def _local(lr: dict) -> dict:
    out = {"copy_TBps": lr.get("copy_roofline_TBps")}
    pl = lr.get("placement")
    if isinstance(pl, dict) and pl.get("frac_copy_roofline"):  # slab placements tried, their fractions
        out["placement"] = pl["frac_copy_roofline"]
    for algo in ("twoshot", "ring", "ring_native"):
        c = lr.get(algo)
        if isinstance(c, dict) and "p50_ms" in c:
            out[algo] = [c["p50_ms"], c.get("frac_copy_roofline")] + ([] if c.get("validated", True) else ["INVALID"])
            if "wire_bytes_per_hop" in c:  # reduce-scatter hop bytes per rank (all-gather: the block)
                out[algo].append(c["wire_bytes_per_hop"][0])
    if "error" in lr:
        out["error"] = str(lr["error"])[:160]
    return out


def _lat(lvs: dict) -> dict:
    out = {}
    for P in ("P8", "P4", "P2"):
        cells = lvs.get(P)
        if not isinstance(cells, list):
            continue
        rows = []
        for c in cells:
            best = c.get("best")
            th = c.get("threshold") or {}
            rows.append([c.get("bytes"), best, (c.get(best) or {}).get("p50_us"), th.get("p50_us")])
        out[P] = rows
        if lvs.get(f"{P}_all_validated") is False:
            out[f"{P}_INVALID"] = True
    return out


def _protocol(p: dict) -> dict:
    out: dict = {}
    ok = [p.get("validated")]
    inproc = {}
    for k, v in (p.get("sizes") or {}).items():
        if isinstance(v, dict) and "us_per_round" in v:
            inproc[k] = v["us_per_round"]
            ok.append(v.get("validated"))
    if "ms_per_round" in p:
        inproc[f"{p.get('bytes_per_worker', 0)}B"] = _r(p["ms_per_round"] * 1e3, 1)
    if inproc:
        out["inproc"] = inproc
    nat = {}
    for k, v in (p.get("native") or {}).items():
        if isinstance(v, dict) and "us_per_round" in v:
            nat[k] = v["us_per_round"]
            ok.append(v.get("validated"))
    if nat:
        out["native"] = nat
    b = p.get("bridge") or {}
    if "ms_per_round" in b:
        out["bridge"] = {f"{p.get('bytes_per_worker', 0)}B": _r(b["ms_per_round"] * 1e3, 1)}
        ok.append(b.get("validated"))
    out["validated"] = all(x is True for x in ok if x is not None) and any(x is not None for x in ok)
    if "error" in p:
        out["error"] = str(p["error"])[:160]
    return out


def _dp(dp: dict) -> tuple[dict, dict]:
    out, ovl = {}, {}
    for m in ("resnet50", "llama3_8b"):
        r = dp.get(m)
        if isinstance(r, dict):
            if "step_ms" in r:
                out[m] = [r["step_ms"], r.get("compute_ms"), r.get("exposed_comm_ms")]
                if "step_ms_auto_schedule" in r:
                    out[m].append(r["step_ms_auto_schedule"])
                if "step_ms_sdma" in r:
                    out[m].append({"sdma": r["step_ms_sdma"]})
            elif "error" in r:
                out[m] = str(r["error"])[:120]
    o = dp.get("overlap_rehearsal") or {}
    for m in ("resnet50", "llama3_8b"):
        r = o.get(m)
        if isinstance(r, dict) and isinstance(r.get("best"), str) and isinstance(r.get(r["best"]), dict):
            b = r[r["best"]]
            ovl[m] = [r["best"], b.get("step_ms"), b.get("exposed_comm_ms"), b.get("gemm_slowdown")]
            if "overlap_vs_serial_tokens8192" in r or "overlap_vs_serial_tokens1024" in r:
                ovl[m + "_vs_serial"] = r.get("overlap_vs_serial_tokens8192") or r.get("overlap_vs_serial_tokens1024")
            cu = r.get("cu_slice")
            if isinstance(cu, dict) and "step_ms" in cu:
                ovl[m + "_cu"] = [cu.get("variant"), cu.get("step_ms"), cu.get("exposed_comm_ms"), cu.get("gemm_slowdown")]
            se = r.get("serial_grid512")
            if isinstance(se, dict) and "step_ms" in se:
                ovl[m + "_serial"] = [se.get("step_ms"), se.get("gemm_slowdown")]
    return out, ovl


def _links(x: dict) -> dict:
    if not isinstance(x, dict) or "error" in x:
        return {"error": str(x.get("error", x))[:160] if isinstance(x, dict) else "?"}
    lat = x.get("flag_us") or {}
    bare = [v for v in lat.get("bare") or [] if v is not None]
    fen = [v for v in lat.get("fenced") or [] if v is not None]
    allr = x.get("all_GBps") or []
    return {"single_GBps": x.get("single_GBps_min_med_max"),
            "all_GBps": [min(allr), max(allr)] if allr else None,
            "ratio": x.get("fanout_ratio"),
            "flag_us": [min(bare) if bare else None, max(bare) if bare else None, max(fen) if fen else None],
            # the coarse-grained push and the pull: [single median, all-peer min]
            **{k: [x[k]["single_GBps_min_med_max"][1], x[k]["all_GBps_min_max"][0]]
               for k in ("coarse", "pull") if isinstance(x.get(k), dict)}}


def compact(result: dict, detail_path: str | None = None) -> dict:
    """The short line: headline fields + compact summaries of every section."""
    out = {k: result[k] for k in HEADLINE_KEYS if k in result}
    v = result.get("validated")
    if isinstance(v, dict):
        out["validated_all"] = all(v.values())
        bad = [k for k, ok in v.items() if not ok]
        if bad:
            out["validation_failed"] = bad
    if "engine_note" in result:
        out["engine_note"] = str(result["engine_note"])[:200]
    if "rccl" in result:
        out["rccl"] = {"algbw": result["rccl"].get("algbw"), "p50_ms": result["rccl"].get("p50_ms")}
        out["speedup_vs_rccl"] = result.get("speedup_vs_rccl")
    if "xgmi_links" in result:
        out["xgmi_links"] = _links(result["xgmi_links"])
    if "xgmi_twoshot" in result:
        out["twoshot_algbw"] = result["xgmi_twoshot"].get("algbw")
    t = result.get("xgmi_threshold")
    if isinstance(t, dict):
        out["threshold"] = {"algbw": t.get("algbw"), "ms": t.get("ms_per_step")} if "algbw" in t else {
            "error": str(t.get("error"))[:120]}
    if isinstance(result.get("collectives"), dict):
        out["collectives"] = {k: [r.get("xgmi_ms"), r.get("rccl_ms"), r.get("speedup_vs_rccl")] if "xgmi_ms" in r
                              else str(r.get("error"))[:80] for k, r in result["collectives"].items()}
    a = result.get("fused_adamw_step")
    if isinstance(a, dict):
        out["adamw"] = {k: a[k] for k in ("fused_ms", "unfused_ms", "speedup", "hbm_TBps", "params") if k in a}
        if "error" in a:
            out["adamw"]["error"] = str(a["error"])[:120]
    if result.get("sweep"):
        out["sweep"] = _sweep(result["sweep"])
    if isinstance(result.get("local_ranks"), dict):
        out["local_ranks"] = _local(result["local_ranks"])
    if isinstance(result.get("latency_vs_size"), dict):
        out["lat_vs_size"] = _lat(result["latency_vs_size"])
    rk = result.get("reduce_kernel")
    if isinstance(rk, dict):
        out["reduce_kernel"] = {"copy_TBps": rk.get("copy_roofline_TBps"),
                                **{P: rk[P].get("frac_copy_roofline") for P in ("P2", "P4", "P8")
                                   if isinstance(rk.get(P), dict)}}
    x = result.get("sdma")
    if isinstance(x, dict) and "skipped" in x:
        out["sdma"] = {"skipped": str(x["skipped"])[:60]}
    elif isinstance(x, dict):  # N > 1: the copy-engine allreduce across the GPUs (child processes)
        out["sdma"] = {"ok": x.get("validated"), "ms": x.get("p50_ms"), "algbw": x.get("algbw")}
        if x.get("errors"):
            out["sdma"]["error"] = str(x["errors"][0])[:100]
    sd = result.get("sdma_local")
    if isinstance(sd, dict):  # copy-engine allreduce, [p50 ms, algbw GB/s] per logical rank count
        out["sdma_local"] = {P: ([sd[P].get("p50_ms"), sd[P].get("algbw_GBps")] if "p50_ms" in sd[P]
                                 else str(sd[P].get("error"))[:80])
                             for P in ("P2", "P8") if isinstance(sd.get(P), dict)}
    if isinstance(result.get("protocol"), dict):
        out["protocol_us"] = _protocol(result["protocol"])
    if isinstance(result.get("stragglers"), dict):
        from benchmarks.stragglers import compact as _strag

        sg = result["stragglers"]
        out["stragglers"] = _strag(sg) if "error" not in sg else {"error": str(sg["error"])[:160]}
    if isinstance(result.get("dp"), dict):
        dp, ovl = _dp(result["dp"])
        if dp:
            out["dp"] = dp
        if ovl:
            out["dp_overlap"] = ovl
        if "error" in result["dp"]:
            out["dp"] = {"error": str(result["dp"]["error"])[:120]}
    if detail_path:
        out["detail"] = detail_path
    return out


def line(result: dict, detail_path: str | None = None, budget: int = LINE_BUDGET) -> str:
    """json.dumps(compact(result)), guaranteed <= budget bytes (sections dropped in order)."""
    c = compact(result, detail_path)
    s = json.dumps(c, separators=(",", ":"))
    dropped = []
    for k in _DROP_ORDER:
        if len(s.encode()) <= budget:
            break
        if k in c:
            del c[k]
            dropped.append(k)
            c["dropped"] = dropped
            s = json.dumps(c, separators=(",", ":"))
    if len(s.encode()) > budget:  # headline alone can never be this large; belt and braces
        c = {k: c[k] for k in HEADLINE_KEYS if k in c}
        c["dropped"] = "all sections (see detail)"
        s = json.dumps(c, separators=(",", ":"))
    return s
