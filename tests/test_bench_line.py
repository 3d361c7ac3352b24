"""The bench result line stays driver-parseable (<= 4 KB, one JSON object) at N = 1 and in the
N = 8 shape, and the headline never becomes a library (RCCL) number.

Fixture: tests/data/bench_full_n1_r03.json is the full round-3 N = 1 result dict from a real
MI355X run (32.7 KB on one line - the line the driver could not parse)."""
import copy
import json
from pathlib import Path

import pytest

from benchmarks.summary import LINE_BUDGET, LIBRARY_ALGOS, compact, line

DATA = Path(__file__).parent / "data" / "bench_full_n1_r03.json"


def _full_n1() -> dict:
    return json.loads(DATA.read_text())


def _n8_shape(base: dict) -> dict:
    """Every section an N = 8 run adds (sweep, collectives, rccl, threshold, dp with the
    schedule variants), with the widest values they can carry."""
    r = copy.deepcopy(base)
    r.update(n_gpus=8, value=540.14, algbw_per_rank=540.14, algbw_sum_over_ranks=4321.12, busbw=945.25)
    r["config"] = dict(r["config"], algo="twoshot@256~1", parallelism="dp8", global_batch=8)
    r["rccl"] = {"algbw": 401.23, "ms_per_step": 0.6691, "p50_ms": 0.6654, "note": "copy + in-place dist.all_reduce"}
    r["speedup_vs_rccl"] = 1.346
    r["xgmi_twoshot"] = {"algbw": 540.14, "ms_per_step": 0.4969}
    r["xgmi_threshold"] = {"algbw": 512.2, "ms_per_step": 0.5241, "max_abs_err": 0.0312, "th_reduce": 1.0,
                           "th_complete": 1.0, "max_lag": 1}
    r["collectives"] = {k: {"xgmi_ms": 0.2512, "xgmi_algbw": 1068.1, "rccl_ms": 0.3124, "rccl_algbw": 859.2,
                            "speedup_vs_rccl": 1.244} for k in ("all_to_all", "all_gather", "reduce_scatter")}
    sweep = []
    size = 4096
    labels = ["ll", "oneshot", "twoshot", "twoshot@128", "twoshot@256", "twoshot@full", "twoshot~1", "twoshot@128~1",
              "twoshot@256~1", "ring", "ring@128", "ring@256", "threshold", "rccl", "rsag"]
    while size <= 256 << 20:
        row = {"bytes": size}
        for a in labels:
            row[f"{a}_p50_us"] = 123456.78
            row[f"{a}_algbw"] = 1234.56
        row["choice"] = "twoshot@256~1"
        row["speedup_vs_rccl"] = 1.234
        sweep.append(row)
        size *= 4
    r["sweep"] = sweep
    for m in ("resnet50", "llama3_8b"):
        r["dp"][m].update(comm_only_ms=123.456, comm_algbw_per_rank=456.78, step_ms_twoshot_128wg=123.456,
                          step_ms_serial=123.456, step_ms_auto_schedule=123.456, auto_schedule=[True, "twoshot@128"],
                          auto_schedule_tuning_ms=[123.4, 123.4, 123.4])
    r["protocol"] = dict(r["protocol"], worker_ids=list(range(8)),
                         bridge={"driver": "x" * 80, "validated": True, "ms_per_round": 0.4326})
    r["sdma"] = {"validated": True, "cross_gpu": True, "p50_ms": 1.2345, "algbw": 217.45, "max_abs_err": 0.0312,
                 "errors": []}
    r["topology"] = {"devices_visible": 8, "ranks": 8, "peer_access": [[1] * 8] * 8,
                     "link_type": [["xgmi"] * 8] * 8, "hops": [[1] * 8] * 8}
    return r


@pytest.mark.parametrize("shape", ["n1", "n8"])
def test_line_under_budget_and_parses(shape):
    full = _full_n1()
    r = full if shape == "n1" else _n8_shape(full)
    assert len(json.dumps(r)) > 8 * LINE_BUDGET  # the dict really is the big one
    s = line(r, "gpurun_out/bench_detail_n1.json")
    assert len(s.encode()) <= LINE_BUDGET < 4096
    d = json.loads(s)
    # the driver's contract fields survive verbatim
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert d[k] == r[k], k
    assert d["detail"] == "gpurun_out/bench_detail_n1.json"
    assert "dropped" not in d, d.get("dropped")  # nothing had to be dropped at these shapes


def test_n1_summaries_carry_the_kernel_figures():
    d = json.loads(line(_full_n1()))
    assert d["local_ranks"]["twoshot"] == [2.0044, 0.972]
    assert d["local_ranks"]["ring"] == [4.4651, 0.563]
    p8 = {row[0]: row for row in d["lat_vs_size"]["P8"]}
    assert p8[4096][1] in ("ll", "auto") and p8[4096][2] < 10
    assert p8[4096][3] == pytest.approx(17.74)  # the straggler-tolerant kernel at 4 KiB
    assert set(d["reduce_kernel"]) >= {"P2", "P4", "P8", "copy_TBps"}
    pr = d["protocol_us"]
    assert pr["validated"] is True
    assert "40B" in pr["inproc"] and "268435456B" in pr["native"] and "268435456B" in pr["inproc"]
    assert d["adamw"]["fused_ms"] == pytest.approx(0.7577)
    assert len(d["dp"]["llama3_8b"]) >= 3


def test_n8_summaries():
    d = json.loads(line(_n8_shape(_full_n1())))
    assert len(d["sweep"]) == 9 and d["sweep"][0] == [4096, "twoshot@256~1", 123456.78, 123456.78]
    assert d["speedup_vs_rccl"] == 1.346 and d["rccl"]["algbw"] == 401.23
    # the headline is the nccl-tests algbw (S / t), the N-sum under its own key
    assert d["value"] == d["algbw_per_rank"] == 540.14 and d["algbw_sum_over_ranks"] == 4321.12
    assert set(d["collectives"]) == {"all_to_all", "all_gather", "reduce_scatter"}


def test_overflow_drops_sections_not_the_headline():
    r = _n8_shape(_full_n1())
    r["engine_note"] = "e" * 5000
    r["latency_vs_size"]["P8"] = r["latency_vs_size"]["P8"] * 30
    s = line(r)
    assert len(s.encode()) <= LINE_BUDGET
    d = json.loads(s)
    assert d["value"] == r["value"] and "lat_vs_size" in d["dropped"]


def test_validation_failures_are_visible():
    r = _full_n1()
    r["validated"] = dict(r["validated"], ring=False)
    d = compact(r)
    assert d["validated_all"] is False and d["validation_failed"] == ["ring"]


def test_tuner_table_never_yields_a_library_path():
    """A table where RCCL was fastest (hand-set, or from an older tuner) still dispatches the
    framework's kernels: _pick maps library entries to the built-in policy."""
    from akka_allreduce_1_amd.parallel.comm import XgmiCommunicator

    c = object.__new__(XgmiCommunicator)
    c.table = [(4096, "ll"), (1 << 20, "rccl"), (64 << 20, "rsag"), (256 << 20, "rccl")]
    assert c._pick(4096) == "ll"
    for nbytes in (8192, 1 << 20, 32 << 20, 256 << 20, 1 << 30):
        assert c._pick(nbytes).split("@")[0] not in LIBRARY_ALGOS
    c.table = [(256 << 20, "twoshot@256")]
    assert c._pick(1 << 30) == "twoshot@256"


def _links(P: int = 8) -> dict:
    """An N = 8 xgmi_links section (akka_allreduce_1_amd/utils/links.py) at its widest."""
    return {"bytes": 67108864, "reps": 5, "grid_per_peer": 64, "store": "st16_wt (two-shot scatter path)",
            "push_GBps": [[0.0 if k == r else 123.45 for k in range(P)] for r in range(P)],
            "all_GBps": [812.34] * P, "single_GBps_min_med_max": [101.23, 123.45, 131.11], "fanout_ratio": 6.58,
            "flag_us": {"bare": [None] + [1.234] * (P - 1), "fenced": [None] + [1.567] * (P - 1)},
            "coarse": {"single_GBps_min_med_max": [90.12, 111.11, 120.5], "all_GBps_min_max": [700.25, 760.5]},
            "pull": {"single_GBps_min_med_max": [60.12, 70.75, 80.5], "all_GBps_min_max": [400.25, 420.5]}}


def test_n8_line_carries_the_link_pack():
    r = _n8_shape(_full_n1())
    r["xgmi_links"] = _links()
    s = line(r, "gpurun_out/bench_detail_n8.json")
    assert len(s.encode()) <= LINE_BUDGET
    d = json.loads(s)
    assert "dropped" not in d
    assert d["xgmi_links"] == {"single_GBps": [101.23, 123.45, 131.11], "all_GBps": [812.34, 812.34],
                               "ratio": 6.58, "flag_us": [1.234, 1.234, 1.567], "coarse": [111.11, 700.25],
                               "pull": [70.75, 400.25]}
    assert d["config"]["algo"].split("@")[0].split("~")[0] not in ("ring_native", "rccl", "rsag")
    assert d["sdma"] == {"ok": True, "ms": 1.2345, "algbw": 217.45}


def test_skipped_sdma_section_says_why():
    """A share-device rehearsal past 6 ranks skips the SDMA child section (2 processes per rank on
    one GPU); the line carries the reason instead of an empty or failed result."""
    r = _n8_shape(_full_n1())
    r["sdma"] = {"skipped": "share-device rehearsal with more than 6 ranks (2 processes per rank on one GPU)"}
    d = json.loads(line(r))
    assert d["sdma"]["skipped"].startswith("share-device rehearsal")
    assert len(json.dumps(d)) <= LINE_BUDGET


def test_link_pack_outlives_every_other_section():
    r = _n8_shape(_full_n1())
    r["xgmi_links"] = _links()
    r["engine_note"] = "e" * 5000
    r["latency_vs_size"]["P8"] = r["latency_vs_size"]["P8"] * 60
    r["sweep"] = r["sweep"] * 10
    d = json.loads(line(r))
    assert "xgmi_links" in d and "lat_vs_size" in d["dropped"]


def test_headline_guard_keeps_lossy_and_library_paths_out():
    from akka_allreduce_1_amd.parallel import comm
    from benchmarks.summary import LOSSY_ALGOS, headline_guard

    assert comm.LOSSY_ALGOS is LOSSY_ALGOS and comm.LIBRARY_ALGOS is LIBRARY_ALGOS  # one definition
    for auto_pick in ("ring_native", "ring_native@128", "rccl", "rsag"):
        algo, note = headline_guard(auto_pick, "auto", 8)
        assert algo == "twoshot" and note
    for ok in ("twoshot@256~1", "ring", "oneshot", "ll", "auto"):
        assert headline_guard(ok, "auto", 8) == (ok, None)
    assert headline_guard("ring_native", "ring_native", 8) == ("ring_native", None)  # explicit --algo


def test_tuner_never_adopts_a_lossy_kernel(monkeypatch):
    """tune() times ring_native as a comparison column but, with exact_only (the default),
    keeps a once-rounded kernel as the choice even when ring_native is fastest."""
    import torch

    from akka_allreduce_1_amd.parallel.comm import XgmiCommunicator

    import torch.distributed as dist

    c = object.__new__(XgmiCommunicator)
    c.rank, c.world, c.device, c.slot_bytes, c.cpu_group, c.group = 0, 8, torch.device("cpu"), 64 << 20, None, None
    c._default_grid, c._default_sized, c._default_units = 512, True, 0

    class _C:
        ll_max_bytes = 512 << 10
        threshold_rows = 0

    c._c = _C()
    speed = {"twoshot": 2.0, "ring_native": 1.0, "oneshot": 3.0}
    cur = {}

    def fake_allreduce(a, b, algo="auto", **kw):
        cur["algo"] = algo

    class _Ev:
        def __init__(self, enable_timing=True):
            pass

        def record(self):
            self.algo = cur.get("algo")

        def elapsed_time(self, other):
            return speed.get(other.algo.split("@")[0], 9.0)

    c.allreduce = fake_allreduce
    c.check = lambda: None
    monkeypatch.setattr(torch.cuda, "Event", _Ev)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(dist, "all_reduce", lambda *a, **k: None)
    monkeypatch.setattr(dist, "broadcast_object_list", lambda *a, **k: None)
    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "gloo")
    import akka_allreduce_1_amd.ops as ops

    monkeypatch.setattr(ops, "fill_uniform", lambda t, seed=0: t)
    rows = c.tune(max_bytes=64 << 10, min_bytes=16 << 10, candidates=("twoshot", "ring_native"), iters=2)
    assert all(r["choice"] == "twoshot" for r in rows) and all("ring_native_p50_us" in r for r in rows)
    rows = c.tune(max_bytes=64 << 10, min_bytes=16 << 10, candidates=("twoshot", "ring_native"), iters=2,
                  exact_only=False)
    assert all(r["choice"] == "ring_native" for r in rows)
