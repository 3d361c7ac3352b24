"""bench.py output contract (the driver parses it): stdout is exactly one JSON line with the
metric / value / config fields, the engine validated, and the DP-step section (BASELINE
configs 4 / 5) present without errors."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_bench_prints_one_json_line_with_contract_fields(tmp_path):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    detail = tmp_path / "detail.json"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1", "--no-tune",
                        "--no-rccl", "--no-threshold", "--no-collectives", "--no-fused-step", "--dp-timeout", "90",
                        "--detail-out", str(detail)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[:2000]
    assert len(lines[0].encode()) < 4096  # the driver parses the last line; long lines are truncated
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["dtype"] == "bf16"
    assert d["engine_ok"] is True and d["validated_all"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in d["config"], k
    assert d["status"] == "ok" and d["config"]["algo"] == "copy (world=1)"
    assert d["detail"] == str(detail)
    for algo in ("twoshot", "ring", "ring_native"):  # [p50 ms, fraction of the copy roofline, ...]
        assert 0 < d["local_ranks"][algo][1] < 1.5, d["local_ranks"]
    assert d["protocol_us"]["validated"] is True, d["protocol_us"]

    full = json.loads(detail.read_text())  # everything else lives in the side file
    assert full["validated_max_abs_err"] == 0.0
    assert full["validated"] and all(full["validated"].values()), full.get("validation")
    assert full["topology"]["devices_visible"] >= 1
    loc = full["local_ranks"]
    assert "error" not in loc, loc
    for algo in ("twoshot", "ring", "ring_native"):
        assert loc[algo]["validated"] and 0 < loc[algo]["frac_copy_roofline"] < 1.5, loc
    proto = full["protocol"]  # the reference's master/worker protocol driving the GPU round engine
    assert "error" not in proto and proto["validated"] and proto["rounds_per_s"] > 0, proto
    for model in ("resnet50", "llama3_8b"):
        row = full["dp"][model]
        assert "error" not in row, row
        assert row["step_ms"] > 0 and row["compute_ms"] > 0
        # world = 1: no bandwidth figure for an allreduce that launches nothing
        assert "comm_algbw_per_rank" not in row and "note" in row
