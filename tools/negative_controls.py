#!/usr/bin/env python3
"""Negative controls of the slot-reuse / flag-ownership tests (tests/test_comm_gpu.py
test_multiprocess_slot_reuse_slow_reader): the same runs with a protection switched off
must FAIL, or the test is not testing it.

  ring_hop_rows  MXAR_RING_FLAGS=hop - the round-3 ring flag layout (row = hop index), whose
                 words had two writers (the ring's predecessor and another kernel's owner)
  no_guard       MXAR_SLOT_GUARD=0 - no entry guard: a fast rank's next launch may push into
                 slots a slow reader has not read yet
  late_forward   test_ring_flag_ownership_late_forward (rank 2's last ring forward held 3 ms,
                 rank 1's all_gather flag on the same word in the hop layout): protected and
                 with MXAR_RING_FLAGS=hop - the deterministic control of the flag ownership

Each case prints one JSON line {case, world, seq, failed_ranks, first_failure}; the
protected runs (no env) are printed too, as the positive side of the A/B.

    python tools/negative_controls.py > gpurun_out/negative_controls.jsonl
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    from tests.test_comm_gpu import _run_flag_owner, _run_slow_reader

    cases = [
        ("protected", {}, 3, 2, "ring"),
        ("ring_hop_rows", {"MXAR_RING_FLAGS": "hop", "MXAR_STUDY": "1"}, 3, 2, "ring"),
        ("protected", {}, 4, 3, "ring"),
        ("ring_hop_rows", {"MXAR_RING_FLAGS": "hop", "MXAR_STUDY": "1"}, 4, 3, "ring"),
        ("no_guard", {"MXAR_SLOT_GUARD": "0", "MXAR_STUDY": "1"}, 3, 2, "ring"),
    ]
    only = set(sys.argv[1:])
    for name, env in (("late_forward_protected", {}),
                      ("late_forward_ring_hop_rows", {"MXAR_RING_FLAGS": "hop", "MXAR_STUDY": "1"}),
                      ("late_forward_no_guard", {"MXAR_SLOT_GUARD": "0", "MXAR_STUDY": "1"}),
                      ("late_forward_hop_rows_no_guard", {"MXAR_RING_FLAGS": "hop", "MXAR_SLOT_GUARD": "0",
                                                          "MXAR_STUDY": "1"})):
        if only and name not in only:
            continue
        print(f"[negative_controls] {name} ...", file=sys.stderr, flush=True)
        bad = _run_flag_owner(env)
        print(json.dumps({"case": name, "env": env, "world": 3, "failed_ranks": len(bad),
                          "first_failure": bad[0][2][:300] if bad else None}), flush=True)
    for name, env, world, slow, seq in cases:
        if only and name not in only:
            continue
        print(f"[negative_controls] {name} world={world} ...", file=sys.stderr, flush=True)
        bad = _run_slow_reader(world, slow, seq, env)
        print(json.dumps({"case": name, "env": env, "world": world, "slow_rank": slow, "seq": seq,
                          "failed_ranks": len(bad), "first_failure": bad[0][2][:300] if bad else None}), flush=True)


if __name__ == "__main__":
    main()
