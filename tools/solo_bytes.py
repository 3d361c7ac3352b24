"""HBM bytes of the DP-overlap rehearsal's comm (benchmarks/sections.py SoloRehearsalComm: one
rank of an 8-GPU two-shot run alone on this GPU) against the per-GPU bytes of a real N = 8
rank. Prints one line per bucket size with the model bytes; run it under one PMC pass per
counter and summarise with tools/prof.py pmc --kernel twoshot --skip 2:

    tools/gpu.sh pmc FETCH_SIZE python tools/solo_bytes.py
    tools/gpu.sh pmc WRITE_SIZE python tools/solo_bytes.py

(FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; together they need 5 TCC counters, one
pass holds 4.)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from benchmarks.sections import SoloRehearsalComm  # noqa: E402


class _Bucket:
    def __init__(self, t):
        self.buffer, self.nbytes = t, t.numel() * t.element_size()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", default="64,256,1024")
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--grid", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for mib in (int(v) for v in a.mib.split(",")):
        t = torch.ones((mib << 20) // 2, dtype=torch.bfloat16, device=dev)
        comm = SoloRehearsalComm([_Bucket(t)], a.world, a.grid)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for i in range(a.calls):
            if i == 2:
                ev[0].record()
            comm.allreduce_(t, op="sum")
        ev[1].record()
        comm.check()
        ms = ev[0].elapsed_time(ev[1]) / max(1, a.calls - 2)
        S = mib << 20
        # the peers contribute zeros and never reduce: the own block (block 0) keeps the input,
        # the gathered blocks read the never-written R slots (zeros)
        blk = -(-(-(-t.numel() // a.world)) // 8) * 8
        ok = bool((t[:blk] == 1).all().item() and (t[blk:] == 0).all().item())
        print(json.dumps({"bucket_MiB": mib, "model_hbm_bytes": SoloRehearsalComm.hbm_bytes(S, a.world),
                          "model_KiB": SoloRehearsalComm.hbm_bytes(S, a.world) / 1024, "ms": round(ms, 4),
                          "GBps": round(SoloRehearsalComm.hbm_bytes(S, a.world) / ms / 1e6, 1), "sum_ok": ok}),
              flush=True)
        del comm, t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
