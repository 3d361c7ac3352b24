#!/usr/bin/env python3
"""All-gather / reduce-scatter / all-to-all (csrc/hip/xgmi_coll.hip) with P logical ranks in
one launch on one GPU, swept over the device workgroup budget and the block size: p50 us per
call. One JSON line per (P, op, block bytes, grid).

    python tools/coll_grid_sweep.py > gpurun_out/coll_grid_sweep.jsonl
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_1_amd._native import C  # noqa: E402

H = C.hip


def main() -> None:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", type=int, nargs="+", default=[64, 128, 256, 512],
                    help="device workgroup budgets (512 = the default grid: launch-size grids apply)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ops = {"all_to_all": H.Coll.AllToAll, "all_gather": H.Coll.AllGather, "reduce_scatter": H.Coll.ReduceScatter}
    for P in (8, 2):
        slot = 16 << 20
        comms = [H.XgmiComm(k, P, 0, slot, 512, 10.0, 0) for k in range(P)]
        for c in comms:
            c.connect_local(comms)
        for blk in (128 << 10, 512 << 10, 2 << 20, 8 << 20):
            m = blk // 2
            for name, op in ops.items():
                in_blocks = 1 if name == "all_gather" else P
                out_blocks = 1 if name == "reduce_scatter" else P
                ins = [torch.randn(in_blocks * m, device=dev).to(torch.bfloat16) for _ in range(P)]
                outs = [torch.empty(out_blocks * m, dtype=torch.bfloat16, device=dev) for _ in range(P)]
                for g in args.grids:
                    for c in comms:
                        c.grid = g
                    call = lambda: H.XgmiComm.collective_local(comms, op, [x.data_ptr() for x in ins],  # noqa: E731
                                                               [y.data_ptr() for y in outs], m, H.DType.BF16,
                                                               torch.cuda.current_stream().cuda_stream, 1.0)
                    for _ in range(3):
                        call()
                    ts = []
                    for _ in range(20):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record()
                        call()
                        e1.record()
                        e1.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    errs = [c.error() for c in comms]
                    print(json.dumps({"P": P, "op": name, "block_bytes": blk, "grid": g,
                                      "p50_us": round(statistics.median(ts), 2), "error": max(errs)}), flush=True)
        del comms
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
