"""Two-shot run-to-run modes: is the 8 x 256 MiB local two-shot's
~2.05 vs ~2.35 ms split the chip's clock, the memory side, or the code?

One process builds `--clusters` LocalClusters in turn (the bench's `local_ranks` geometry:
8 logical ranks in one launch, grid 512, slots of 2 blocks). For each cluster it times the
two-shot and the engine's copy kernel (event pairs, as bench.py does) while ONE probe wave
on a side stream samples s_memtime against the 100 MHz s_memrealtime (csrc/hip/kernels.hip
clock_probe_kernel), so every row carries the core clock the timed calls ran at. Run it
under `tools/gpu.sh pmc "GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" python
tools/twoshot_modes.py --no-probe` for the per-dispatch clock and L2-to-fabric requests.

    python tools/twoshot_modes.py [--clusters 4] [--iters 30] [--mib 256] [--P 8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402


def pct(v, q):
    s = sorted(v)
    return s[min(len(s) - 1, int(q / 100 * len(s)))]


class Probe:
    """One wave sampling (core cycles, 100 MHz ticks) every 0.1 ms on its own stream."""

    def __init__(self, dev, samples: int):
        self.dev, self.samples = dev, samples
        self.side = torch.cuda.Stream(device=dev)
        self.buf = torch.zeros(2 * samples, dtype=torch.int64, device=dev)

    def start(self):
        with torch.cuda.stream(self.side):
            self.buf.zero_()
        C.hip.clock_probe(self.buf.data_ptr(), self.samples, 10_000, self.side.cuda_stream)

    def mhz(self):
        torch.cuda.synchronize(self.dev)
        v = self.buf.view(self.samples, 2).cpu().double()
        ok = v[:, 1] > 0
        if ok.sum() < 3:
            return None
        c, r = v[ok, 0], v[ok, 1]
        return round(float((c[-1] - c[0]) / (r[-1] - r[0]) * 100.0), 1)


def times(fn, iters, dev, probe):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    torch.cuda.synchronize(dev)
    if probe:
        probe.start()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize(dev)
    ms = [a.elapsed_time(b) for a, b in ev]
    return ms, (probe.mhz() if probe else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=4)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--placement-tries", type=int, default=1,
                    help="LocalCluster placement_tries: slab placements timed at construction (fastest kept)")
    ap.add_argument("--staggers", default="0",
                    help="comma list of byte offsets: rank k's input / output start k x offset past a "
                         "multiple of the buffer size inside one allocation (each row tries every one)")
    ap.add_argument("--vary", choices=["both", "io", "slabs"], default="both",
                    help="what is allocated anew per row: everything, only the rank buffers (one "
                         "cluster kept), or only the cluster's slabs (one set of rank buffers kept)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    S, P = a.mib << 20, a.P
    n = S // 2
    st = torch.cuda.current_stream(dev).cuda_stream
    # the probe runs for the timed window only: ~2.5 ms per call
    probe = None if a.no_probe else Probe(dev, max(8, int(a.iters * 2.6 * 10)))
    cl = xs = ys = None
    for k in range(a.clusters):
        x = torch.empty(S, dtype=torch.uint8, device=dev)
        y = torch.empty_like(x)

        def cp():
            C.hip.copy(x.data_ptr(), y.data_ptr(), S, st)

        for _ in range(3):
            cp()
        cms, cmhz = times(cp, a.iters, dev, probe)
        del x, y
        if k == 0 or a.vary != "io":
            cl = LocalCluster(P, slot_bytes=2 * -(-S // P) + (1 << 20), grid=512, timeout_s=10.0,
                              placement_tries=a.placement_tries, placement_bytes=S)
        staggers = [int(v) for v in a.staggers.split(",")]
        for stg in staggers:
            if k == 0 or a.vary != "slabs" or len(staggers) > 1:
                # the previous row's buffers stay alive while these are taken: new pages, not reused ones
                if stg == 0:
                    xs2 = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=500 + j) for j in range(P)]
                    ys2 = [torch.empty_like(t) for t in xs2]
                else:  # one allocation per side, rank j at j x (S + stg) bytes (stg a multiple of 16)
                    bx = torch.empty(P * (S + stg), dtype=torch.uint8, device=dev)
                    by = torch.empty_like(bx)
                    xs2 = [fill_uniform(bx[j * (S + stg):j * (S + stg) + S].view(torch.bfloat16), seed=500 + j)
                           for j in range(P)]
                    ys2 = [by[j * (S + stg):j * (S + stg) + S].view(torch.bfloat16) for j in range(P)]
                keep = (xs, ys) if k else None  # noqa: F841 - held until the next row
                xs, ys = xs2, ys2

            def ts():
                cl.allreduce(xs, ys, algo="twoshot")

            for _ in range(3):
                ts()
            cl.check()
            tms, tmhz = times(ts, a.iters, dev, probe)
            cl.check()
            c50, t50 = pct(cms, 50), pct(tms, 50)
            copy_tbps = 2 * S / (c50 / 1e3) / 1e12
            # two-shot HBM bytes, utils.timing.hbm_bytes: P inputs read + P outputs written + slabs
            from akka_allreduce_1_amd.utils.timing import hbm_bytes
            tbps = hbm_bytes(S, P, "twoshot", 2) / (t50 / 1e3) / 1e12
            print(json.dumps({"row": k, "vary": a.vary, "stagger": stg,
                              "copy_ms": [round(pct(cms, 10), 4), round(c50, 4), round(pct(cms, 90), 4)],
                              "copy_TBps": round(copy_tbps, 3), "copy_core_MHz": cmhz,
                              "twoshot_ms": [round(pct(tms, 10), 4), round(t50, 4), round(pct(tms, 90), 4)],
                              "twoshot_TBps": round(tbps, 3), "frac_copy": round(tbps / copy_tbps, 3),
                              "twoshot_core_MHz": tmhz, "placement": cl.placement}), flush=True)
        if a.vary == "both":
            del cl, xs, ys
            cl = xs = ys = None
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
