"""Ring-kernel probe: the latency table's exact sequence (P logical ranks, a threshold lag ring
in the slab, ll / oneshot / twoshot before the ring, views of larger buffers, NaN-filled
outputs), printing the max error vs fp32 and the first bad indices per rank."""
import sys
import torch
sys.path.insert(0, ".")
from akka_allreduce_1_amd.ops import fill_uniform
from akka_allreduce_1_amd.parallel import LocalCluster

dev = torch.device("cuda", 0)
MAX = int(sys.argv[1]) if len(sys.argv) > 1 else (256 << 20)
for P in (8, 4):
    for lag in (1, None):
        for pre in (("ll", "oneshot", "twoshot"), ("oneshot",), ()):
            slot = -(-MAX // P) + (1 << 20)
            cl = LocalCluster(P, slot_bytes=slot, grid=512, timeout_s=5.0, max_lag=lag)
            nmax = MAX // 2
            X = [fill_uniform(torch.empty(nmax, dtype=torch.bfloat16, device=dev), seed=900 + k) for k in range(P)]
            Y = [torch.empty_like(t) for t in X]
            for n in (2048, 1 << 20):
                xs = [t[:n] for t in X]
                ys = [t[:n] for t in Y]
                ref = sum(x.float() for x in xs)
                for a in pre:
                    cl.allreduce(xs, ys, algo=a)
                for y in ys:
                    y.fill_(float("nan"))
                cl.allreduce(xs, ys, algo="ring")
                cl.check()
                err = max((y.float() - ref).abs().max().item() for y in ys)
                bad = [(k, torch.nonzero(~((ys[k].float() - ref).abs() <= 0.1)).flatten()[:4].tolist()) for k in range(P)]
                print(P, lag, pre, n, "err", err, bad, flush=True)
            del cl, X, Y
            torch.cuda.empty_cache()
