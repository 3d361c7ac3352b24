import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akka_allreduce_1_amd.ops import fill_uniform
from akka_allreduce_1_amd.parallel import LocalCluster
dev = torch.device("cuda", 0)
for fence in (3, 0):
  for P, n, algo, slot, grid in [(2, 1 << 20, "twoshot", 4 << 20, 32), (2, 1 << 18, "twoshot", 4 << 20, 32), (2, 1 << 20, "twoshot", 4 << 20, 8),
                        (2, 1 << 20, "oneshot", 8 << 20, 32), (2, 40000, "twoshot", 4 << 20, 32), (2, 20000, "twoshot", 4 << 20, 32)]:
    cl = LocalCluster(P, slot_bytes=slot, grid=grid)
    for c in cl.comms: c.fence = fence
    xs = [fill_uniform(torch.empty(n, device=dev), seed=k) for k in range(P)]
    ys = cl.allreduce(xs, algo=algo)
    cl.check()
    ref = xs[0] + xs[1]
    for k, y in enumerate(ys):
        bad = (y - ref).abs() > 1e-5
        nb = int(bad.sum())
        if nb:
            idx = bad.nonzero().flatten()
            d = idx[1:] - idx[:-1]
            runs = (d != 1).nonzero().flatten()
            starts = [int(idx[0])] + [int(idx[i + 1]) for i in runs[:8]]
            print(f"fence={fence} P={P} n={n} {algo} grid={grid} rank{k}: {nb} bad, first runs start {starts}; y==x_own? {bool(torch.allclose(y[idx], xs[k][idx]))} y==0? {bool((y[idx]==0).all())}")
        else:
            print(f"fence={fence} P={P} n={n} {algo} grid={grid} rank{k}: ok")
