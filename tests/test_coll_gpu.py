"""xGMI all-to-all / all-gather / reduce-scatter (csrc/hip/xgmi_coll.hip) on one MI355X:
P logical ranks in one launch (LocalCluster) and 2 processes with IPC-mapped slabs.
Data movement is checked bit-exact; the reduce-scatter against an fp32 rank-order sum."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402

DEV = torch.device("cuda", 0)


def _inputs(P, n, dtype, seed):
    return [fill_uniform(torch.empty(n, dtype=dtype, device=DEV), seed=seed + k) for k in range(P)]


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m", [8, 4096, 300_000])
def test_all_to_all_all_gather_reduce_scatter(P, dtype, m):
    cl = LocalCluster(P, slot_bytes=256 << 10, grid=64, timeout_s=10.0)  # 300k elements -> several segments
    xs = _inputs(P, P * m, dtype, seed=17 * m + P)
    ys = cl.collective("all_to_all", xs)
    cl.check()
    for r in range(P):
        for s in range(P):
            assert torch.equal(ys[r][s * m:(s + 1) * m], xs[s][r * m:(r + 1) * m]), (r, s)
    gs = [x[:m].contiguous() for x in xs]
    ag = cl.collective("all_gather", gs)
    cl.check()
    full = torch.cat(gs)
    for r in range(P):
        assert torch.equal(ag[r], full), r
    rs = cl.collective("reduce_scatter", xs, scale=0.5)
    cl.check()
    for r in range(P):
        ref = torch.zeros(m, device=DEV)
        for s in range(P):
            ref += xs[s][r * m:(r + 1) * m].float()
        err = (rs[r].float() - 0.5 * ref).abs().max().item()
        assert err <= (1e-6 if dtype == torch.float32 else 1e-2 * P), (r, err)


def test_collectives_interleaved_with_allreduce():
    """Slots are reused across kernel types and epochs: every result stays exact."""
    P, m = 4, 65536
    cl = LocalCluster(P, slot_bytes=1 << 20, grid=64, timeout_s=10.0)
    for it in range(6):
        xs = _inputs(P, P * m, torch.float32, seed=100 * it)
        kind = ["all_to_all", "allreduce", "reduce_scatter", "all_gather", "allreduce", "all_to_all"][it]
        if kind == "allreduce":
            ys = cl.allreduce(xs, algo="twoshot" if it == 1 else "ll")
            ref = sum(x for x in xs)
            assert all((y - ref).abs().max().item() < 1e-5 for y in ys)
        elif kind == "all_gather":
            gs = [x[:m].contiguous() for x in xs]
            assert all(torch.equal(y, torch.cat(gs)) for y in cl.collective(kind, gs))
        elif kind == "reduce_scatter":
            ys = cl.collective(kind, xs)
            for r in range(P):
                ref = sum(x[r * m:(r + 1) * m] for x in xs)
                assert (ys[r] - ref).abs().max().item() < 1e-5
        else:
            ys = cl.collective(kind, xs)
            assert all(torch.equal(ys[r][s * m:(s + 1) * m], xs[s][r * m:(r + 1) * m]) for r in range(P) for s in range(P))
        cl.check()


def test_collective_rejects_overlap_and_unaligned_blocks():
    cl = LocalCluster(2, slot_bytes=1 << 20, grid=8)
    xs = [torch.zeros(2 * 1024, device=DEV) for _ in range(2)]
    with pytest.raises(Exception, match="overlap"):
        cl.collective("all_to_all", xs, xs)
    with pytest.raises(Exception, match="16 bytes"):
        cl.collective("all_to_all", [torch.zeros(2 * 3, device=DEV) for _ in range(2)])


def _mp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import XgmiCommunicator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, msg = True, ""
    try:
        comm = XgmiCommunicator(device=0, slot_bytes=1 << 20, grid=16, timeout_s=15.0)
        for dtype in (torch.float32, torch.bfloat16):
            m = 70_000  # > slot per block for fp32: two segments
            xs = [fill_uniform(torch.empty(world * m, dtype=dtype, device=DEV), seed=50 + k) for k in range(world)]
            y = comm.all_to_all(xs[rank])
            g = comm.all_gather(xs[rank][:m].contiguous())
            z = comm.reduce_scatter(xs[rank], op="avg")
            comm.check()
            for s in range(world):
                if not torch.equal(y[s * m:(s + 1) * m], xs[s][rank * m:(rank + 1) * m]):
                    ok, msg = False, f"{dtype} all_to_all block {s}"
                if not torch.equal(g[s * m:(s + 1) * m], xs[s][:m]):
                    ok, msg = False, f"{dtype} all_gather block {s}"
            ref = sum(x[rank * m:(rank + 1) * m].float() for x in xs) / world
            if (z.float() - ref).abs().max().item() > (1e-6 if dtype == torch.float32 else 1e-2):
                ok, msg = False, f"{dtype} reduce_scatter"
    except Exception as e:  # noqa: BLE001
        ok, msg = False, repr(e)
    q.put((rank, ok, msg))
    dist.destroy_process_group()


def test_collectives_two_processes_ipc():
    from akka_allreduce_1_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_mp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad


def _hier_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import HierarchicalCommunicator, XgmiCommunicator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, msg = True, ""
    try:
        h = HierarchicalCommunicator(cols=2)
        h.row_comm = XgmiCommunicator(h.row_group, device=0, slot_bytes=1 << 20, grid=16, timeout_s=15.0)
        n = 2 * 40_000
        xs = [fill_uniform(torch.empty(n, device=DEV), seed=900 + k) for k in range(world)]
        y = h.allreduce(xs[rank], op="avg")
        h.row_comm.check()
        ref = sum(x for x in xs) / world
        err = (y - ref).abs().max().item()
        if err > 1e-5:
            ok, msg = False, f"err {err}"
        if h.row_comm.native.stats.coll < 2:
            ok, msg = False, "row steps did not run on the xGMI kernels"
    except Exception as e:  # noqa: BLE001
        ok, msg = False, repr(e)
    q.put((rank, ok, msg))
    dist.destroy_process_group()


def test_hierarchical_rows_on_xgmi_collectives():
    """2 x 2 grid of processes: reduce-scatter / all-gather inside a row on the xGMI kernels,
    the column allreduce on gloo."""
    from akka_allreduce_1_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_hier_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(4)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad


def _stress_worker(rank, world, port, q):
    """The same random sequence of operations on every rank (shared seed): every allreduce
    algorithm, the collectives and threshold rounds interleaved, random sizes and dtypes,
    in place and out of place - every result checked against gloo on fp32 copies."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import random

    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import XgmiCommunicator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, msg = True, ""
    try:
        comm = XgmiCommunicator(device=0, slot_bytes=512 << 10, grid=16, timeout_s=15.0, max_lag=1)
        rng = random.Random(1234)
        for it in range(int(os.environ.get("MXAR_STRESS_ITERS", "120"))):
            op = rng.choice(["twoshot", "oneshot", "ll", "ring", "auto", "threshold", "thr_algo", "a2a", "ag", "rs"])
            dtype = rng.choice([torch.float32, torch.bfloat16, torch.float16])
            el = 16 // torch.empty(0, dtype=dtype).element_size()
            m = rng.choice([1, 3, 100, 4096, 50_000, 200_000]) * el
            if op == "threshold":
                m = min(m, (512 << 10) // 16)  # one launch: n * es <= world * slot
            n = m * world if op in ("a2a", "rs") else m
            x = fill_uniform(torch.empty(n, dtype=dtype, device=DEV), seed=it * 100 + rank)
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=DEV), seed=it * 100 + k) for k in range(world)]
            tol = 1e-5 if dtype == torch.float32 else 2e-2 * world
            if op in ("twoshot", "oneshot", "ll", "ring", "auto", "threshold", "thr_algo"):
                inplace = rng.random() < 0.5
                if op == "thr_algo":  # the threshold kernel as an exact allreduce algorithm (falls back if too big)
                    y = comm.allreduce(x, x if inplace else None, algo="threshold")
                elif op == "threshold":
                    y = comm.allreduce_threshold(x, x if inplace else None)
                else:
                    y = comm.allreduce(x, x if inplace else None, algo=op)
                ref = sum(t.float() for t in xs)
            elif op == "a2a":
                y = comm.all_to_all(x)
                ref = torch.cat([xs[s][rank * m:(rank + 1) * m].float() for s in range(world)])
                tol = 0
            elif op == "ag":
                y = comm.all_gather(x)
                ref = torch.cat([t.float() for t in xs])
                tol = 0
            else:
                y = comm.reduce_scatter(x)
                ref = sum(t[rank * m:(rank + 1) * m].float() for t in xs)
            comm.check()
            err = (y.float() - ref).abs().max().item()
            if err > tol:
                ok, msg = False, f"it {it} {op} {dtype} m={m}: err {err}"
                break
    except Exception as e:  # noqa: BLE001
        ok, msg = False, repr(e)
    q.put((rank, ok, msg))
    dist.destroy_process_group()


def test_multiprocess_random_operation_stress():
    """4 ranks x 120 operations by default; MXAR_STRESS_RANKS / MXAR_STRESS_ITERS for a soak."""
    from akka_allreduce_1_amd.parallel import free_port

    world = int(os.environ.get("MXAR_STRESS_RANKS", "4"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_stress_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=float(os.environ.get("MXAR_STRESS_TIMEOUT", "110"))) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad
