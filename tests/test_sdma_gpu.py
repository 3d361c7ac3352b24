"""SDMA bucket allreduce (csrc/hip/sdma_comm.h): cross-rank copies on the copy engines, a
small-grid reduce and gather on the CUs. Compared with an fp32 torch reference summed in
rank order (one rounding)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402

DEV = torch.device("cuda", 0)


def _ref(xs):
    acc = torch.zeros(xs[0].numel(), device=xs[0].device)
    for x in xs:
        acc += x.float()
    return acc


def _tol(dtype, P):
    return 1e-6 * P if dtype == torch.float32 else 1e-2 * P


@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [7, 4096 + 5, 1 << 20, 3_000_017])
def test_local_sdma_allreduce(P, dtype, n):
    from akka_allreduce_1_amd.parallel import LocalSdmaCluster

    cl = LocalSdmaCluster(P, slot_bytes=2 << 20, grid=8)
    for it in range(3):  # both slot parities, then reuse
        xs = [fill_uniform(torch.empty(n, dtype=dtype, device=DEV), seed=50 * it + k) for k in range(P)]
        ys = cl.allreduce(xs)
        torch.cuda.synchronize()
        cl.check()
        ref = _ref(xs)
        for k, y in enumerate(ys):
            err = (y.float() - ref).abs().max().item()
            assert err <= _tol(dtype, P), (it, k, err)


def test_local_sdma_inplace_mean_and_many_calls():
    from akka_allreduce_1_amd.parallel import LocalSdmaCluster

    P = 2
    cl = LocalSdmaCluster(P, slot_bytes=1 << 20, grid=4)
    for it in range(40):  # more calls than the signal ring holds
        n = [1000, 300_001, 65_536][it % 3]
        xs = [fill_uniform(torch.empty(n, device=DEV), seed=it * 7 + k) for k in range(P)]
        ref = _ref(xs) / P
        cl.allreduce(xs, xs, op="avg")
        for y in xs:
            torch.testing.assert_close(y, ref, rtol=0, atol=1e-6)
    cl.check()
    assert cl.comms[0].stats["calls"] >= 40


def _mp_worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import SdmaCommunicator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, msg = True, ""
    try:
        comm = SdmaCommunicator(device=0, slot_bytes=2 << 20, grid=8, engines_per_peer=1, timeout_s=15.0)
        for it, (n, dtype) in enumerate([(100_003, torch.float32), (1 << 20, torch.bfloat16), (5, torch.float32),
                                         (3_000_001, torch.bfloat16)] * 2):
            xs = [fill_uniform(torch.empty(n, dtype=dtype, device=DEV), seed=100 * it + k) for k in range(world)]
            y = comm.allreduce(xs[rank])
            torch.cuda.synchronize()
            comm.check()
            err = (y.float() - _ref(xs)).abs().max().item()
            if err > _tol(dtype, world):
                ok, msg = False, f"it {it} n={n} {dtype} err={err}"
                break
    except Exception as e:  # report, never hang the parent
        ok, msg = False, repr(e)
    results.put((rank, ok, msg))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_sdma_allreduce(world):
    from akka_allreduce_1_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_mp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad
