"""Threshold (straggler-tolerant) fused allreduce - csrc/hip/xgmi_threshold.hip - on one MI355X.

The reference's thReduce / thComplete / maxLag semantics on the xGMI kernel:
* th = 1: identical to an exact allreduce, every chunk counts P contributions;
* a straggling rank (idling in the kernel): the other ranks reduce their blocks without it
  and give up its block (zeros, count 0) once thComplete of the chunks are in; the
  straggler itself still sees every contribution to its own block;
* the lag ring (multi-process, separate launches): a rank that runs ahead never
  overwrites a row the slower rank still reads - the slower rank's own block is exact in
  every round.
Reference sums are fp32 in rank order over the contributions the counts report.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from akka_allreduce_1_amd.ops import fill_uniform  # noqa: E402
from akka_allreduce_1_amd.parallel import LocalCluster  # noqa: E402

DEV = torch.device("cuda", 0)


def _sum(xs, ranks):
    acc = torch.zeros(xs[0].numel(), device=xs[0].device)
    for k in ranks:
        acc += xs[k].float()
    return acc


def _blocks(n, P, nch, dtype):
    """(block, chunk) geometry of the kernel: block = ceil(n/P) rounded to 16 B, chunk = ceil(block/nch)."""
    el = 16 // torch.empty(0, dtype=dtype).element_size()
    block = -(-n // P)
    block = -(-block // el) * el
    chunk = -(-block // nch)
    chunk = -(-chunk // el) * el
    return block, chunk


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("max_lag", [0, 2])
def test_threshold_one_is_exact(P, dtype, max_lag):
    cl = LocalCluster(P, slot_bytes=1 << 20, grid=64, timeout_s=10.0, max_lag=max_lag)
    for it in range(4):  # cycles through the lag-ring rows
        n = [100_003, 4096, 777][it % 3]
        xs = [fill_uniform(torch.empty(n, dtype=dtype, device=DEV), seed=31 * it + k) for k in range(P)]
        ys, counts = cl.allreduce_threshold(xs, th_reduce=1.0, th_complete=1.0)
        cl.check()
        ref = _sum(xs, range(P))
        for k, y in enumerate(ys):
            err = (y.float() - ref).abs().max().item()
            assert err <= (1e-6 if dtype == torch.float32 else 1e-2 * P), f"it {it} rank {k}: {err}"
        assert counts.shape[:2] == (P, P) and bool((counts == P).all()), counts
    assert cl.comms[0].stats.threshold == 4


@pytest.mark.parametrize("P", [3, 4])
def test_straggler_is_left_out_and_its_block_given_up(P):
    slow = P - 1
    cl = LocalCluster(P, slot_bytes=1 << 20, grid=32, timeout_s=10.0, max_lag=0)
    cl.comms[0].set_straggler(slow, 5000.0)  # 5 ms idle at the start of the slow rank
    th = (P - 1) / P
    n = 50_001
    xs = [fill_uniform(torch.empty(n, device=DEV), seed=900 + k) for k in range(P)]
    ys, counts = cl.allreduce_threshold(xs, th_reduce=th, th_complete=th)
    cl.check()
    nch = counts.shape[2]
    block, chunk = _blocks(n, P, nch, torch.float32)
    fast = [k for k in range(P) if k != slow]
    without = _sum(xs, fast)
    full = _sum(xs, range(P))
    for k in range(P):
        for j in range(P):
            lo, hi = j * block, min(n, (j + 1) * block)
            if lo >= hi:
                continue
            got = ys[k][lo:hi]
            cj = counts[k, j]
            if k == slow and j == slow:  # the straggler saw everyone's contribution to its block
                assert bool((cj == P).all()), cj
                torch.testing.assert_close(got, full[lo:hi], rtol=0, atol=1e-6)
            elif j == slow:  # fast ranks gave the straggler's block up
                assert bool((cj == 0).all()), cj
                assert bool((got == 0).all())
            else:  # blocks of fast owners: reduced without the straggler
                assert bool((cj == P - 1).all()), (k, j, cj)
                torch.testing.assert_close(got, without[lo:hi], rtol=0, atol=1e-6)


@pytest.mark.parametrize("P", [3, 4])
def test_straggler_rescaled_mean_over_contributors(P):
    """rescale=True + op="avg": a chunk summed from cnt contributions is divided by cnt
    (the mean over the ranks that made it), fused into the kernel."""
    slow = 0
    cl = LocalCluster(P, slot_bytes=1 << 20, grid=32, timeout_s=10.0, max_lag=0)
    cl.comms[0].set_straggler(slow, 5000.0)
    th = (P - 1) / P
    n = 20_011
    xs = [fill_uniform(torch.empty(n, device=DEV), seed=300 + k) for k in range(P)]
    ys, counts = cl.allreduce_threshold(xs, th_reduce=th, th_complete=th, op="avg", rescale=True)
    cl.check()
    block, _ = _blocks(n, P, counts.shape[2], torch.float32)
    fast_mean = _sum(xs, [k for k in range(P) if k != slow]) / (P - 1)
    full_mean = _sum(xs, range(P)) / P
    for k in range(P):
        for j in range(P):
            lo, hi = j * block, min(n, (j + 1) * block)
            if lo >= hi:
                continue
            got = ys[k][lo:hi]
            if k == slow and j == slow:
                torch.testing.assert_close(got, full_mean[lo:hi], rtol=0, atol=1e-6)
            elif j == slow:
                assert bool((got == 0).all())
            else:
                assert bool((counts[k, j] == P - 1).all())
                torch.testing.assert_close(got, fast_mean[lo:hi], rtol=0, atol=1e-6)


def _lag_worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import time

    import torch.distributed as dist

    from akka_allreduce_1_amd.ops.kernels import dtype_code
    from akka_allreduce_1_amd.parallel import XgmiCommunicator

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, msg = True, ""
    try:
        comm = XgmiCommunicator(device=0, slot_bytes=1 << 20, grid=8, timeout_s=20.0, max_lag=1)
        n, rounds = 40_000, 8
        nch = comm._c.threshold_chunks(n, dtype_code(torch.float32))
        block, chunk = _blocks(n, world, nch, torch.float32)
        outs = []
        for r in range(rounds):
            if rank == 1:
                time.sleep(0.02)  # the slow rank launches every round late
            x = fill_uniform(torch.empty(n, device=DEV), seed=1000 * r + rank)
            y, cnt = comm.allreduce_threshold(x, th_reduce=0.5, th_complete=0.5, counts=True)
            outs.append((y, cnt))
        comm.check()
        if rank == 0 and not any(bool((cnt[1] == 0).any()) for _, cnt in outs):
            ok, msg = False, "rank 0 never ran ahead of the slow rank (no given-up chunk)"
        for r, (y, cnt) in enumerate(outs):
            xs = [fill_uniform(torch.empty(n, device=DEV), seed=1000 * r + k) for k in range(world)]
            if rank == 1 and not bool((cnt[1] == 2).all()):  # slow rank: own block always complete
                ok, msg = False, f"round {r}: slow rank's own block counts {cnt[1].tolist()}"
            for j in range(world):
                lo, hi = j * block, min(n, (j + 1) * block)
                for c in range(nch):
                    clo, chi = lo + c * chunk, min(hi, lo + (c + 1) * chunk)
                    if clo >= chi:
                        continue
                    k = int(cnt[j, c])
                    if k == 2:
                        ref = _sum(xs, range(world))[clo:chi]
                    elif k == 1:
                        ref = xs[j][clo:chi].float()  # the owner's contribution alone
                    else:
                        ref = torch.zeros(chi - clo, device=DEV)
                    if (y[clo:chi] - ref).abs().max().item() > 1e-6:
                        ok, msg = False, f"round {r} block {j} chunk {c}: count {k} but data differs"
    except Exception as e:  # noqa: BLE001 - report, never hang the parent
        ok, msg = False, repr(e)
    results.put((rank, ok, msg))
    dist.destroy_process_group()


def test_lag_ring_two_processes():
    from akka_allreduce_1_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_lag_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad


def test_threshold_interleaved_with_lockstep_algorithms():
    """Threshold rounds keep their own round count and slab rows: interleaving them with
    two-shot / one-shot / ring launches on the same communicator stays correct."""
    P, n = 4, 30_011
    cl = LocalCluster(P, slot_bytes=1 << 20, grid=32, timeout_s=10.0, max_lag=1)
    for it, algo in enumerate(["twoshot", "threshold", "oneshot", "ring", "threshold", "threshold", "twoshot"]):
        xs = [fill_uniform(torch.empty(n, device=DEV), seed=77 * it + k) for k in range(P)]
        if algo == "threshold":
            ys, counts = cl.allreduce_threshold(xs)
            assert bool((counts == P).all())
        else:
            ys = cl.allreduce(xs, algo=algo)
        cl.check()
        ref = _sum(xs, range(P))
        for y in ys:
            assert (y - ref).abs().max().item() <= 1e-6, algo


def test_threshold_needs_a_lag_ring():
    cl = LocalCluster(2, slot_bytes=1 << 20, grid=8)
    xs = [torch.zeros(1024, device=DEV) for _ in range(2)]
    with pytest.raises(Exception, match="threshold_rows"):
        cl.allreduce_threshold(xs)


_ONESHOT_GRID_CHILD = r"""
import torch
from akka_allreduce_1_amd.ops import fill_uniform
from akka_allreduce_1_amd.parallel import LocalCluster
dev = torch.device("cuda", 0)
P, n = 8, 64 * 1024  # 128 KiB bf16 per rank
cl = LocalCluster(P, slot_bytes=(1 << 20), grid=64, timeout_s=5.0, max_lag=1)
xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=dev), seed=k) for k in range(P)]
ys = [torch.empty_like(x) for x in xs]
ref = sum(x.float() for x in xs)
for _ in range(3):
    cl.allreduce_threshold(xs, ys, counts=False)
    torch.cuda.synchronize()
    cl.check()
    err = max((y.float() - ref).abs().max().item() for y in ys)
    assert err <= ref.abs().max().item() * 2 ** -7, err
print("ok")
"""


def test_oneshot_body_workgroups_past_the_fast_pass():
    """The threshold kernel's one-shot body where the grid is too small for every workgroup's
    fast pass (default grid 64, 8 x 128 KiB, the body allowed up to 256 KiB): its chunk-by-chunk
    form timed out there, so the host now takes the two-shot body for such geometries - the
    rounds must complete exact (profiles/round6 section 12). A child process, so the
    construction-time knobs apply to it alone."""
    import subprocess
    import sys

    env = dict(os.environ, MXAR_GRID="64", MXAR_STUDY="1", MXAR_TH_ONESHOT_MAX=str(256 << 10))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _ONESHOT_GRID_CHILD], env=env, cwd=root, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]


def test_threshold_body_transitions_round_to_round():
    """Threshold rounds whose body changes from call to call on ONE cluster: one-shot (16 KiB,
    64 KiB), one-shot or two-shot by the grid guard (256 KiB at grid 64: 8 ranks share the
    launch), two-shot (512 KiB), then one-shot again - the rows, tags and flags each body leaves
    behind must not leak into the next (profiles/round6 section 12). Every round exact."""
    P = 8
    cl = LocalCluster(P, slot_bytes=1 << 20, grid=64, timeout_s=5.0, max_lag=1)
    for rep, S in enumerate([16 << 10, 64 << 10, 256 << 10, 512 << 10, 64 << 10, 16 << 10]):
        n = S // 2
        xs = [fill_uniform(torch.empty(n, dtype=torch.bfloat16, device=DEV), seed=k + 31 * rep) for k in range(P)]
        ys = [torch.empty_like(x) for x in xs]
        ref = sum(x.float() for x in xs)
        for _ in range(3):
            cl.allreduce_threshold(xs, ys, counts=False)
            torch.cuda.synchronize()
            cl.check()
            err = max((y.float() - ref).abs().max().item() for y in ys)
            assert err <= ref.abs().max().item() * 2 ** -7, (S, err)
