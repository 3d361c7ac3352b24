"""BucketedGradReducer + XgmiCommunicator: 2 processes on one MI355X (IPC-mapped slabs),
gradients overlapped with backward on the comm stream, checked against per-rank references.
mode "threshold": every bucket goes through the straggler-tolerant kernel (th = 1 with the
fused rescale, so the result must still be the exact mean)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _model(seed, dtype):
    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 128), torch.nn.GELU(),
                            torch.nn.Linear(128, 8))
    return m.to(device="cuda:0", dtype=dtype)


def _worker(rank, world, port, q, dtype, mode):
    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import BucketedGradReducer, XgmiCommunicator

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        thr = mode == "threshold"
        comm = XgmiCommunicator(device=0, slot_bytes=1 << 20, grid=8, timeout_s=15.0, max_lag=1 if thr else None)
        m, ref = _model(0, dtype), _model(0, dtype)
        red = BucketedGradReducer(m, comm, bucket_bytes=32 << 10, op="avg", rescale=thr,
                                  algo="auto" if thr else "twoshot@4",
                                  overlap="auto" if mode == "auto" else True, tune_steps=1)
        assert red.threshold == thr
        assert len(red.buckets) >= 3
        g = torch.Generator(device="cuda:0")
        data = [torch.randn(16, 64, device="cuda:0", generator=g.manual_seed(10 + r)).to(dtype) for r in range(world)]
        # auto: 5 tuning steps (one per candidate schedule), then the agreed schedule
        for step in range(7 if mode == "auto" else 3):
            red.zero_grad()
            m(data[rank] * (step + 1)).float().pow(2).mean().backward()
            red.wait()
            comm.check()
            grads = []
            for r in range(world):
                ref.zero_grad()
                ref(data[r] * (step + 1)).float().pow(2).mean().backward()
                grads.append([p.grad.float().clone() for p in ref.parameters()])
            for i, p in enumerate(m.parameters()):
                exp = sum(gr[i] for gr in grads) / world
                scale = exp.abs().max().item() + 1e-3
                tol = (1e-5 if dtype == torch.float32 else 2e-2) * scale
                err = (p.grad.float() - exp).abs().max().item()
                assert err <= tol, (step, i, err, tol)
        if mode == "auto":
            assert red.schedule is not None and "schedule" in red.stats, red.stats
            # communicator grid, 128 workgroups, a 32-CU slice, serial, and the copy-engine (SDMA)
            # allreduce
            sm = red.stats["schedule_ms"]
            assert len(sm) == 5 and "overlap:sdma" in sm and "overlap:cu32:twoshot@64" in sm, red.stats
        q.put((rank, True, ""))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["exact", "threshold", "auto"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ddp_reducer_xgmi_two_processes(dtype, mode):
    from akka_allreduce_1_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, dtype, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad[0][2]


def _mixed_stream_worker(rank, world, port, q):
    """The reducer's buckets are still queued on its comm stream when user code calls the SAME
    communicator on the default stream: the communicator orders the second stream after its
    previous launch (XgmiComm::order_after_last), so both results are exact."""
    import torch.distributed as dist

    from akka_allreduce_1_amd.ops import fill_uniform
    from akka_allreduce_1_amd.parallel import BucketedGradReducer, XgmiCommunicator

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = XgmiCommunicator(device=0, slot_bytes=1 << 20, grid=8, timeout_s=15.0)
        m, ref = _model(0, torch.float32), _model(0, torch.float32)
        red = BucketedGradReducer(m, comm, bucket_bytes=32 << 10, op="avg", algo="twoshot@4")
        g = torch.Generator(device="cuda:0")
        data = [torch.randn(16, 64, device="cuda:0", generator=g.manual_seed(50 + r)) for r in range(world)]
        for step in range(4):
            xs = [fill_uniform(torch.empty(300_001, device="cuda:0"), seed=100 * step + r) for r in range(world)]
            red.zero_grad()
            m(data[rank] * (step + 1)).pow(2).mean().backward()  # buckets enqueued on the comm stream
            y = comm.allreduce(xs[rank], algo="twoshot")  # default stream, same communicator
            red.wait()
            comm.check()
            exp_y = xs[0] + xs[1]
            assert (y - exp_y).abs().max().item() <= 1e-5, ("user allreduce", step)
            grads = []
            for r in range(world):
                ref.zero_grad()
                ref(data[r] * (step + 1)).pow(2).mean().backward()
                grads.append([p.grad.clone() for p in ref.parameters()])
            for i, p in enumerate(m.parameters()):
                exp = sum(gr[i] for gr in grads) / world
                err = (p.grad - exp).abs().max().item()
                assert err <= 1e-5 * (exp.abs().max().item() + 1e-3), ("reducer", step, i, err)
        assert comm.native.stats.stream_switches >= 4, comm.native.stats.stream_switches
        q.put((rank, True, ""))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_reducer_and_default_stream_share_a_communicator():
    from akka_allreduce_1_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_mixed_stream_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad[0][2]


def _zero_worker(rank, world, port, q, fused=False):
    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import ShardedDataParallel, XgmiCommunicator

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = XgmiCommunicator(device=0, slot_bytes=1 << 20, grid=8, timeout_s=15.0)
        make = lambda ps: torch.optim.Adam(ps, lr=1e-3)  # noqa: E731
        m, ref = _model(0, torch.float32), _model(0, torch.float32)
        if fused:  # one fused reduce-scatter + AdamW + all-gather launch per bucket
            zdp = ShardedDataParallel(m, comm, None, bucket_bytes=32 << 10,
                                      fused_adamw={"lr": 1e-3, "betas": (0.9, 0.999), "eps": 1e-8,
                                                   "weight_decay": 0.0}, step_in_backward=fused == "backward")
        else:
            zdp = ShardedDataParallel(m, comm, make, bucket_bytes=32 << 10)
        ref_opt = make(list(ref.parameters()))
        g = torch.Generator(device="cuda:0")
        data = [torch.randn(16, 64, device="cuda:0", generator=g.manual_seed(30 + r)) for r in range(world)]
        for step in range(3):
            zdp.zero_grad()
            m(data[rank]).pow(2).mean().backward()
            zdp.step()
            comm.check()
            grads = []
            for r in range(world):
                ref.zero_grad()
                ref(data[r]).pow(2).mean().backward()
                grads.append([p.grad.clone() for p in ref.parameters()])
            for i, p in enumerate(ref.parameters()):
                p.grad = sum(gr[i] for gr in grads) / world
            ref_opt.step()
            for p, rp in zip(m.parameters(), ref.parameters()):
                err = (p - rp).abs().max().item()
                assert err <= 1e-5, (step, err)
        if fused:
            assert comm.native.stats.adamw == 3 * len(zdp.buckets)
            # resume: a fresh model + ShardedDataParallel loaded from a checkpoint of this state
            # takes the same next step as the original
            import copy

            saved, msaved = copy.deepcopy(zdp.state_dict()), copy.deepcopy(m.state_dict())

            def one(mm, zz):
                zz.zero_grad()
                mm(data[rank] * 2).pow(2).mean().backward()
                zz.step()
                comm.check()

            one(m, zdp)
            m2 = _model(1, torch.float32)
            m2.load_state_dict(msaved)
            zdp2 = ShardedDataParallel(m2, comm, None, bucket_bytes=32 << 10,
                                       fused_adamw={"lr": 1e-3, "betas": (0.9, 0.999), "eps": 1e-8,
                                                    "weight_decay": 0.0}, step_in_backward=fused == "backward")
            zdp2.load_state_dict(saved)
            one(m2, zdp2)
            for p, p2 in zip(m.parameters(), m2.parameters()):
                assert (p - p2).abs().max().item() <= 1e-6
        else:
            assert comm.native.stats.coll >= 2 * 3 * len(zdp.buckets)  # RS + AG per bucket per step on xGMI
        q.put((rank, True, ""))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fused", [False, "step", "backward"])
def test_sharded_data_parallel_xgmi_two_processes(fused):
    from akka_allreduce_1_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_zero_worker, args=(r, 2, port, q, fused)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    bad = [r for r in res if not r[1]]
    assert not bad, bad[0][2]


def test_comm_stream_has_priority_over_compute():
    """Side streams for overlapped collectives are high priority: a normal-priority stream can
    share the compute stream's hardware queue and then serialises with it
    (profiles/zero_step_in_backward.md)."""
    from akka_allreduce_1_amd.parallel.comm import comm_stream

    s = comm_stream(torch.device("cuda", 0))
    assert s.priority < torch.cuda.current_stream(0).priority


def test_process_with_cu_masked_streams_exits_cleanly():
    """A process that made CU-masked streams (compute_stream_excluding, the "cuN:" schedules)
    and ran work on them exits with status 0: the streams still alive at interpreter exit are
    destroyed by an atexit hook while the HIP runtime is whole (ddp.py _destroy_live_masked; a
    masked stream left to the runtime's own teardown once ended the process with SIGSEGV)."""
    import subprocess
    import sys

    code = (
        "import torch\n"
        "from akka_allreduce_1_amd.parallel.ddp import compute_stream_excluding\n"
        "s = compute_stream_excluding('cuda:0', 32)\n"
        "with torch.cuda.stream(s):\n"
        "    a = torch.randn(1024, 1024, device='cuda:0'); b = (a @ a).sum()\n"
        "torch.cuda.synchronize(); print('ok', float(b) == float(b))\n"
    )
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=root,
                       env=dict(os.environ, PYTHONPATH=root))
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert "ok True" in r.stdout
