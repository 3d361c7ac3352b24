"""BucketedGradReducer on CPU with gloo (world 2, multi-process) and bucket layout math."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from akka_allreduce_1_amd.parallel.ddp import BucketedGradReducer, TorchDistComm, bucket_sizes


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(7, 33), torch.nn.ReLU(), torch.nn.Linear(33, 5), torch.nn.ReLU(),
                               torch.nn.Linear(5, 3))


def test_bucket_layout_single_process():
    import torch.distributed as dist

    if dist.is_initialized():
        pytest.skip("dist already initialised")
    m = _model(0)
    shapes = [tuple(p.shape) for p in m.parameters()]
    sizes = bucket_sizes(shapes, 4, bucket_bytes=200 * 4)
    assert sum(sizes) >= sum(p.numel() for p in m.parameters()) * 4
    assert all(s % 16 == 0 for s in sizes)


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model(0)  # identical init on every rank
        ref = _model(0)
        red = BucketedGradReducer(m, TorchDistComm(), bucket_bytes=256, op="avg")
        assert len(red.buckets) > 1
        data = [torch.randn(4, 7, generator=torch.Generator().manual_seed(100 + r)) for r in range(world)]
        for step in range(3):
            red.zero_grad()
            m(data[rank] * (step + 1)).pow(2).sum().backward()
            red.wait()
            # reference: average of per-rank gradients computed locally
            grads = []
            for r in range(world):
                ref.zero_grad()
                ref(data[r] * (step + 1)).pow(2).sum().backward()
                grads.append([p.grad.clone() for p in ref.parameters()])
            for i, p in enumerate(m.parameters()):
                exp = sum(g[i] for g in grads) / world
                assert torch.allclose(p.grad, exp, atol=1e-5), (step, i)
            # gradients are bucket views
            for b in red.buckets:
                for p, off in zip(b.params, b.offsets):
                    assert p.grad.data_ptr() == b.buffer.data_ptr() + off * b.buffer.element_size()
        # unused parameter still reduced (as zeros) and the collective order stays aligned
        extra = torch.nn.Linear(3, 3)
        m2 = torch.nn.ModuleList([m, extra])
        red.remove_hooks()
        red2 = BucketedGradReducer(m2, TorchDistComm(), bucket_bytes=128)
        red2.zero_grad()
        m(data[rank]).sum().backward()
        red2.wait()
        assert torch.all(extra.weight.grad == 0)
        # schedule agreement (overlap="auto"): a schedule is as fast as its slowest rank, and
        # every rank keeps the same one - rank 0 alone would pick 0, rank 1 alone 1
        times = [[1.0, 5.0, 3.0], [4.0, 2.0, 3.0]][rank]
        i, best = red2._agree(times)
        assert i == 2 and best.tolist() == [4.0, 5.0, 3.0], (i, best)
        q.put((rank, True, ""))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_reducer_gloo_world2():
    from akka_allreduce_1_amd.parallel.comm import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    bad = [r for r in res if not r[1]]
    assert not bad, bad[0][2]


def _zero_worker(rank, world, port, q):
    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import ShardedDataParallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for opt_name in ("sgd", "adam"):
            make = (lambda ps: torch.optim.SGD(ps, lr=0.05, momentum=0.9)) if opt_name == "sgd" else (
                lambda ps: torch.optim.Adam(ps, lr=0.01))
            m, ref = _model(0), _model(0)
            zdp = ShardedDataParallel(m, TorchDistComm(), make, bucket_bytes=300)
            assert len(zdp.buckets) > 1
            ref_opt = make(list(ref.parameters()))
            data = [torch.randn(4, 7, generator=torch.Generator().manual_seed(200 + r)) for r in range(world)]
            for step in range(4):
                zdp.zero_grad()
                m(data[rank] * (step + 1)).pow(2).sum().backward()
                zdp.step()
                # reference: full optimizer on the averaged full gradient
                ref_opt.zero_grad()
                grads = []
                for r in range(world):
                    ref.zero_grad()
                    ref(data[r] * (step + 1)).pow(2).sum().backward()
                    grads.append([p.grad.clone() for p in ref.parameters()])
                for i, p in enumerate(ref.parameters()):
                    p.grad = sum(g[i] for g in grads) / world
                ref_opt.step()
                for p, rp in zip(m.parameters(), ref.parameters()):
                    assert torch.allclose(p, rp, atol=1e-5), (opt_name, step)
            # every rank holds optimizer state for its shard only
            n_state = sum(t.numel() for st in zdp.optimizer.state.values() for t in st.values() if torch.is_tensor(t)
                          and t.dim() > 0)
            total = sum(b.numel for b in zdp.buckets)
            assert n_state <= total * (2 if opt_name == "adam" else 1) // world
            zdp.remove_hooks()
        q.put((rank, True, ""))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_data_parallel_matches_full_optimizer_gloo():
    from akka_allreduce_1_amd.parallel.comm import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_zero_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    bad = [r for r in res if not r[1]]
    assert not bad, bad[0][2]


def _resume_worker(rank, world, port, q, path):
    """Train 3 steps, checkpoint (model once + one optimizer shard per rank), train 2 more;
    a fresh model + ShardedDataParallel loaded from the checkpoint must reproduce those 2."""
    import torch.distributed as dist

    from akka_allreduce_1_amd.parallel import ShardedDataParallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def make(ps):
            return torch.optim.Adam(ps, lr=0.01)
        data = [torch.randn(4, 7, generator=torch.Generator().manual_seed(300 + s)) for s in range(5)]

        def train(m, zdp, steps):
            for s in steps:
                zdp.zero_grad()
                m(data[s] * (rank + 1)).pow(2).sum().backward()
                zdp.step()

        m = _model(0)
        zdp = ShardedDataParallel(m, TorchDistComm(), make, bucket_bytes=300)
        train(m, zdp, range(3))
        if rank == 0:
            torch.save(m.state_dict(), os.path.join(path, "model.pt"))
        torch.save(zdp.state_dict(), os.path.join(path, f"optim_rank{rank}.pt"))
        dist.barrier()
        train(m, zdp, range(3, 5))

        m2 = _model(1)  # different init: everything must come from the checkpoint
        m2.load_state_dict(torch.load(os.path.join(path, "model.pt"), weights_only=True))
        zdp2 = ShardedDataParallel(m2, TorchDistComm(), make, bucket_bytes=300)
        zdp2.load_state_dict(torch.load(os.path.join(path, f"optim_rank{rank}.pt"), weights_only=True))
        assert zdp2.stats["steps"] == 3
        train(m2, zdp2, range(3, 5))
        for p, p2 in zip(m.parameters(), m2.parameters()):
            assert torch.equal(p, p2)
        bad = dict(zdp2.state_dict(), rank=(rank + 1) % world)
        try:
            zdp.load_state_dict(bad)
            raise AssertionError("a checkpoint of another rank must be refused")
        except ValueError:
            pass
        zdp.remove_hooks()
        zdp2.remove_hooks()
        q.put((rank, True, ""))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((rank, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_checkpoint_resume_gloo(tmp_path):
    from akka_allreduce_1_amd.parallel.comm import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_resume_worker, args=(r, 2, port, q, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    bad = [r for r in res if not r[1]]
    assert not bad, bad[0][2]
