"""GPU side of the point-to-point protocol (parallel/p2p.py): the staged reduce runs the HIP
reduce_slots kernel on padded rows, and the XgmiCommunicator dispatches algo="p2p"/"rsag"
(RCCL point-to-point / reduce-scatter + all-gather) on the nccl backend. RCCL refuses two
ranks on one GPU, so the RCCL paths run as a 1-rank job here; the multi-rank protocol is
covered on gloo (tests/test_p2p_hier.py)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("P,n", [(2, 1), (3, 1001), (8, 65543)])
def test_reduce_rows_on_padded_staging_rows(dtype, P, n):
    from akka_allreduce_1_amd.ops import fill_uniform
    from akka_allreduce_1_amd.parallel.p2p import reduce_rows

    stride = (n + 7) // 8 * 8
    buf = fill_uniform(torch.empty(P * stride, dtype=dtype, device="cuda"), seed=P * n)
    slots = buf.view(P, stride)[:, :n]
    out = torch.empty(n, dtype=dtype, device="cuda")
    reduce_rows(slots, out, scale=0.25)
    ref = slots.float().sum(0) * 0.25
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert (out.float() - ref).abs().max().item() <= tol


def _one_rank(q):
    try:
        from akka_allreduce_1_amd.ops import fill_uniform
        from akka_allreduce_1_amd.parallel import XgmiCommunicator, init_distributed

        os.environ.pop("RANK", None)
        init_distributed("nccl")
        comm = XgmiCommunicator(slot_bytes=1 << 20)
        x = fill_uniform(torch.empty(300_001, dtype=torch.bfloat16, device="cuda"), seed=5)
        for algo in ("p2p", "rsag", "rccl", "twoshot"):
            y = comm.allreduce(x, algo=algo)
            torch.cuda.synchronize()
            assert torch.equal(y, x), algo
            z = comm.allreduce(x, op="avg", algo=algo)
            assert torch.equal(z, x), algo
        comm.check()
        assert comm.p2p.stats["calls"] == 4
        q.put((True, ""))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((False, traceback.format_exc()))


def test_xgmi_communicator_dispatches_rccl_p2p_algos():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_one_rank, args=(q,))
    p.start()
    ok, msg = q.get(timeout=180)
    p.join(timeout=60)
    if p.is_alive():
        p.kill()
    assert ok, msg
