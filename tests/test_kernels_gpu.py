"""Numerics of the HIP data-plane kernels vs plain PyTorch fp32 references (gfx950)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from akka_allreduce_1_amd.ops import bucket_copy, cast, fill_iota, fill_uniform, reduce_slots  # noqa: E402
from akka_allreduce_1_amd.ops.kernels import BucketTable  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("P,n", [(1, 1000), (2, 4096), (3, 12345), (8, 1 << 20), (5, 7)])
def test_reduce_slots_matches_fp32_reference(dtype, P, n):
    padded = torch.randn(P, (n + 7) // 8 * 8, device=DEV).to(dtype)  # 16-B aligned rows
    slots = padded[:, :n]
    out = reduce_slots(slots)
    ref = torch.zeros(n, device=DEV)
    for p in range(P):  # same summation order as the kernel and the reference's reduce loop
        ref += slots[p].float()
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert torch.equal(out, ref)
    else:  # one rounding of the fp32 sum (RNE), like torch's conversion
        assert torch.equal(out, ref.to(dtype))


def test_reduce_slots_scale_and_tail():
    slots = torch.randn(4, 1008, device=DEV)[:, :1003]
    out = reduce_slots(slots, scale=0.25)
    ref = slots.sum(0) * 0.25
    torch.cuda.synchronize()
    assert torch.allclose(out, ref, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_fill_iota_is_reference_data_source(dtype):
    t = fill_iota(torch.empty(1000, dtype=dtype, device=DEV), offset=3)
    ref = (torch.arange(1000, device=DEV, dtype=torch.float64) + 3).to(dtype)
    assert torch.equal(t, ref)


def test_fill_uniform_range_and_determinism():
    a = fill_uniform(torch.empty(1 << 16, device=DEV), seed=5)
    b = fill_uniform(torch.empty(1 << 16, device=DEV), seed=5)
    c = fill_uniform(torch.empty(1 << 16, device=DEV), seed=6)
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert a.min() >= -1 and a.max() < 1 and abs(a.mean().item()) < 0.02


@pytest.mark.parametrize("low", [torch.bfloat16, torch.float16])
def test_cast_roundtrip_matches_torch(low):
    x = torch.randn(100_003, device=DEV)
    y = cast(x, low)
    assert torch.equal(y, x.to(low))
    z = cast(y, torch.float32)
    assert torch.equal(z, y.float())
    other = torch.float16 if low == torch.bfloat16 else torch.bfloat16
    assert torch.equal(cast(y, other), y.float().to(other))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_bucket_copy_pack_unpack(dtype):
    ts = [torch.randn(s, device=DEV).to(dtype) for s in (17, 4096, 3, 1000, 64)]
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o += (t.numel() + 7) // 8 * 8  # 16-B aligned member offsets
    bucket = torch.zeros(o, dtype=dtype, device=DEV)
    table = BucketTable(ts, offs, DEV)
    bucket_copy(table, bucket, pack=True)
    for t, off in zip(ts, offs):
        assert torch.equal(bucket[off:off + t.numel()], t)
    bucket.mul_(2)
    bucket_copy(table, bucket, pack=False)
    torch.cuda.synchronize()
    for t, off in zip(ts, offs):
        assert torch.equal(t, bucket[off:off + t.numel()])
