"""Thin wrappers: torch tensor -> (device pointer, stream) -> native HIP launch.

Kernels (csrc/hip/kernels.hip):
  reduce_slots  K1 of SURVEY §2.4, the reference's `reduce` (AllreduceWorker.scala:240-251)
  fill_iota     K9, the reference data source `data[i] = i + iteration` (AllreduceWorker.scala:285-291)
  fill_uniform  synthetic random gradients (benchmarks)
  cast          fp32 <-> bf16
  bucket_copy   flatten many gradient tensors into one bucket and back (bucket fusion)
"""
from __future__ import annotations

from typing import Sequence

import torch

from .._native import C

_H = C.hip
_DT = {torch.float32: _H.DType.F32, torch.bfloat16: _H.DType.BF16, torch.float16: _H.DType.F16}


def dtype_code(dt: torch.dtype):
    try:
        return _DT[dt]
    except KeyError:
        raise TypeError(f"unsupported dtype {dt}: the HIP data plane handles float32, bfloat16 and float16") from None


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def reduce_slots(slots: torch.Tensor, out: torch.Tensor | None = None, scale: float = 1.0) -> torch.Tensor:
    """out[i] = scale * sum_p slots[p, i] with fp32 accumulation in peer order 0..P-1.

    `slots` is a [P, n] tensor (float32 or bfloat16); rows must start 16-byte aligned.
    """
    if not slots.is_cuda:
        raise ValueError("slots must be a GPU tensor")
    if slots.dim() != 2 or slots.stride(1) != 1:
        raise ValueError("slots must be [P, n] with unit stride along n (rows may be padded)")
    P, n = slots.shape
    if out is None:
        out = torch.empty(n, dtype=slots.dtype, device=slots.device)
    _check(out, "out")
    if out.numel() != n or out.dtype != slots.dtype:
        raise ValueError("out must have n elements of the slots dtype")
    _H.reduce_slots(slots.data_ptr(), slots.stride(0), P, out.data_ptr(), n, dtype_code(slots.dtype), float(scale),
                    _stream(slots))
    return out


def fill_iota(t: torch.Tensor, offset: float = 0.0) -> torch.Tensor:
    """t[i] = i + offset (the reference's basic data source)."""
    _check(t, "t")
    _H.fill_iota(t.data_ptr(), t.numel(), float(offset), dtype_code(t.dtype), _stream(t))
    return t


def fill_uniform(t: torch.Tensor, seed: int) -> torch.Tensor:
    """t[i] = U(-1, 1) from a stateless hash of (seed, i): reproducible synthetic gradients."""
    _check(t, "t")
    _H.fill_uniform(t.data_ptr(), t.numel(), int(seed) & (2**64 - 1), dtype_code(t.dtype), _stream(t))
    return t


def cast(src: torch.Tensor, dtype: torch.dtype, out: torch.Tensor | None = None) -> torch.Tensor:
    _check(src, "src")
    if out is None:
        out = torch.empty(src.shape, dtype=dtype, device=src.device)
    _check(out, "out")
    _H.cast(src.data_ptr(), dtype_code(src.dtype), out.data_ptr(), dtype_code(out.dtype), src.numel(), _stream(src))
    return out


class BucketTable:
    """Device table of (ptr, numel, offset) triples for `bucket_copy`, built once per bucket."""

    def __init__(self, tensors: Sequence[torch.Tensor], offsets: Sequence[int], device: torch.device):
        rows = []
        for t, off in zip(tensors, offsets):
            _check(t, "bucket member")
            rows += [t.data_ptr(), t.numel(), int(off)]
        self.count = len(tensors)
        self.total = sum(t.numel() for t in tensors)
        self.table = torch.tensor(rows, dtype=torch.int64).to(device)


def bucket_copy(table: BucketTable, bucket: torch.Tensor, pack: bool) -> None:
    """pack=True: bucket[off_i : off_i + n_i] = t_i for every member; pack=False: the reverse."""
    _check(bucket, "bucket")
    _H.bucket_copy(table.table.data_ptr(), table.count, bucket.data_ptr(), dtype_code(bucket.dtype), bool(pack),
                   table.total, _stream(bucket))
