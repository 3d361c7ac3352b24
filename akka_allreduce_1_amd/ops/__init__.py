"""HIP/CDNA4 data-plane ops on torch tensors (gfx950 kernels in `csrc/hip/kernels.hip`).

Every op runs the in-tree native kernel; there is no eager PyTorch fallback. On a machine
without a GPU the ops raise (tests for them are marked `gpu`).
"""
from .kernels import bucket_copy, cast, dtype_code, fill_iota, fill_uniform, reduce_slots  # noqa: F401
