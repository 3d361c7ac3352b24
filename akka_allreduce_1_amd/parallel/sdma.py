"""Bucket allreduce with the cross-rank copies on the SDMA copy engines (csrc/hip/sdma_comm.h).

The CU kernels of `XgmiCommunicator` move every byte with spinning workgroups; beside
backward's GEMMs those workgroups are CUs the GEMMs do not get (profiles/round3/README.md:
GEMMs 1.48x slower, comm 1.70x). Here the reference's ScatterBlock and ReduceBlock transfers
(AllreduceWorker.scala:194-238; SURVEY §2.4 K2, "hipMemcpyPeerAsync writes the source slice
directly into the owner's scatter slot") run on the copy engines; CUs only reduce the own
block and gather the peers' reduced blocks locally, in small grids.

`SdmaCommunicator`   one process per GPU (torch.distributed group), handles over gloo
`LocalSdmaCluster`   P logical ranks in ONE process on one GPU (rehearsal / tests); each rank
                     has its own stream and its own SDMA engines
"""
from __future__ import annotations

import os
from typing import Sequence

import torch

from .._native import C
from .comm import CommError, _KERNEL_DTYPES, _current_stream, _describe

_H = C.hip


_XDEV_VALIDATED = [False]


def mark_xdev_validated() -> None:
    """Allow SDMA copies across GPUs in this process: called once a cross-GPU SDMA allreduce of
    the same job has been validated where a fault could not take the caller down (bench.py
    runs it in child processes first, `benchmarks/sdma_xdev.py`)."""
    _XDEV_VALIDATED[0] = True


def xdev_allowed() -> bool:
    return _XDEV_VALIDATED[0] or os.environ.get("MXAR_SDMA_XDEV", "0") == "1"


class SdmaCommunicator:
    """Allreduce of the ranks of a torch.distributed group with SDMA cross-rank copies."""

    accepts_stream = True

    def __init__(self, group=None, *, device: torch.device | int | None = None, slot_bytes: int = 64 << 20,
                 grid: int = 128, engines_per_peer: int = 0, timeout_s: float = 20.0, cpu_group=None,
                 validate: bool = True):
        """validate: one small allreduce checked against the exact sum on every rank before the
        communicator is handed out (collective; a wrong result raises CommError everywhere)."""
        import torch.distributed as dist

        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if cpu_group is None:
            cpu_group = group if dist.get_backend(group) == "gloo" else dist.new_group(
                ranks=None if group is None else dist.get_process_group_ranks(group), backend="gloo")
        self.cpu_group = cpu_group
        # Engine copies into ANOTHER GPU's memory: allowed once validated for this job in a
        # process a fault cannot take down (mark_xdev_validated), or with MXAR_SDMA_XDEV=1.
        # Decided from the ranks' PCI locations BEFORE anything is allocated; every rank sees
        # the same locations, so every rank decides the same way.
        locs: list = [None] * self.world
        dist.all_gather_object(locs, int(_H.pci_location(self.device.index)), group=cpu_group)
        self.cross_gpu = len(set(locs)) > 1
        if self.cross_gpu and not xdev_allowed():
            raise CommError("SdmaCommunicator across GPUs needs a validated run first "
                            "(mark_xdev_validated / benchmarks/sdma_xdev.py) or MXAR_SDMA_XDEV=1")
        c, h, err = None, None, ""
        try:
            c = _H.SdmaComm(self.rank, self.world, self.device.index, slot_bytes, grid, engines_per_peer, timeout_s)
            h = c.handle()
        except Exception as e:  # noqa: BLE001 - every rank learns of it below
            err = f"rank {self.rank}: {e}"
        hs: list = [None] * self.world
        dist.all_gather_object(hs, (h, err), group=cpu_group)
        errs = [e for _, e in hs if e]
        if errs:
            raise CommError("SdmaCommunicator setup failed: " + "; ".join(errs))
        try:
            c.connect([x for x, _ in hs])
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {e}"
        st: list = [None] * self.world
        dist.all_gather_object(st, err, group=cpu_group)
        errs = [e for e in st if e]
        if errs:
            raise CommError("SdmaCommunicator connect failed: " + "; ".join(errs))
        self._c = c
        self._dev = self.device.index
        if validate:
            self.validate()

    def validate(self, n: int = 1 << 20 | 12345) -> float:
        """One allreduce of n fp32 elements against the exact sum (every rank regenerates every
        rank's input from its seed); collective. Returns the max error, raises CommError on
        any rank's failure."""
        import torch.distributed as dist

        from ..ops import fill_uniform

        err, msg = float("inf"), ""
        try:
            xs = [fill_uniform(torch.empty(n, device=self.device), seed=4242 + k) for k in range(self.world)]
            ref = torch.zeros(n, device=self.device)
            for x in xs:
                ref += x
            y = self.allreduce(xs[self.rank])
            torch.cuda.synchronize(self.device)
            self.check()
            err = (y - ref).abs().max().item()
        except Exception as e:  # noqa: BLE001 - every rank learns of it below
            msg = repr(e)
        ok = err <= 1e-5 * self.world
        res: list = [None] * self.world
        dist.all_gather_object(res, (ok, err, msg), group=self.cpu_group)
        bad = [(k, r) for k, r in enumerate(res) if not r[0]]
        if bad:
            raise CommError(f"SdmaCommunicator validation failed: {bad}")
        return max(r[1] for r in res)

    def allreduce(self, inp: torch.Tensor, out: torch.Tensor | None = None, *, op: str = "sum", algo: str = "sdma",
                  stream: int | None = None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(inp)
        if op not in ("sum", "avg"):
            raise ValueError(f"unsupported op {op!r}")
        code = _KERNEL_DTYPES.get(inp.dtype)
        if code is None or not (inp.is_contiguous() and out.is_contiguous()) or out.numel() != inp.numel():
            raise ValueError("SDMA allreduce: contiguous fp32 / bf16 / fp16 tensors of equal size")
        self._c.allreduce(inp.data_ptr(), out.data_ptr(), inp.numel(), code,
                          _current_stream(self._dev) if stream is None else stream,
                          1.0 / self.world if op == "avg" else 1.0)
        return out

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum", algo: str = "sdma", stream: int | None = None):
        return self.allreduce(t, t, op=op, stream=stream)

    @property
    def native(self):
        return self._c

    def check(self) -> None:
        e = self._c.error()
        if e:
            raise CommError(f"SDMA allreduce rank {self.rank}: {_describe(e)}")


class LocalSdmaCluster:
    """P logical ranks of the SDMA allreduce in one process on one GPU, all on the caller's
    stream in one interleaved schedule (SdmaComm::allreduce_local): every wait only needs
    releases queued before it, so no rank's wait can hold up a peer's progress."""

    def __init__(self, world: int, *, slot_bytes: int = 16 << 20, grid: int = 128, engines_per_peer: int = 0,
                 timeout_s: float = 10.0, device: int | None = None):
        dev = torch.cuda.current_device() if device is None else device
        self.world = world
        self.device = torch.device("cuda", dev)
        self.comms = [_H.SdmaComm(k, world, dev, slot_bytes, grid, engines_per_peer, timeout_s) for k in range(world)]
        for c in self.comms:
            c.connect_local(self.comms)

    def allreduce(self, inputs: Sequence[torch.Tensor], outputs: Sequence[torch.Tensor] | None = None, *,
                  op: str = "sum", stream: int | None = None) -> list[torch.Tensor]:
        if len(inputs) != self.world:
            raise ValueError("one input per logical rank")
        outputs = list(outputs) if outputs is not None else [torch.empty_like(x) for x in inputs]
        n = inputs[0].numel()
        for x, y in zip(inputs, outputs):
            if x.numel() != n or y.numel() != n or x.dtype != inputs[0].dtype or y.dtype != x.dtype:
                raise ValueError("all ranks must pass the same shape and dtype")
        _H.SdmaComm.allreduce_local(self.comms, [x.data_ptr() for x in inputs], [y.data_ptr() for y in outputs], n,
                                    _KERNEL_DTYPES[inputs[0].dtype],
                                    _current_stream(self.device.index) if stream is None else stream,
                                    1.0 / self.world if op == "avg" else 1.0)
        return outputs

    def check(self) -> None:
        for c in self.comms:
            e = c.error()
            if e:
                state = " || ".join(x.debug_state() for x in self.comms)
                raise CommError(f"SDMA allreduce rank {c.rank}: {_describe(e)}; state: {state}")
