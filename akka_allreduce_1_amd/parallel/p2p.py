"""The reference's direct allreduce protocol over torch.distributed point-to-point.

The reference moves every ScatterBlock / ReduceBlock as an individual actor message over
Akka remoting (AllreduceWorker.scala:194-209 scatter, :230-238 broadcast). Its MI355X
counterpart for ranks whose slabs are NOT directly mapped (different nodes, or a fabric
without IPC) is point-to-point RCCL: grouped `send`/`recv` per peer, which RCCL runs as
one fused launch per group over xGMI (or the NIC between nodes). The same code runs on
gloo for the CPU tests.

`P2PCommunicator.allreduce` with algo="p2p", per segment of at most `world * chunk`
elements:

1. **ScatterBlock**: block j of the input goes to rank j; rank r receives the P-1 other
   contributions to its own block into the staging rows `slots[s]` (one grouped
   send/recv batch, peers in the reference's rotated order `(r + 1 + i) % P`).
2. **reduce**: `slots[r]` holds the own input; the P rows are summed with fp32
   accumulation in rank order (the HIP `reduce_slots` kernel on GPU,
   AllreduceWorker.scala:240-251; an fp32 torch sum on CPU), scaled once (mean fused),
   rounded once, straight into the output block.
3. **ReduceBlock broadcast**: the reduced block goes to every peer; every peer's block is
   received straight into the output (a second grouped batch).

`chunk_bytes` plays the role of the reference's `maxChunkSize` (AllreduceMessage.scala:15):
it caps the staging memory and the size of one P2P message. algo="rsag" is the library
form of the same two phases (`reduce_scatter_tensor` + `all_gather_into_tensor`).
Thresholds < 1 are not offered here: a posted P2P receive cannot be abandoned, which is why
the straggler-tolerant path lives in the xGMI kernels (csrc/hip/xgmi_threshold.hip).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def reduce_rows(slots: torch.Tensor, out: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """out = scale * sum over the rows of `slots`, fp32 accumulation in row order, one
    rounding. GPU float32/bfloat16/float16 -> the HIP reduce_slots kernel; anything else -> torch."""
    if slots.is_cuda and slots.dtype in (torch.float32, torch.bfloat16, torch.float16):
        from ..ops import reduce_slots

        return reduce_slots(slots, out, scale=scale)
    acc = slots[0].to(torch.float32)
    for s in range(1, slots.shape[0]):
        acc = acc + slots[s].to(torch.float32)
    if scale != 1.0:
        acc = acc * scale
    out.copy_(acc)
    return out


def block_bounds(m: int, world: int, align: int = 1) -> list[tuple[int, int]]:
    """Block j = [j*b, min((j+1)*b, m)) with b = ceil(m / P) (AllreduceWorker.scala:211-228)
    rounded up to a multiple of `align` elements, trailing blocks empty instead of the
    reference's short range table."""
    b = -(-m // world)
    b = -(-b // align) * align
    return [(min(j * b, m), min((j + 1) * b, m)) for j in range(world)]


class P2PCommunicator:
    """Direct two-shot allreduce from grouped point-to-point sends (RCCL or gloo)."""

    ALGOS = ("p2p", "rsag")

    def __init__(self, group=None, *, chunk_bytes: int = 64 << 20):
        if not dist.is_initialized():
            raise RuntimeError("P2PCommunicator needs torch.distributed")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.chunk_bytes = int(chunk_bytes)
        self._staging: tuple | None = None  # (key, tensor): one live staging buffer
        self.stats = {"calls": 0, "segments": 0, "bytes": 0, "p2p_ops": 0}

    def _peer(self, k: int) -> int:
        return k if self.group is None else dist.get_global_rank(self.group, k)

    def _rows(self, rows: int, n: int, like: torch.Tensor) -> torch.Tensor:
        """[rows, n] staging view; row starts 16-B aligned for the reduce kernel."""
        align = max(1, 16 // like.element_size())
        stride = (n + align - 1) // align * align
        key = (like.device, like.dtype)
        if self._staging is None or self._staging[0] != key or self._staging[1].numel() < rows * stride:
            self._staging = (key, torch.empty(rows * stride, dtype=like.dtype, device=like.device))
        return self._staging[1][:rows * stride].view(rows, stride)[:, :n]

    def _batch(self, ops: list) -> None:
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            self.stats["p2p_ops"] += len(ops)

    # ------------------------------------------------------------------ collectives
    def allreduce(self, inp: torch.Tensor, out: torch.Tensor | None = None, *, op: str = "sum",
                  algo: str = "p2p") -> torch.Tensor:
        """out = sum (or mean) over ranks of inp; `out=inp` is in place."""
        if out is None:
            out = torch.empty_like(inp)
        if not (inp.is_contiguous() and out.is_contiguous()) or inp.numel() != out.numel() or inp.dtype != out.dtype:
            raise ValueError("inp/out must be contiguous with the same numel and dtype")
        if op not in ("sum", "avg"):
            raise ValueError(f"unsupported op {op!r}")
        if algo not in self.ALGOS:
            raise ValueError(f"unknown algo {algo!r} (one of {self.ALGOS})")
        scale = 1.0 / self.world if op == "avg" else 1.0
        x, y = inp.view(-1), out.view(-1)
        n = x.numel()
        self.stats["calls"] += 1
        self.stats["bytes"] += n * x.element_size()
        if self.world == 1:
            if y.data_ptr() != x.data_ptr():
                y.copy_(x)
            if scale != 1.0:
                y.mul_(scale)
            return out
        seg = self.world * max(1, self.chunk_bytes // x.element_size())
        for off in range(0, n, seg):
            m = min(seg, n - off)
            (self._segment_p2p if algo == "p2p" else self._segment_rsag)(x[off:off + m], y[off:off + m], scale)
            self.stats["segments"] += 1
        return out

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum", algo: str = "p2p") -> torch.Tensor:
        return self.allreduce(t, t, op=op, algo=algo)

    def _segment_p2p(self, x: torch.Tensor, y: torch.Tensor, scale: float) -> None:
        P, r = self.world, self.rank
        # GPU: 16-B aligned blocks, so the reduce kernel can write the output block in place
        bounds = block_bounds(x.numel(), P, 16 // x.element_size() if x.is_cuda else 1)
        lo, hi = bounds[r]
        blen = hi - lo
        order = [(r + 1 + i) % P for i in range(P - 1)]  # rotated fan-out, AllreduceWorker.scala:197
        slots = self._rows(P, max(blen, 1), x)
        # 1. ScatterBlock: my part of block j to j; the peers' parts of my block into slots
        ops = []
        for j in order:
            jlo, jhi = bounds[j]
            if jhi > jlo:
                ops.append(dist.P2POp(dist.isend, x[jlo:jhi], self._peer(j), self.group))
            if blen > 0:
                ops.append(dist.P2POp(dist.irecv, slots[j, :blen], self._peer(j), self.group))
        self._batch(ops)
        # 2. reduce into the output block (the own row is staged too: the rows share one
        # stride for the kernel, and an in-place call overwrites the input block)
        if blen > 0:
            slots[r, :blen].copy_(x[lo:hi])
            dst = y[lo:hi]
            if dst.is_cuda and dst.data_ptr() % 16:  # unaligned output tensor: reduce into the own row
                reduce_rows(slots[:, :blen], slots[r, :blen], scale)
                dst.copy_(slots[r, :blen])
            else:
                reduce_rows(slots[:, :blen], dst, scale)
        # 3. ReduceBlock broadcast: my reduced block to every peer, theirs into my output
        ops = []
        for j in order:
            jlo, jhi = bounds[j]
            if blen > 0:
                ops.append(dist.P2POp(dist.isend, y[lo:hi], self._peer(j), self.group))
            if jhi > jlo:
                ops.append(dist.P2POp(dist.irecv, y[jlo:jhi], self._peer(j), self.group))
        self._batch(ops)

    def _segment_rsag(self, x: torch.Tensor, y: torch.Tensor, scale: float) -> None:
        """reduce_scatter_tensor + all_gather_into_tensor over equal padded blocks."""
        P = self.world
        m = x.numel()
        b = -(-m // P)
        if m == P * b:
            src = x
        else:
            src = self._rows(1, P * b, x)[0]
            src[:m].copy_(x)
            src[m:].zero_()
        shard = torch.empty(b, dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(shard, src, group=self.group)
        if scale != 1.0:
            shard.mul_(scale)
        if m == P * b and y.data_ptr() != x.data_ptr():
            dist.all_gather_into_tensor(y, shard, group=self.group)
        else:
            full = torch.empty(P * b, dtype=x.dtype, device=x.device)
            dist.all_gather_into_tensor(full, shard, group=self.group)
            y.copy_(full[:m])

    def __repr__(self) -> str:
        return f"P2PCommunicator(rank={self.rank}, world={self.world}, chunk={self.chunk_bytes >> 20} MiB)"
