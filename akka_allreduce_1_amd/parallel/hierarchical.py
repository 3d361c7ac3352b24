"""Two-level (row / column) allreduce.

The reference only names this layout: its peer map is "workers in the same row/col,
including self" (AllreduceWorker.scala:14), with one flat group implemented. On MI355X the
two levels are physical: a row is the 8 GPUs of one node on the xGMI mesh, a column is
the same local GPU across nodes (NIC). Each level runs the reference's two-shot pattern:

1. row reduce-scatter (ScatterBlock + reduce inside the node): rank (i, j) ends up with
   the node-sum of block j, 1/cols of the vector;
2. column allreduce of that block across nodes: only N/cols bytes per rank leave a node,
   and all `cols` NIC paths of a node carry traffic at once;
3. row all-gather (ReduceBlock broadcast inside the node).

Intra-node traffic equals a flat allreduce's; inter-node traffic drops by `cols` against
a flat ring across every rank. `col_comm` is anything with `allreduce_(t, op=...)`
(default: torch.distributed all_reduce on the column group, i.e. RCCL or gloo). `row_comm`
is anything with `reduce_scatter(inp, out)` / `all_gather(inp, out)` over the row group -
an `XgmiCommunicator(group=h.row_group)` runs both row steps as single xGMI launches
(csrc/hip/xgmi_coll.hip); default: torch.distributed on the row group.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class _GroupAllreduce:
    def __init__(self, group):
        self.group = group

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum") -> torch.Tensor:
        dist.all_reduce(t, group=self.group)
        if op == "avg":
            t.div_(dist.get_world_size(self.group))
        return t


class HierarchicalCommunicator:
    """Allreduce over a rows x cols grid of ranks (rank = row * cols + col)."""

    def __init__(self, cols: int, *, backend: str | None = None, col_comm=None, row_comm=None):
        if not dist.is_initialized():
            raise RuntimeError("HierarchicalCommunicator needs torch.distributed")
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        if cols < 1 or self.world % cols:
            raise ValueError(f"cols={cols} must divide world={self.world}")
        self.cols = cols
        self.rows = self.world // cols
        self.row, self.col = divmod(self.rank, cols)
        # every rank creates every group, in the same order (torch.distributed rule)
        row_groups = [dist.new_group([r * cols + c for c in range(cols)], backend=backend) for r in range(self.rows)]
        col_groups = [dist.new_group([r * cols + c for r in range(self.rows)], backend=backend)
                      for c in range(cols)]
        self.row_group = row_groups[self.row]
        self.col_group = col_groups[self.col]
        self.col_comm = col_comm if col_comm is not None else _GroupAllreduce(self.col_group)
        self.row_comm = row_comm
        self.stats = {"calls": 0, "row_bytes": 0, "col_bytes": 0}

    def allreduce(self, inp: torch.Tensor, out: torch.Tensor | None = None, *, op: str = "sum") -> torch.Tensor:
        """out = sum (or mean) over all ranks of inp; `out=inp` is in place."""
        if out is None:
            out = torch.empty_like(inp)
        if op not in ("sum", "avg"):
            raise ValueError(f"unsupported op {op!r}")
        x, y = inp.reshape(-1), out.view(-1)
        n = x.numel()
        C = self.cols
        b = -(-n // C)
        if n == C * b:
            src = x
        else:
            src = torch.zeros(C * b, dtype=x.dtype, device=x.device)
            src[:n].copy_(x)
        shard = torch.empty(b, dtype=x.dtype, device=x.device)
        # 1. intra-node reduce-scatter
        if C > 1 and self.row_comm is not None:
            self.row_comm.reduce_scatter(src, shard)
        elif C > 1:
            dist.reduce_scatter_tensor(shard, src, group=self.row_group)
        else:
            shard.copy_(src)
        # 2. inter-node allreduce of this rank's block
        if self.rows > 1:
            self.col_comm.allreduce_(shard, op="sum")
        if op == "avg":
            shard.div_(self.world)
        # 3. intra-node all-gather
        gather = (self.row_comm.all_gather if self.row_comm is not None else
                  lambda i, o: dist.all_gather_into_tensor(o, i, group=self.row_group))
        if C > 1 and n == C * b and y.data_ptr() != x.data_ptr():
            gather(shard, y)
        elif C > 1:
            full = torch.empty(C * b, dtype=x.dtype, device=x.device)
            gather(shard, full)
            y.copy_(full[:n])
        else:
            y.copy_(shard[:n])
        es = x.element_size()
        self.stats["calls"] += 1
        self.stats["row_bytes"] += 2 * (C - 1) * b * es
        self.stats["col_bytes"] += b * es
        return out

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum", algo: str | None = None) -> torch.Tensor:
        return self.allreduce(t, t, op=op)

    def __repr__(self) -> str:
        return f"HierarchicalCommunicator(rank={self.rank}, grid={self.rows}x{self.cols})"
