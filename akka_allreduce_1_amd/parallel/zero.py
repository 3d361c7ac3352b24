"""Sharded data parallelism on the reference's two phases (ZeRO-2 style).

An allreduce is a reduce-scatter followed by an all-gather (the reference's ScatterBlock +
reduce, then ReduceBlock broadcast: AllreduceWorker.scala:194-251). Data-parallel training
does not need the second half for gradients: after the reduce-scatter every rank owns the
averaged gradient of 1/P of the parameters, so it can keep the optimizer state for that
1/P only, update its parameter shard, and all-gather the updated parameters. Same bytes on
the wire as an allreduce, 1/P of the optimizer memory and optimizer FLOPs per rank.

`ShardedDataParallel(model, comm, optimizer_factory)`:

* parameters are grouped into buckets of ~`bucket_bytes`; each bucket has ONE flat
  parameter buffer and ONE flat gradient buffer, and every `param.data` / `param.grad` is a
  view into them (sizes padded to a multiple of world x 16 B so shards stay aligned);
* a post-accumulate-grad hook launches a bucket's reduce-scatter (mean) on a side stream as
  soon as the bucket is complete - overlapped with the rest of backward;
* `step()` joins the side stream, runs the optimizer on the local shard views (one flat
  parameter per bucket: `optimizer_factory(list_of_shard_params)`), then all-gathers every
  bucket's updated shard back into the full flat parameter buffer.

`comm` needs `reduce_scatter(inp, out, op=)` and `all_gather(inp, out)` on the current stream:
`XgmiCommunicator` (one xGMI launch each, csrc/hip/xgmi_coll.hip) or `TorchDistComm` (RCCL /
gloo).

`fused_adamw={"lr": ..., "betas": ..., "eps": ..., "weight_decay": ...}` (XgmiCommunicator
only): every bucket's reduce-scatter, AdamW on the fp32 shard state and parameter all-gather
run as ONE launch per bucket at `step()` (csrc/hip/xgmi_adam.hip); `optimizer_factory` is
then unused (pass None) and the optimizer state is `self.adamw_states`.

`step_in_backward=True` (with `fused_adamw`, GPU): a bucket's fused step is launched on the
side stream the moment its last gradient is accumulated, so communication AND the optimizer
overlap the rest of backward ("optimizer in backward"). Valid because a parameter's
AccumulateGrad hook fires after its autograd node has used it; parameters shared between
layers (tied weights) must not be used with this mode. `comm_grid` sets the workgroup count
of the fused launches (0 = engine default).
"""
from __future__ import annotations

from typing import Callable, Iterable

import torch

from .comm import comm_stream

_ALIGN_BYTES = 16


class _Bucket:
    def __init__(self, index: int, dtype: torch.dtype):
        self.index = index
        self.dtype = dtype
        self.params: list[torch.nn.Parameter] = []
        self.offsets: list[int] = []
        self.numel = 0
        self.flat_param: torch.Tensor | None = None
        self.flat_grad: torch.Tensor | None = None
        self.grad_shard: torch.Tensor | None = None
        self.shard_param: torch.nn.Parameter | None = None
        self.pending = 0
        self.launched = False


class ShardedDataParallel:
    def __init__(self, module: torch.nn.Module | Iterable[torch.nn.Parameter], comm,
                 optimizer_factory: Callable[[list[torch.nn.Parameter]], torch.optim.Optimizer] | None, *,
                 bucket_bytes: int = 64 << 20, overlap: bool = True, fused_adamw: dict | None = None,
                 step_in_backward: bool = False, comm_grid: int = 0):
        params = module.parameters() if isinstance(module, torch.nn.Module) else module
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        self.comm = comm
        self.world = int(getattr(comm, "world"))
        self.rank = int(getattr(comm, "rank"))
        self.device = self.params[0].device
        self.on_gpu = self.device.type == "cuda"
        self.overlap = overlap and self.on_gpu
        self.stream = comm_stream(self.device) if self.on_gpu else None
        self.buckets = self._build(bucket_bytes)
        self.slot_of = {id(p): (b, off) for b in self.buckets for p, off in zip(b.params, b.offsets)}
        self.fused = dict(fused_adamw) if fused_adamw is not None else None
        if self.fused is not None:
            self.fused["grid"] = int(comm_grid)
        self.adamw_states: list[dict] = []
        self._t = 0
        if self.fused is not None:
            if not hasattr(comm, "step_adamw"):
                raise ValueError("fused_adamw needs a communicator with step_adamw (XgmiCommunicator)")
            cap = comm.world * comm.slot_bytes
            for b in self.buckets:
                if b.numel * b.flat_param.element_size() > cap:
                    raise ValueError(f"fused_adamw: bucket of {b.numel} elements exceeds world * slot_bytes = {cap} B")
            self.adamw_states = [comm.adamw_state(b.flat_param) for b in self.buckets]
            # without step_in_backward the fused launch runs in step(); with it, from the hooks
            self.overlap = bool(step_in_backward) and self.on_gpu
            self.optimizer = None
        else:
            if step_in_backward:
                raise ValueError("step_in_backward needs fused_adamw")
            self.optimizer = optimizer_factory([b.shard_param for b in self.buckets])
        self.step_in_backward = self.fused is not None and self.overlap
        self._t_started = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self._next = 0
        self.stats = {"steps": 0, "reduce_scatter_bytes": 0, "all_gather_bytes": 0}

    # ------------------------------------------------------------------ layout
    def _build(self, bucket_bytes: int) -> list[_Bucket]:
        buckets: list[_Bucket] = []
        cur: dict[torch.dtype, _Bucket] = {}
        for p in reversed(self.params):  # backward produces the last layers first
            es = p.element_size()
            align = max(1, _ALIGN_BYTES // es)
            b = cur.get(p.dtype)
            if b is not None and b.numel > 0 and (b.numel + p.numel()) * es > bucket_bytes:
                b = None
            if b is None:
                b = _Bucket(len(buckets), p.dtype)
                buckets.append(b)
                cur[p.dtype] = b
            off = (b.numel + align - 1) // align * align
            b.params.append(p)
            b.offsets.append(off)
            b.numel = off + p.numel()
        for b in buckets:
            es = torch.empty(0, dtype=b.dtype).element_size()
            unit = self.world * max(1, _ALIGN_BYTES // es)  # every shard 16-B sized and aligned
            b.numel = (b.numel + unit - 1) // unit * unit
            b.flat_param = torch.zeros(b.numel, dtype=b.dtype, device=self.device)
            b.flat_grad = torch.zeros(b.numel, dtype=b.dtype, device=self.device)
            for p, off in zip(b.params, b.offsets):
                view = b.flat_param[off:off + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
                p.grad = b.flat_grad[off:off + p.numel()].view_as(p)
            s = b.numel // self.world
            b.grad_shard = torch.zeros(s, dtype=b.dtype, device=self.device)
            shard = torch.nn.Parameter(b.flat_param[self.rank * s:(self.rank + 1) * s], requires_grad=True)
            shard.grad = b.grad_shard
            b.shard_param = shard
            b.pending = len(b.params)
        return buckets

    # ------------------------------------------------------------------ hooks
    def _on_grad(self, p: torch.Tensor) -> None:
        b, off = self.slot_of[id(p)]
        expect = b.flat_grad.data_ptr() + off * b.flat_grad.element_size()
        if p.grad is not None and p.grad.data_ptr() != expect:  # .grad was replaced: fold it back
            view = b.flat_grad[off:off + p.numel()].view_as(p)
            view.copy_(p.grad)
            p.grad = view
        b.pending -= 1
        if b.pending == 0 and self.overlap:
            self._launch_ready()

    def _launch_ready(self, all_: bool = False) -> None:
        while self._next < len(self.buckets) and (all_ or self.buckets[self._next].pending == 0):
            self._reduce(self.buckets[self._next])
            self._next += 1

    def _fused_bucket(self, b: _Bucket) -> None:
        if not self._t_started:  # first bucket of this backward: a new optimizer step
            self._t += 1
            self._t_started = True
        st = self.adamw_states[b.index]
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            self.comm.step_adamw(b.flat_grad, b.flat_param, st, step=self._t, **self.fused)
        b.launched = True
        self.stats["reduce_scatter_bytes"] += b.flat_grad.numel() * b.flat_grad.element_size()
        self.stats["all_gather_bytes"] += b.flat_param.numel() * b.flat_param.element_size()

    def _reduce(self, b: _Bucket) -> None:
        if self.fused is not None:
            self._fused_bucket(b)
            return
        if self.on_gpu:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                self.comm.reduce_scatter(b.flat_grad, b.grad_shard, op="avg")
        else:
            self.comm.reduce_scatter(b.flat_grad, b.grad_shard, op="avg")
        b.launched = True
        self.stats["reduce_scatter_bytes"] += b.flat_grad.numel() * b.flat_grad.element_size()

    # ------------------------------------------------------------------ step API
    def step(self) -> None:
        """Finish the gradient reduce-scatter, update the local shards, all-gather the
        parameters (call after backward)."""
        if self.step_in_backward:
            self._launch_ready(all_=True)  # buckets whose parameters got no gradient
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            for b in self.buckets:
                b.pending = len(b.params)
                b.launched = False
            self._next = 0
            self._t_started = False
            self.stats["steps"] += 1
            return
        if self.fused is not None:
            self._t += 1
            for b, st in zip(self.buckets, self.adamw_states):
                self.comm.step_adamw(b.flat_grad, b.flat_param, st, step=self._t, **self.fused)
                self.stats["reduce_scatter_bytes"] += b.flat_grad.numel() * b.flat_grad.element_size()
                self.stats["all_gather_bytes"] += b.flat_param.numel() * b.flat_param.element_size()
            for b in self.buckets:
                b.pending = len(b.params)
            self.stats["steps"] += 1
            return
        self._launch_ready(all_=True)
        if self.on_gpu:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        self.optimizer.step()
        for b in self.buckets:
            # the shard is part of the gather's output buffer: gather from a copy
            src = b.shard_param.detach().clone()
            self.comm.all_gather(src, b.flat_param)
            self.stats["all_gather_bytes"] += b.flat_param.numel() * b.flat_param.element_size()
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
        self._next = 0
        self.stats["steps"] += 1

    # ------------------------------------------------------------------ checkpoint / resume
    def state_dict(self) -> dict:
        """This rank's shard of the optimizer state, for resume (the reference
        checkpoints nothing; its master restarts at round 0). Parameters are not included -
        every rank holds them in full, so save `module.state_dict()` once. Tensors are
        references, as in `torch.optim.Optimizer.state_dict`; `torch.save` one file per rank
        and reload with `torch.load(..., weights_only=True)`."""
        sd = {"world": self.world, "rank": self.rank, "step": self._t, "steps": self.stats["steps"],
              "layout": [[b.numel, str(b.dtype), len(b.params)] for b in self.buckets]}
        if self.fused is not None:
            sd["adamw"] = [{k: st[k] for k in ("master", "exp_avg", "exp_avg_sq")} for st in self.adamw_states]
        else:
            sd["optimizer"] = self.optimizer.state_dict()
        return sd

    def load_state_dict(self, sd: dict) -> None:
        """Resume from `state_dict()` of the same rank of a run with the same parameters,
        bucket_bytes, world size and optimizer kind."""
        layout = [[b.numel, str(b.dtype), len(b.params)] for b in self.buckets]
        if (sd.get("world"), sd.get("rank")) != (self.world, self.rank):
            raise ValueError(f"checkpoint of rank {sd.get('rank')}/{sd.get('world')}, this is {self.rank}/{self.world}")
        if [list(x) for x in sd.get("layout", [])] != layout:
            raise ValueError("checkpoint bucket layout differs (parameters or bucket_bytes changed)")
        if self.fused is not None:
            if "adamw" not in sd:
                raise ValueError("checkpoint has no fused AdamW state")
            for st, saved in zip(self.adamw_states, sd["adamw"]):
                for k in ("master", "exp_avg", "exp_avg_sq"):
                    if saved[k].shape != st[k].shape:
                        raise ValueError(f"{k}: shape {tuple(saved[k].shape)} != {tuple(st[k].shape)}")
                    st[k].copy_(saved[k])
        else:
            if "optimizer" not in sd:
                raise ValueError("checkpoint has no optimizer state")
            self.optimizer.load_state_dict(sd["optimizer"])
        self._t = int(sd["step"])
        self.stats["steps"] = int(sd["steps"])

    def zero_grad(self) -> None:
        for b in self.buckets:
            b.flat_grad.zero_()

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def describe(self) -> list[dict]:
        return [{"bucket": b.index, "dtype": str(b.dtype), "params": len(b.params), "numel": b.numel,
                 "shard": b.numel // self.world} for b in self.buckets]
