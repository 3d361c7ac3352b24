"""Bucketed, backward-overlapped data-parallel gradient allreduce.

The reference allreduces one flat vector per round, pulled from a `dataSource` and handed
to a `dataSink` (AllreduceWorker.scala:171-192). A trainer's "vector" is its gradient set,
so this module makes the gradients themselves the flat vectors:

* Parameters are grouped into buckets of ~`bucket_bytes` (in reverse registration order,
  which is roughly the order autograd produces gradients). Each bucket owns ONE contiguous
  HBM buffer and every parameter's `.grad` is a view into it (members 16-byte aligned), so
  backward accumulates straight into the buffer that is allreduced - no pack/unpack copy.
* A post-accumulate-grad hook counts ready members; a full bucket is allreduced on a
  dedicated HIP stream while backward keeps running. Buckets are launched strictly in
  bucket order (a later bucket that is ready first waits), so every rank issues the same
  collective sequence - the same "every rank must agree" rule the reference's round
  protocol relies on.
* `wait()` (end of backward) launches any bucket that never became ready (unused
  parameters), then joins the comm stream into the compute stream.
* CU-sliced schedules: an algo label `cuN:<algo>` (e.g. "cu32:twoshot@64") runs the bucket
  allreduces on a comm stream whose kernels may use only N of the GPU's CUs
  (hipExtStreamCreateWithCUMask, spread over every XCD): the collective then occupies a fixed
  slice of the GPU instead of a workgroup on every CU beside backward's GEMMs. With the
  training step on `compute_stream_excluding(device, N)` the split is complete: GEMMs on the
  other CUs only, none of their tiles beside a spinning comm workgroup.
* `overlap="auto"`: the first steps try each candidate schedule - buckets beside backward at
  the communicator's grid, beside backward at 128 workgroups, on a 32-CU slice, all after backward - for
  `tune_steps` steps each, timing first-gradient -> comm joined on the GPU; the ranks agree on
  the fastest (MAX over ranks of each candidate's best step) and keep it. Sharing the GPU with
  backward's GEMMs is not free: on one MI355X the serial schedule won at every grid
  (profiles/round3/README.md, DP overlap at kernel level), while across GPUs the comm is
  link-bound - the measurement decides, per job.

`comm` is anything with `allreduce_(tensor, op=...)` that runs on the current stream:
`XgmiCommunicator` (fused xGMI kernels), or `TorchDistComm` (RCCL / gloo; CPU tests).

Straggler-tolerant steps (`th_reduce` / `th_complete` < 1, the reference's thresholds,
AllreduceWorker.scala:116-145): every bucket is reduced by the threshold kernel
(`XgmiCommunicator.allreduce_threshold`, communicator built with `max_lag`), so a slow rank
delays nobody: its late contributions are left out of this step's sums, and with
`rescale=True` each partial chunk is extrapolated by world / contributors inside the kernel.
"""
from __future__ import annotations

import atexit
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import torch

from .comm import comm_stream

_ALIGN_BYTES = 16

# CU-masked streams this module created and still holds. Those alive at interpreter exit are
# destroyed then, while the HIP runtime is still whole: a masked stream left to the runtime's
# own teardown crashed the process at exit under rocprofv3's library (exit status 139).
_LIVE_MASKED: set[int] = set()
_ATEXIT = [False]


def _masked_stream(device_index: int, cus: int, exclude: bool) -> int:
    from .._native import C

    raw = C.hip.stream_create_cu_mask(device_index, cus, exclude)
    if not _ATEXIT[0]:
        atexit.register(_destroy_live_masked)
        _ATEXIT[0] = True
    _LIVE_MASKED.add(raw)
    return raw


def _release_masked(raw: int) -> None:
    if raw in _LIVE_MASKED:
        _LIVE_MASKED.discard(raw)
        from .._native import C

        C.hip.stream_destroy(raw)


def _destroy_live_masked() -> None:
    for raw in list(_LIVE_MASKED):
        try:
            _release_masked(raw)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def compute_stream_excluding(device, cus: int) -> "torch.cuda.ExternalStream":
    """A stream on every CU of `device` except the `cus` CUs a "cuN:" comm schedule uses (the
    same spread-out selection, csrc/hip/hip_bind.cc stream_create_cu_mask): run forward and
    backward under `with torch.cuda.stream(s):` and the GEMMs never share a CU with the
    overlapped collective - a GEMM otherwise waits for its slowest tile, and a tile on a CU
    beside a spinning comm workgroup is slow. The stream lives as long as the process."""
    dev = torch.device(device)
    raw = _masked_stream(dev.index if dev.index is not None else torch.cuda.current_device(), cus, True)
    return torch.cuda.ExternalStream(raw, device=dev)


class TorchDistComm:
    """Adapter: torch.distributed all_reduce (RCCL on GPU, gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum", algo: str | None = None) -> torch.Tensor:
        import torch.distributed as dist

        dist.all_reduce(t, group=self.group)
        if op == "avg":
            t.div_(self.world)
        return t

    def reduce_scatter(self, inp: torch.Tensor, out: torch.Tensor, *, op: str = "sum") -> torch.Tensor:
        import torch.distributed as dist

        dist.reduce_scatter_tensor(out, inp, group=self.group)
        if op == "avg":
            out.div_(self.world)
        return out

    def all_gather(self, inp: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        import torch.distributed as dist

        dist.all_gather_into_tensor(out, inp, group=self.group)
        return out


@dataclass
class GradBucket:
    index: int
    dtype: torch.dtype
    params: list = field(default_factory=list)
    offsets: list = field(default_factory=list)
    numel: int = 0
    buffer: torch.Tensor | None = None
    pending: int = 0
    ready: bool = False
    launched: bool = False
    done: object = None  # torch.cuda.Event

    @property
    def nbytes(self) -> int:
        return self.numel * torch.empty(0, dtype=self.dtype).element_size()


class BucketedGradReducer:
    def __init__(self, params: Iterable[torch.nn.Parameter] | torch.nn.Module, comm, *,
                 bucket_bytes: int = 64 << 20, op: str = "avg", overlap: bool = True,
                 first_bucket_bytes: int | None = None, sync: str = "native", event_scope: int = 1,
                 th_reduce: float = 1.0, th_complete: float = 1.0, rescale: bool = False, algo: str = "auto",
                 tune_steps: int = 2, schedule_candidates: Sequence[tuple[bool, str]] | None = None):
        """sync: how the comm stream is ordered after backward's gradient writes -
        "native" = reusable HIP events created with `event_scope` (1: device-scope release,
        enough within one GPU; 0: HIP default system-scope), "torch" = torch.cuda events.
        th_reduce / th_complete < 1 (or rescale): threshold rounds per bucket (module doc).
        algo: the communicator's algorithm label per bucket, e.g. "twoshot@128": a bucket
        reduced while backward still runs competes with it for CUs, and fewer persistent
        workgroups leave more of the GPU to the GEMMs (default: the tuned / built-in choice)."""
        self._masked: dict[int, tuple[int, object]] = {}  # CUs -> (raw masked stream, torch ExternalStream)
        self._cus = 0
        self.algo = algo
        self.threshold = th_reduce < 1.0 or th_complete < 1.0 or rescale
        self.th = (float(th_reduce), float(th_complete), bool(rescale))
        if self.threshold and not hasattr(comm, "allreduce_threshold"):
            raise ValueError("threshold rounds need a communicator with allreduce_threshold (XgmiCommunicator)")
        if isinstance(params, torch.nn.Module):
            params = params.parameters()
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        self.comm = comm
        self.op = op
        self.device = self.params[0].device
        self.on_gpu = self.device.type == "cuda"
        # overlap="auto": schedule tuning (module doc); candidates are (overlap, algo label)
        self._auto = False
        self._ev0 = self._ev1 = None
        self.schedule = ("overlap" if overlap and overlap != "auto" and self.on_gpu else "serial", algo)
        self.overlap = bool(overlap) and overlap != "auto" and self.on_gpu
        if overlap == "auto" and self.on_gpu and not self.threshold:
            self.tune_schedule(tune_steps, schedule_candidates)
        self.stream = comm_stream(self.device) if self.on_gpu else None
        self.sync = sync if self.on_gpu else "none"
        self.buckets = self._build(bucket_bytes, first_bucket_bytes)
        if self.threshold:
            cap = getattr(comm, "world", 1) * getattr(comm, "slot_bytes", 0)
            big = [b.nbytes for b in self.buckets if b.nbytes > cap]
            if big:
                raise ValueError(f"threshold rounds need buckets <= world * slot_bytes = {cap} B (largest {max(big)})")
        self._events: list[int] = []
        if self.sync == "native":
            from .._native import C

            self._H = C.hip
            # one compute->comm event per bucket + one comm->compute event
            self._events = [self._H.event_create(event_scope) for _ in range(len(self.buckets) + 1)]
        # per parameter: (bucket, offset, address its .grad view must have) - the hook runs
        # once per parameter per step, so it does one data_ptr() call and no arithmetic
        self.slot_of: dict[int, tuple[GradBucket, int, int]] = {}
        for b in self.buckets:
            es = b.buffer.element_size()
            for p, off in zip(b.params, b.offsets):
                self.slot_of[id(p)] = (b, off, b.buffer.data_ptr() + off * es)
        # raw stream handles: a bucket hand-off enters no torch stream context
        from .comm import _current_stream

        self._cur_stream = _current_stream
        self._dev_index = self.device.index if self.on_gpu else -1
        self._comm_raw = self.stream.cuda_stream if self.stream is not None else None
        self._base_stream = (self.stream, self._comm_raw)
        self._set_algo(self.label)  # a "cuN:" schedule chosen before the streams existed
        # communicators that take a raw `stream=` argument (XgmiCommunicator) skip the context
        self._raw_ok = self.on_gpu and bool(getattr(comm, "accepts_stream", False))
        self._next = 0
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad_ready) for p in self.params]
        self.stats = {"steps": 0, "buckets_launched": 0, "bytes": 0}

    # ------------------------------------------------------------------ CU slices
    def _set_algo(self, label: str) -> None:
        """Adopt an algo label: "cuN:<algo>" = <algo> on a comm stream restricted to N CUs."""
        cus, algo = 0, label
        if isinstance(label, str) and label.startswith("cu") and ":" in label:
            head, algo = label.split(":", 1)
            cus = int(head[2:])
        self.algo = algo
        if not self.on_gpu or getattr(self, "_base_stream", None) is None:
            self._cus = cus
            return
        if cus == self._cus and (cus == 0 or cus in self._masked):
            return
        if cus:
            if cus not in self._masked:
                raw = _masked_stream(self.device.index, cus, False)
                self._masked[cus] = (raw, torch.cuda.ExternalStream(raw, device=self.device))
            raw, ext = self._masked[cus]
            prev_raw = self._comm_raw
            self.stream, self._comm_raw = ext, raw
            # buckets of the previous stream finish first (the communicator also orders its
            # launches across streams, XgmiComm::order_after_last)
            if prev_raw is not None and prev_raw != raw:
                self.stream.wait_stream(torch.cuda.ExternalStream(prev_raw, device=self.device))
        else:
            self.stream, self._comm_raw = self._base_stream
        self._cus = cus

    @property
    def label(self) -> str:
        return f"cu{self._cus}:{self.algo}" if self._cus else self.algo

    # ------------------------------------------------------------------ layout
    def _build(self, bucket_bytes: int, first_bucket_bytes: int | None) -> list[GradBucket]:
        buckets: list[GradBucket] = []
        cur: dict[torch.dtype, GradBucket] = {}
        limit_first = first_bucket_bytes or bucket_bytes
        for p in reversed(self.params):  # backward produces late layers first
            es = p.element_size()
            align = max(1, _ALIGN_BYTES // es)
            b = cur.get(p.dtype)
            cap = limit_first if not buckets else bucket_bytes
            if b is not None and b.numel > 0 and (b.numel + p.numel()) * es > cap:
                b = None
            if b is None:
                b = GradBucket(index=len(buckets), dtype=p.dtype)
                buckets.append(b)
                cur[p.dtype] = b
            off = (b.numel + align - 1) // align * align
            b.params.append(p)
            b.offsets.append(off)
            b.numel = off + p.numel()
        for b in buckets:
            es = torch.empty(0, dtype=b.dtype).element_size()
            align = max(1, _ALIGN_BYTES // es)
            b.numel = (b.numel + align - 1) // align * align
            b.buffer = torch.zeros(b.numel, dtype=b.dtype, device=self.device)
            for p, off in zip(b.params, b.offsets):
                g = b.buffer[off:off + p.numel()].view_as(p)
                if p.grad is not None:
                    g.copy_(p.grad)
                p.grad = g  # gradient-as-bucket-view: autograd accumulates in place
            b.pending = len(b.params)
        return buckets

    # ------------------------------------------------------------------ hooks
    def _on_grad_ready(self, p: torch.Tensor) -> None:
        if self._auto and self._ev0 is None:  # first gradient of a tuning step
            self._ev0 = torch.cuda.Event(enable_timing=True)
            self._ev0.record()
        b, off, expect = self.slot_of[id(p)]
        g = p.grad
        if g is not None and g.data_ptr() != expect:
            # .grad was replaced (e.g. zero_grad(set_to_none=True)): fold it back into the
            # bucket view - one copy; use reducer.zero_grad() to avoid it
            view = b.buffer[off:off + p.numel()].view_as(p)
            view.copy_(p.grad)
            p.grad = view
        b.pending -= 1
        if b.pending == 0:
            b.ready = True
            if self.overlap:
                self._launch_ready()

    def _launch_ready(self) -> None:
        while self._next < len(self.buckets) and self.buckets[self._next].ready:
            self._launch(self.buckets[self._next])
            self._next += 1

    def _reduce(self, b: GradBucket) -> None:
        if self.threshold:
            thr, thc, rescale = self.th
            self.comm.allreduce_threshold(b.buffer, b.buffer, th_reduce=thr, th_complete=thc, op=self.op,
                                          rescale=rescale)
        elif self.algo != "auto":
            self.comm.allreduce_(b.buffer, op=self.op, algo=self.algo)
        else:
            self.comm.allreduce_(b.buffer, op=self.op)

    def _launch(self, b: GradBucket) -> None:
        if self.sync == "native":
            cs = self._cur_stream(self._dev_index)
            ev = self._events[b.index]
            self._H.event_record(ev, cs)
            self._H.stream_wait_event(self._comm_raw, ev)
            if self._raw_ok and not self.threshold:  # straight onto the comm stream
                self.comm.allreduce_(b.buffer, op=self.op, algo=self.algo, stream=self._comm_raw)
            else:
                with torch.cuda.stream(self.stream):
                    self._reduce(b)
            b.done = True
        elif self.on_gpu:
            compute = torch.cuda.current_stream(self.device)
            self.stream.wait_stream(compute)
            with torch.cuda.stream(self.stream):
                self._reduce(b)
                b.done = torch.cuda.Event()
                b.done.record(self.stream)
        else:
            self._reduce(b)
        b.launched = True
        self.stats["buckets_launched"] += 1
        self.stats["bytes"] += b.nbytes

    # ------------------------------------------------------------------ step API
    def wait(self) -> None:
        """Finish the gradient allreduce of this step (call after backward, before the
        optimizer). Buckets whose parameters got no gradient are reduced too (as zeros)."""
        for b in self.buckets:
            b.ready = True
        self._launch_ready()
        # the comm stream runs the buckets in order: joining after the last one is enough
        if self.sync == "native":
            ev = self._events[-1]
            self._H.event_record(ev, self._comm_raw)
            self._H.stream_wait_event(self._cur_stream(self._dev_index), ev)
        elif self.on_gpu:
            last = [b for b in self.buckets if b.done is not None]
            if last:
                torch.cuda.current_stream(self.device).wait_event(last[-1].done)
        for b in self.buckets:
            b.pending = len(b.params)
            b.ready = b.launched = False
            b.done = None
        self._next = 0
        self.stats["steps"] += 1
        if self._auto:
            self._tune_step()

    def _agree(self, times: Sequence[float]) -> tuple[int, torch.Tensor]:
        """The schedule every rank keeps: per candidate the MAX over ranks of its best step time
        (a schedule is as fast as its slowest rank), then the fastest candidate - the same
        index on every rank (ties: the first)."""
        best = torch.tensor(list(times), dtype=torch.float64)
        import torch.distributed as dist

        # Only a job without a process group decides alone. With one, a failing MAX reduce
        # must raise: ranks keeping different schedules would launch different kernels.
        if dist.is_available() and dist.is_initialized():
            grp = getattr(self.comm, "cpu_group", None)
            if grp is not None or not self.on_gpu:  # a gloo group: a CPU tensor
                dist.all_reduce(best, op=dist.ReduceOp.MAX, group=grp if grp is not None else
                                getattr(self.comm, "group", None))
            else:
                t = best.to(self.device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=getattr(self.comm, "group", None))
                best = t.cpu()
        return int(torch.argmin(best).item()), best

    def tune_schedule(self, tune_steps: int = 2, candidates: Sequence[tuple[bool, str]] | None = None) -> None:
        """(Re)start schedule tuning: the next len(candidates) x tune_steps steps try each
        (overlap, algo) candidate; then the fastest (agreed over the ranks) is kept."""
        if not self.on_gpu or self.threshold:
            return
        xgmi = bool(getattr(self.comm, "accepts_stream", False))
        base = self.schedule[1] if self.schedule else self.label
        default = ([(True, base), (True, "twoshot@128"), (True, "cu32:twoshot@64"), (False, base)] if xgmi
                   else [(True, base), (False, base)])
        if xgmi and getattr(self.comm, "world", 1) > 1 and getattr(type(self.comm), "sdma", None) is not None \
                and candidates is None:
            # the copy-engine allreduce leaves the CUs to backward's GEMMs; created here, on
            # every rank at the same step (its construction is collective)
            try:
                self.comm.sdma
                default.append((True, "sdma"))
            except Exception:  # noqa: BLE001 - no SDMA engines: the CU schedules only
                pass
        self._cands = list(candidates or default)
        self._tune_steps = max(1, int(tune_steps))
        self._times: list[list[float]] = [[] for _ in self._cands]
        self._step_i = 0
        self._ev0 = self._ev1 = None
        self.overlap = self._cands[0][0]
        self._set_algo(self._cands[0][1])
        self.schedule = None
        self._auto = True

    def _tune_step(self) -> None:
        """One step of schedule tuning (overlap="auto"): time it, move to the next candidate,
        and after the last one agree on the fastest over the ranks and keep it."""
        if self._ev0 is not None:
            self._ev1 = torch.cuda.Event(enable_timing=True)
            self._ev1.record()
            self._ev1.synchronize()  # tuning steps only: the CPU waits for this step's comm
            self._times[self._step_i // self._tune_steps].append(self._ev0.elapsed_time(self._ev1))
        self._ev0 = None
        self._step_i += 1
        k = self._step_i // self._tune_steps
        if k < len(self._cands):
            self.overlap = self._cands[k][0]
            self._set_algo(self._cands[k][1])
            return
        i, best = self._agree([min(t) if t else float("inf") for t in self._times])
        self.overlap = self._cands[i][0]
        self._set_algo(self._cands[i][1])
        self.schedule = ("overlap" if self.overlap else "serial", self.label)
        self.stats["schedule_ms"] = {f"{'overlap' if o else 'serial'}:{a}": round(float(x), 3)
                                     for (o, a), x in zip(self._cands, best.tolist())}
        self.stats["schedule"] = f"{self.schedule[0]}:{self.schedule[1]}"
        self._auto = False

    def zero_grad(self) -> None:
        for b in self.buckets:
            b.buffer.zero_()

    def __del__(self):
        for e in getattr(self, "_events", []):
            try:
                self._H.event_destroy(e)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass
        self._events = []
        for raw, _ in getattr(self, "_masked", {}).values():
            try:
                _release_masked(raw)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass
        self._masked = {}

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def describe(self) -> list[dict]:
        return [{"bucket": b.index, "dtype": str(b.dtype), "params": len(b.params), "bytes": b.nbytes}
                for b in self.buckets]


def bucket_sizes(shapes: Sequence[tuple[int, ...]], elem_bytes: int, bucket_bytes: int) -> list[int]:
    """Bucket byte sizes the reducer would build for parameter `shapes` (reverse order)."""
    sizes, cur = [], 0
    align = max(1, _ALIGN_BYTES // elem_bytes)
    for shp in reversed(list(shapes)):
        n = 1
        for d in shp:
            n *= d
        if cur > 0 and (cur + n) * elem_bytes > bucket_bytes:
            sizes.append((cur + align - 1) // align * align * elem_bytes)
            cur = 0
        cur = (cur + align - 1) // align * align + n
    if cur:
        sizes.append((cur + align - 1) // align * align * elem_bytes)
    return sizes
