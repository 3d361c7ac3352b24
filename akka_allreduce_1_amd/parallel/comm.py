"""Communicators over the xGMI data plane (`csrc/hip/xgmi_comm.*`).

`XgmiCommunicator` - one process per GPU (torchrun / torch.distributed). Rendezvous and the
    exchange of IPC handles go over a CPU (gloo) group; the data moves in ONE fused HIP
    launch per segment: direct push reduce-scatter + direct push all-gather over the xGMI
    mesh (the reference's ScatterBlock/ReduceBlock pattern, AllreduceWorker.scala:194-238),
    or a one-shot push + local reduce for small tensors. RCCL (`backend="nccl"`) stays
    reachable as `algo="rccl"` for comparison and for dtypes the kernels do not cover.
`LocalCluster` - P logical ranks inside ONE process (one or several GPUs): the same kernels,
    consecutive ranks of one device in ONE launch. This is how the multi-rank protocol is run on a
    single MI355X and what `tests/test_comm_gpu.py` checks.

Reduction semantics: fp32 accumulation in rank order 0..P-1, one rounding to the output
dtype (bf16 sums are never accumulated in bf16 - MI355X_MICROARCH.md, global float atomics).
"""
from __future__ import annotations

import os
import socket
from typing import Sequence

import torch

from .._native import C
from ..algos import LIBRARY_ALGOS, LOSSY_ALGOS  # noqa: F401 - one definition (algos.py)

_H = C.hip

ALGOS = {"auto": _H.Algo.Auto, "twoshot": _H.Algo.TwoShot, "oneshot": _H.Algo.OneShot, "ring": _H.Algo.Ring,
         "ll": _H.Algo.LL, "ring_native": _H.Algo.RingNative}
DEFAULT_SLOT_BYTES = int(os.environ.get("MXAR_SLOT_BYTES", 64 << 20))


class CommError(RuntimeError):
    """A device-side wait timed out (a peer never delivered); the communicator is poisoned."""


_ERR_NAMES = {1: "scatter wait timed out", 2: "reduce wait timed out", 4: "barrier / slot-reuse wait timed out", 8: "bad arguments",
              16: "a peer stayed more than maxLag rounds behind"}


def _describe(err: int) -> str:
    return ", ".join(v for k, v in _ERR_NAMES.items() if err & k) or f"code {err}"


def _dtype_code(dt: torch.dtype):
    from ..ops.kernels import dtype_code

    return dtype_code(dt)


_KERNEL_DTYPES = {torch.float32: _H.DType.F32, torch.bfloat16: _H.DType.BF16, torch.float16: _H.DType.F16}
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _current_stream(device_index: int) -> int:
    """Raw handle of the current HIP stream of `device_index` (torch's own fast accessor when
    present, ~10x cheaper than torch.cuda.current_stream(...).cuda_stream)."""
    if _raw_stream is not None:
        return _raw_stream(device_index)
    return torch.cuda.current_stream(device_index).cuda_stream


def comm_stream(device) -> "torch.cuda.Stream":
    """Side stream for collectives overlapped with compute (gradient buckets, fused optimizer
    steps). High priority on purpose: HIP hands out hardware queues to streams round-robin
    within a priority level (GPU_MAX_HW_QUEUES per process), so a normal-priority side stream
    can share the compute stream's queue - its kernels then run strictly in order with the
    GEMMs and nothing overlaps (seen in a rocprofv3 kernel trace: both streams on one
    Queue_Id). A high-priority stream is served from a queue of its own, and the dispatcher
    favours it, so a persistent collective's workgroups become resident next to the GEMMs."""
    return torch.cuda.Stream(device=device, priority=-1)


def free_port() -> int:
    """A bindable port BELOW the kernel's ephemeral range. A port the kernel hands out for
    bind(0) is also what gloo's own pair connections draw from, so a rendezvous on it can
    lose the port to another job's connection before the store listens (EADDRINUSE)."""
    import random

    lo = 20000
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            eph = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        eph = 32768
    hi = max(lo + 1000, eph - 1)
    rng = random.Random()
    for _ in range(64):
        port = rng.randrange(lo, hi)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init_distributed(backend: str = "nccl") -> tuple[int, int, int]:
    """Initialise torch.distributed from torchrun's env (or as a 1-rank job on 127.0.0.1).

    Returns (rank, world_size, local_rank) and binds the process to cuda:local_rank.
    """
    import torch.distributed as dist

    if "RANK" not in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend == "nccl" and torch.cuda.is_available():
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl" and torch.cuda.is_available():
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


class XgmiCommunicator:
    """Allreduce over directly mapped peer HBM for the ranks of a torch.distributed group."""

    accepts_stream = True  # allreduce(..., stream=<raw hipStream_t>) (the DP reducer uses it)

    def __init__(self, group=None, *, device: torch.device | int | None = None, slot_bytes: int | None = None,
                 grid: int = 0, timeout_s: float = 20.0, cpu_group=None, max_lag: int | None = None):
        """max_lag: enables `allreduce_threshold`, whose ranks may run up to max_lag rounds
        ahead of the slowest peer (a lag ring of max_lag + 1 extra slot rows in the slab)."""
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("XgmiCommunicator needs torch.distributed (see init_distributed)")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.slot_bytes = int(slot_bytes or DEFAULT_SLOT_BYTES)
        if cpu_group is None:
            backend = dist.get_backend(group)
            cpu_group = group if backend == "gloo" else dist.new_group(
                ranks=None if group is None else dist.get_process_group_ranks(group), backend="gloo")
        self.cpu_group = cpu_group
        # Every step that can fail locally is followed by an all-gather of its status, so a
        # failure on one rank raises on every rank instead of leaving the others blocked in
        # the next collective.
        self._c, handle, err = None, None, ""
        try:
            self._c = _H.XgmiComm(self.rank, self.world, self.device.index, self.slot_bytes, grid, timeout_s,
                                  0 if max_lag is None else max_lag + 1)
            handle = self._c.ipc_handle()
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {e}"
        handles: list = [None] * self.world
        dist.all_gather_object(handles, (handle, err), group=cpu_group)
        errs = [e for _, e in handles if e]
        if errs:
            raise CommError("XgmiCommunicator setup failed: " + "; ".join(errs))
        try:
            self._c.connect([h for h, _ in handles])
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {e}"
        status: list = [None] * self.world
        dist.all_gather_object(status, err, group=cpu_group)
        errs = [e for e in status if e]
        if errs:
            raise CommError("XgmiCommunicator connect failed: " + "; ".join(errs))
        self.table: list[tuple[int, str]] = []  # (max bytes, algo) from tune(); empty = built-in policy
        self._default_grid = self._c.grid
        self._grid = self._c.grid
        self._default_sized = bool(self._c.size_grid)  # launch-size grids (MXAR_SIZE_GRID)
        self._sized = self._default_sized
        self._default_units = self._units = self._c.units_per_wg  # MXAR_TWOSHOT_UNITS or 0 (by size)
        self._dev = self.device.index
        self._launch: dict[str, tuple] = {}  # algo label -> (native Algo, grid, units, launch-size grid)
        self._p2p = None
        self._sdma = None
        self._sdma_error: CommError | None = None

    @property
    def sdma(self):
        """The same ranks' SDMA allreduce (parallel/sdma.py: cross-rank copies on the copy
        engines), created on first use - collectively: every rank must reach it together
        (BucketedGradReducer.tune_schedule does)."""
        if self._sdma is None:
            if self._sdma_error is not None:  # failed before on every rank: not tried again
                raise self._sdma_error
            from .sdma import SdmaCommunicator

            try:
                self._sdma = SdmaCommunicator(self.group, device=self.device, slot_bytes=self.slot_bytes,
                                              cpu_group=self.cpu_group)
            except CommError as e:  # collective: every rank raised the same
                self._sdma_error = e
                raise
        return self._sdma

    @property
    def p2p(self):
        """The reference protocol over RCCL point-to-point (parallel/p2p.py), created lazily."""
        if self._p2p is None:
            from .p2p import P2PCommunicator

            self._p2p = P2PCommunicator(self.group, chunk_bytes=self.slot_bytes)
        return self._p2p

    # ------------------------------------------------------------------ tuning
    def tune(self, max_bytes: int = 256 << 20, dtype: torch.dtype = torch.bfloat16, iters: int = 10,
             candidates: Sequence[str] = ("oneshot", "twoshot", "rccl"), min_bytes: int = 4 << 10,
             grids: Sequence[int] = (), grid_min_bytes: int = 1 << 20, exact_only: bool = True) -> list[dict]:
        """Measure p50 latency of every algorithm per power-of-4 size class in
        [min_bytes, max_bytes] and keep the fastest per class (the slowest rank's p50
        decides; rank 0's choice is broadcast so every rank dispatches identically - a split
        decision would deadlock). `grids`: extra workgroup counts tried for twoshot / ring at
        sizes >= grid_min_bytes (labels "twoshot@256"); only counts <= the default grid, so
        every workgroup stays resident. Where the two-shot picks its flat geometry (blocks of
        >= 2 MiB: one chunk per workgroup, grouped scatter), the coarse one is tried too
        ("twoshot~1", "twoshot@256~1": one scatter unit per workgroup): on one GPU flat wins
        by up to 22 % at 8 ranks, over xGMI links the measured choice decides. `exact_only`: the
        per-hop-rounded kernels (LOSSY_ALGOS) are timed but never adopted. Returns one row per
        size: {bytes, <algo>_p50_us, choice}."""
        import torch.distributed as dist

        from ..ops import fill_uniform
        from ..utils.timing import percentile

        es = torch.empty(0, dtype=dtype).element_size()
        x = fill_uniform(torch.empty(max_bytes // es, dtype=dtype, device=self.device), seed=self.rank)
        y = torch.empty_like(x)
        src0 = 0 if self.cpu_group is None else dist.get_global_rank(self.cpu_group, 0)
        rows, table = [], []
        sizes, size = [], min_bytes
        while size < max_bytes:
            sizes.append(size)
            size *= 4
        sizes.append(max_bytes)
        extra = [g for g in grids if 0 < g < self._default_grid]
        for size in sizes:
            n = size // es
            best, best_t, row = None, float("inf"), {"bytes": size}
            labels = []
            for algo in candidates:
                labels.append(algo)
                if algo in ("twoshot", "ring", "ring_native") and size >= grid_min_bytes:
                    labels += [f"{algo}@{g}" for g in extra]
                    if algo == "twoshot" and grids and self._default_sized:
                        # the default grid sizes itself by the launch's bytes; the full grid too,
                        # so a link-bound xGMI launch can still pick it
                        labels.append("twoshot@full")
                if algo == "twoshot" and self.world > 2 and self._default_units == 0 and size // self.world >= (2 << 20):
                    labels += ["twoshot~1"] + [f"twoshot@{g}~1" for g in extra]
            for algo in labels:
                if algo == "oneshot" and (size > self.slot_bytes or size > (8 << 20)):
                    continue
                if algo == "ll" and size > self._c.ll_max_bytes:
                    continue
                if algo == "threshold" and not self._threshold_fits(x[:size // es]):
                    continue
                if algo == "rccl" and dist.get_backend(self.group) != "nccl":
                    continue
                a, b = x[:n], y[:n]
                for _ in range(2):
                    self.allreduce(a, b, algo=algo)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(iters)]
                torch.cuda.synchronize(self.device)
                for e0, e1 in evs:
                    e0.record()
                    self.allreduce(a, b, algo=algo)
                    e1.record()
                torch.cuda.synchronize(self.device)
                p50 = percentile([e0.elapsed_time(e1) for e0, e1 in evs], 50)
                t = torch.tensor([p50], device=self.device, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                row[f"{algo}_p50_us"] = round(t.item() * 1e3, 2)
                row[f"{algo}_algbw"] = round(size / (t.item() / 1e3) / 1e9, 2)
                # library paths are comparison columns: the table only ever holds this
                # framework's kernels (a split of RCCL vs xGMI is reported, never adopted)
                base = algo.split("@")[0].split("~")[0]
                if (algo not in LIBRARY_ALGOS and not (exact_only and base in LOSSY_ALGOS)
                        and t.item() < best_t):
                    best, best_t = algo, t.item()
            if best is None:  # only library candidates were given: keep the built-in policy
                best = "auto"
            if "rccl_p50_us" in row and best != "auto":
                row["speedup_vs_rccl"] = round(row["rccl_p50_us"] / row[f"{best}_p50_us"], 3)
            choice = [best]
            dist.broadcast_object_list(choice, src=src0, group=self.cpu_group)
            row["choice"] = choice[0]
            rows.append(row)
            table.append((size, choice[0]))
        self.check()
        self.table = table
        return rows

    def _pick(self, nbytes: int) -> str:
        """The tuned kernel label for a message of `nbytes` ("auto" = built-in size policy).
        Never a library path: tune() does not adopt them, and a hand-set table entry naming
        one is ignored here too."""
        for limit, algo in self.table:
            if nbytes <= limit:
                return "auto" if algo.split("@")[0] in LIBRARY_ALGOS else algo
        tail = [a for _, a in self.table if a.split("@")[0] not in LIBRARY_ALGOS]
        return tail[-1] if tail else "auto"

    # ------------------------------------------------------------------ collectives
    def allreduce(self, inp: torch.Tensor, out: torch.Tensor | None = None, *, op: str = "sum",
                  algo: str = "auto", stream: int | None = None) -> torch.Tensor:
        """out = sum (or mean) over ranks of inp. `out=inp` gives an in-place allreduce.
        `stream`: raw HIP stream handle to enqueue on (default: torch's current stream) - the
        DP reducer passes its comm stream without entering a torch stream context.

        The kernel path costs a few microseconds of host time per call (tools/host_overhead.py):
        integer device checks, a cached (Algo, grid) per algorithm label, the raw current-stream
        handle, no per-call imports."""
        if out is None:
            out = torch.empty_like(inp)
        if inp.get_device() != self._dev or out.get_device() != self._dev:
            raise ValueError(f"tensors must live on {self.device}")
        if not (inp.is_contiguous() and out.is_contiguous()) or inp.numel() != out.numel() or inp.dtype != out.dtype:
            raise ValueError("inp/out must be contiguous with the same numel and dtype")
        if op != "sum" and op != "avg":
            raise ValueError(f"unsupported op {op!r}")
        if algo == "auto" and self.table:
            algo = self._pick(inp.numel() * inp.element_size())
        code = _KERNEL_DTYPES.get(inp.dtype)
        launch = self._launch.get(algo) if code is not None else None
        if launch is not None:  # the mean is fused into the kernel (scale applied to the fp32 sum)
            kind, grid, units, sized = launch
            if self._grid != grid:
                self._c.grid = grid
                self._grid = grid
            if self._sized != sized:  # "algo@full": the full grid at every size
                self._c.size_grid = sized
                self._sized = sized
            if self._units != units:  # two-shot geometry: scatter units per workgroup (0 = by size)
                self._c.units_per_wg = units
                self._units = units
            self._c.allreduce(inp.data_ptr(), out.data_ptr(), inp.numel(), code,
                              _current_stream(self._dev) if stream is None else stream, kind,
                              1.0 / self.world if op == "avg" else 1.0)
        elif algo == "sdma":  # copy-engine transfers (parallel/sdma.py); the mean fused into its reduce
            return self.sdma.allreduce(inp, out, op=op, stream=stream)
        elif algo == "threshold" and self._threshold_fits(inp):
            # the straggler-tolerant kernel at th = 1 is an exact allreduce with its own
            # geometry (one chunk per workgroup, round-robin gather); a tune() candidate
            self.allreduce_threshold(inp, out, op=op, stream=stream)
        elif algo in ("p2p", "rsag", "rccl") or code is None:
            # library paths enqueue on torch's current stream: make it the caller's stream,
            # so a DP reducer's bucket still overlaps with compute (no raw-stream argument)
            with self._on_stream(stream):
                if algo in ("p2p", "rsag"):  # the same protocol over RCCL point-to-point / RS+AG
                    self.p2p.allreduce(inp, out, op=op, algo=algo)
                else:
                    import torch.distributed as dist

                    if out.data_ptr() != inp.data_ptr():
                        out.copy_(inp)
                    dist.all_reduce(out, group=self.group)
                    if op == "avg":
                        out.div_(self.world)
        else:
            # "twoshot@256": workgroup count chosen by tune(); "twoshot@256~1": and one scatter
            # unit per workgroup (coarse chunks) instead of the size-based geometry
            # "twoshot@full": the default grid without launch-size sizing
            label, _, u = algo.partition("~")
            name, _, g = label.partition("@")
            if name == "threshold":  # no lag ring, or too large for one launch
                return self.allreduce(inp, out, op=op, algo="twoshot", stream=stream)
            if name not in ALGOS:
                raise ValueError(f"unknown algo {algo!r}")
            full = g == "full"
            self._launch[algo] = (ALGOS[name], int(g) if g and not full else self._default_grid,
                                  int(u) if u else self._default_units, self._default_sized and not full)
            return self.allreduce(inp, out, op=op, algo=algo, stream=stream)
        return out

    def _on_stream(self, stream: int | None):
        """Context making the raw HIP stream `stream` torch's current stream (no-op for None)."""
        import contextlib

        if stream is None:
            return contextlib.nullcontext()
        return torch.cuda.stream(torch.cuda.ExternalStream(stream, device=self.device))

    def allreduce_(self, t: torch.Tensor, *, op: str = "sum", algo: str = "auto",
                   stream: int | None = None) -> torch.Tensor:
        return self.allreduce(t, t, op=op, algo=algo, stream=stream)

    def _threshold_fits(self, t: torch.Tensor) -> bool:
        return (self.world > 1 and self._c.threshold_rows > 0 and t.dtype in _KERNEL_DTYPES
                and t.numel() * t.element_size() <= self.world * self.slot_bytes)

    def allreduce_threshold(self, inp: torch.Tensor, out: torch.Tensor | None = None, *, th_reduce: float = 1.0,
                            th_complete: float = 1.0, counts: bool = False, op: str = "sum", rescale: bool = False,
                            stream: int | None = None):
        """Straggler-tolerant allreduce round (the reference's thReduce / thComplete / maxLag
        semantics, csrc/hip/xgmi_threshold.hip). Returns `out`, or `(out, counts)` with
        counts an int32 [world, nch] tensor: contributions summed per output chunk (0 = the
        chunk was given up and is zero). The tensor must fit one launch (<= world * slot).
        op="avg" divides by world; rescale=True extrapolates a chunk summed from cnt < world
        contributions by world / cnt inside the kernel (with avg: the mean over the ranks
        that contributed) - the reference leaves partial sums unscaled."""
        if op not in ("sum", "avg"):
            raise ValueError(f"unsupported op {op!r}")
        if out is None:
            out = torch.empty_like(inp)
        if inp.device != self.device or out.device != self.device or inp.numel() != out.numel():
            raise ValueError(f"inp/out must live on {self.device} with the same numel")
        if not (inp.is_contiguous() and out.is_contiguous()) or inp.dtype != out.dtype:
            raise ValueError("inp/out must be contiguous with the same dtype")
        code = _dtype_code(inp.dtype)
        cnt = None
        if counts:
            cnt = torch.zeros(self.world, self._c.threshold_chunks(inp.numel(), code), dtype=torch.int32,
                              device=self.device)
        self._c.allreduce_threshold(inp.data_ptr(), out.data_ptr(), inp.numel(), code,
                                    _current_stream(self._dev) if stream is None else stream, th_reduce, th_complete,
                                    0 if cnt is None else cnt.data_ptr(), 1.0 / self.world if op == "avg" else 1.0,
                                    rescale)
        return (out, cnt) if counts else out

    # ------------------------------------------------------------------ other collectives
    def _coll_ok(self, inp: torch.Tensor, out: torch.Tensor, m: int) -> bool:
        if inp.get_device() != self._dev or out.get_device() != self._dev:
            raise ValueError(f"tensors must live on {self.device}")
        if not (inp.is_contiguous() and out.is_contiguous()) or inp.dtype != out.dtype:
            raise ValueError("inp/out must be contiguous with the same dtype")
        return inp.dtype in _KERNEL_DTYPES and (m * inp.element_size()) % 16 == 0

    def all_to_all(self, inp: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """inp / out: world equal blocks; block s of out on rank r = block r of inp on rank s.
        One xGMI launch (csrc/hip/xgmi_coll.hip); RCCL when the block is not 16-B sized."""
        if out is None:
            out = torch.empty_like(inp)
        if inp.numel() % self.world or out.numel() != inp.numel():
            raise ValueError("all_to_all needs world equal blocks and out.numel() == inp.numel()")
        m = inp.numel() // self.world
        if self._coll_ok(inp, out, m):
            self._c.collective(_H.Coll.AllToAll, inp.data_ptr(), out.data_ptr(), m, _KERNEL_DTYPES[inp.dtype],
                               _current_stream(self._dev))
        else:
            import torch.distributed as dist

            dist.all_to_all_single(out.view(-1), inp.reshape(-1), group=self.group)
        return out

    def all_gather(self, inp: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """out = concatenation over ranks of inp (world x inp.numel())."""
        m = inp.numel()
        if out is None:
            out = torch.empty(self.world * m, dtype=inp.dtype, device=inp.device)
        if out.numel() != self.world * m:
            raise ValueError("all_gather output must hold world x inp.numel() elements")
        if self._coll_ok(inp, out, m):
            self._c.collective(_H.Coll.AllGather, inp.data_ptr(), out.data_ptr(), m, _KERNEL_DTYPES[inp.dtype],
                               _current_stream(self._dev))
        else:
            import torch.distributed as dist

            dist.all_gather_into_tensor(out.view(-1), inp.reshape(-1), group=self.group)
        return out

    def reduce_scatter(self, inp: torch.Tensor, out: torch.Tensor | None = None, *, op: str = "sum") -> torch.Tensor:
        """out (inp.numel() / world elements) on rank r = sum (or mean) over ranks of block r
        of inp; fp32 accumulation in rank order, one rounding."""
        if op not in ("sum", "avg"):
            raise ValueError(f"unsupported op {op!r}")
        if inp.numel() % self.world:
            raise ValueError("reduce_scatter needs world equal blocks")
        m = inp.numel() // self.world
        if out is None:
            out = torch.empty(m, dtype=inp.dtype, device=inp.device)
        if out.numel() != m:
            raise ValueError("reduce_scatter output must hold inp.numel() / world elements")
        if self._coll_ok(inp, out, m):
            self._c.collective(_H.Coll.ReduceScatter, inp.data_ptr(), out.data_ptr(), m, _KERNEL_DTYPES[inp.dtype],
                               _current_stream(self._dev), 1.0 / self.world if op == "avg" else 1.0)
        else:
            import torch.distributed as dist

            dist.reduce_scatter_tensor(out.view(-1), inp.reshape(-1), group=self.group)
            if op == "avg":
                out.div_(self.world)
        return out

    def barrier(self) -> None:
        self._c.barrier(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ health
    def error(self) -> int:
        return int(self._c.error())

    def check(self) -> None:
        """Synchronise and raise CommError if any device-side wait timed out."""
        torch.cuda.synchronize(self.device)
        e = self.error()
        if e:
            raise CommError(f"rank {self.rank}: {_describe(e)} (error word {e:#x}){self._ctl_note()}")

    def _ctl_note(self) -> str:
        """The rank's control words for a failure report: the launch epoch (compare it across
        ranks: every rank runs the same launch sequence), the workgroup ticket (0 between
        launches) and the epochs of the last launches whose S / R reads peers wait for."""
        try:
            w = list(self._c.ctl_words())
        except Exception:  # noqa: BLE001 - diagnostics must not mask the error
            return ""
        note = f"; launch epoch {w[0]}, ticket {w[1]}, reads-done epochs S {w[12]} R {w[13]}"
        return note + (" - ticket not 0 between launches" if w[1] else "")

    def step_adamw(self, grads: torch.Tensor, params: torch.Tensor, state: dict, *, lr: float,
                   betas: tuple[float, float] = (0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                   step: int, op: str = "avg", grid: int = 0) -> torch.Tensor:
        """One fused sharded-DP step (csrc/hip/xgmi_adam.hip): reduce-scatter `grads` (mean by
        default), AdamW on this rank's shard state, all-gather the new `params` (in place,
        identical on every rank) - one launch. `state` = {"master", "exp_avg", "exp_avg_sq"}:
        fp32 tensors of `shard_len(n)` elements holding block `rank` (see `adamw_state`).
        `grid` > 0 overrides the workgroup count (fewer leave CUs to overlapped GEMMs)."""
        if grads.numel() != params.numel() or grads.dtype != params.dtype:
            raise ValueError("grads and params must match in size and dtype")
        g = grid if grid > 0 else self._default_grid
        if self._grid != g:
            self._c.grid = g
            self._grid = g
        if self._sized != self._default_sized:  # an "@full" label must not leak in here
            self._c.size_grid = self._default_sized
            self._sized = self._default_sized
        if self._units != self._default_units:  # a tuned "~1" two-shot label must not leak in here
            self._c.units_per_wg = self._default_units
            self._units = self._default_units
        h = _H.AdamW()
        h.lr, (h.beta1, h.beta2), h.eps, h.weight_decay, h.step = lr, betas, eps, weight_decay, step
        self._c.step_adamw(grads.data_ptr(), params.data_ptr(), params.numel(), _dtype_code(params.dtype),
                           _current_stream(self._dev), state["master"].data_ptr(), state["exp_avg"].data_ptr(),
                           state["exp_avg_sq"].data_ptr(), h, 1.0 / self.world if op == "avg" else 1.0)
        return params

    def shard_len(self, n: int, dtype: torch.dtype) -> int:
        """Elements of the block a rank owns in a fused step over n elements."""
        return self._c.block_elems(n, _dtype_code(dtype))

    def adamw_state(self, params: torch.Tensor) -> dict:
        """Fresh fp32 shard state for `step_adamw`: master = this rank's block of params."""
        b = self.shard_len(params.numel(), params.dtype)
        lo, hi = self.rank * b, min(params.numel(), (self.rank + 1) * b)
        master = torch.zeros(b, dtype=torch.float32, device=self.device)
        if hi > lo:
            master[:hi - lo].copy_(params.view(-1)[lo:hi].float())
        return {"master": master, "exp_avg": torch.zeros_like(master), "exp_avg_sq": torch.zeros_like(master)}

    def reset(self) -> None:
        """Recover after a CommError (a peer missed a deadline): every rank calls this
        collectively. Each rank drains its device, all ranks meet on the CPU group, every rank
        zeroes its flags / LL slots / epoch counters, and all meet again - so no rank can see
        a stale flag of the failed collective, and epochs restart from the same value on every
        rank. The slabs' IPC mappings stay valid."""
        import torch.distributed as dist

        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.cpu_group)
        self._c.reset_local()
        dist.barrier(group=self.cpu_group)

    @property
    def native(self):
        return self._c

    @property
    def stats(self):
        return self._c.stats

    def __repr__(self) -> str:
        return (f"XgmiCommunicator(rank={self.rank}, world={self.world}, device={self.device}, "
                f"slot={self.slot_bytes >> 20} MiB, grid={self._c.grid})")


class LocalCluster:
    """P logical ranks in one process; rank k lives on `devices[k]`.

    Consecutive ranks on the same device are served by ONE launch (blockIdx.y = rank), so
    their spinning workgroups are co-resident by construction; different devices run
    their launches concurrently. `grid` is the workgroup budget per device.
    """

    def __init__(self, world: int, devices: Sequence[int] | None = None, *, slot_bytes: int = 16 << 20,
                 grid: int = 32, timeout_s: float = 10.0, max_lag: int | None = None, placement_tries: int = 1,
                 placement_bytes: int = 0, placement_dtype: torch.dtype = torch.bfloat16,
                 placement_min_frac: float = 0.95):
        """placement_tries > 1 (one device only): time one two-shot of `placement_bytes` per
        rank against the copy roofline and, while it runs below `placement_min_frac` of it,
        build the slabs anew on other physical pages (the earlier ones are held until the
        choice is made), up to that many times; the fastest placement is kept
        (`placement` reports the tries and fractions). The two-shot's speed at 8 x 256 MiB
        depends on where the driver puts the slab and buffer pages, by up to 17 %
        (profiles/round5/README.md section 10). The timing buffers are freed into torch's
        cache, so buffers of the same size allocated next reuse the pages that were timed."""
        if devices is None:
            devices = [torch.cuda.current_device()] * world
        if len(devices) != world:
            raise ValueError("need one device per logical rank")
        self.world = world
        self.devices = [torch.device("cuda", d) for d in devices]
        rows = 0 if max_lag is None else max_lag + 1  # threshold lag ring (allreduce_threshold)

        def build():
            comms = [_H.XgmiComm(k, world, self.devices[k].index, slot_bytes, grid, timeout_s, rows)
                     for k in range(world)]
            for c in comms:
                c.connect_local(comms)
            return comms

        self.comms = build()
        self.placement: dict = {"tries": 1}
        if placement_tries > 1 and len(set(self.devices)) == 1 and world > 1:
            self._place(build, placement_tries, placement_bytes or world * (slot_bytes // 2), placement_dtype,
                        placement_min_frac)
        self.groups: list[list[int]] = []
        for k in range(world):
            if self.groups and self.devices[self.groups[-1][-1]] == self.devices[k]:
                self.groups[-1].append(k)
            else:
                self.groups.append([k])

    def _place(self, build, tries: int, nbytes: int, dtype: torch.dtype, min_frac: float) -> None:
        from ..ops import fill_uniform
        from ..utils.timing import hbm_bytes

        dev = self.devices[0]
        es = torch.empty(0, dtype=dtype).element_size()
        n = max(1, nbytes // es)
        S = n * es
        stream = _current_stream(dev.index)
        # the order a caller's rank buffers are usually taken in: inputs, then outputs
        xs = [fill_uniform(torch.empty(n, dtype=dtype, device=dev), seed=900 + k) for k in range(self.world)]
        ys = [torch.empty_like(t) for t in xs]
        code = _dtype_code(dtype)

        def timed_ms(fn, iters: int = 7, warm: int = 2, q: float = 0.5) -> float:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
            for _ in range(warm):
                fn()
            for a, b in ev:
                a.record()
                fn()
                b.record()
            torch.cuda.synchronize(dev)
            return sorted(a.elapsed_time(b) for a, b in ev)[int(q * (iters - 1))]

        # the roofline: the copy kernel's best of 20 (its first calls run up to 10 % slow, which
        # would flatter every placement)
        copy_ms = timed_ms(lambda: C.hip.copy(xs[0].data_ptr(), ys[0].data_ptr(), S, stream), 20, 5, 0.0)
        roof = hbm_bytes(S, self.world, "twoshot", es) / (2 * S / copy_ms)  # ms at the copy's rate
        held, fracs = [], []
        comms = self.comms
        for t in range(tries):
            if t:
                comms = build()  # the earlier slabs are still held: these land on other pages
            ms = timed_ms(lambda: _H.XgmiComm.allreduce_local(
                comms, [x.data_ptr() for x in xs], [y.data_ptr() for y in ys], n, code, stream, ALGOS["twoshot"], 1.0))
            errs = [c.error() for c in comms]
            if any(errs):
                raise CommError("placement probe: " + "; ".join(f"rank {k}: {_describe(e)}"
                                                               for k, e in enumerate(errs) if e))
            held.append(comms)
            fracs.append(round(roof / ms, 3))
            if fracs[-1] >= min_frac:
                break
        keep = max(range(len(fracs)), key=lambda i: fracs[i])
        self.comms = held[keep]
        del held, comms, xs, ys  # the other placements' slabs are freed here
        self.placement = {"tries": len(fracs), "frac_copy_roofline": fracs, "kept": keep,
                          "bytes_per_rank": S, "copy_ms": round(copy_ms, 4)}

    def _check(self, inputs, outputs) -> list[torch.Tensor]:
        if len(inputs) != self.world:
            raise ValueError("one input per logical rank")
        outputs = list(outputs) if outputs is not None else [torch.empty_like(x) for x in inputs]
        n = inputs[0].numel()
        for k in range(self.world):
            x, y = inputs[k], outputs[k]
            if x.numel() != n or y.numel() != n or x.dtype != inputs[0].dtype or y.dtype != x.dtype:
                raise ValueError("all ranks must pass the same shape and dtype")
            if x.device != self.devices[k] or y.device != self.devices[k]:
                raise ValueError(f"rank {k} tensors must live on {self.devices[k]}")
            if not (x.is_contiguous() and y.is_contiguous()):
                raise ValueError("tensors must be contiguous")
        return outputs

    def allreduce(self, inputs: Sequence[torch.Tensor], outputs: Sequence[torch.Tensor] | None = None, *,
                  algo: str = "auto", op: str = "sum", stream: int | None = None) -> list[torch.Tensor]:
        """`stream`: raw HIP stream for a single-device cluster (default: the current one)."""
        outputs = self._check(inputs, outputs)
        n = inputs[0].numel()
        code = _dtype_code(inputs[0].dtype)
        for g in self.groups:
            dev = self.devices[g[0]]
            _H.XgmiComm.allreduce_local([self.comms[k] for k in g], [inputs[k].data_ptr() for k in g],
                                        [outputs[k].data_ptr() for k in g], n, code,
                                        _current_stream(dev.index) if stream is None else stream, ALGOS[algo],
                                        1.0 / self.world if op == "avg" else 1.0)
        return outputs

    def allreduce_threshold(self, inputs: Sequence[torch.Tensor], outputs: Sequence[torch.Tensor] | None = None, *,
                            th_reduce: float = 1.0, th_complete: float = 1.0, op: str = "sum", rescale: bool = False,
                            counts: bool = True):
        """One straggler-tolerant round for every logical rank (see
        XgmiCommunicator.allreduce_threshold). Returns (outputs, counts[world, world, nch]);
        counts=False skips the counts tensor (no allocation per call) and returns (outputs, None)."""
        outputs = self._check(inputs, outputs)
        n = inputs[0].numel()
        code = _dtype_code(inputs[0].dtype)
        cnts = []
        for g in self.groups:
            dev = self.devices[g[0]]
            cnt = None
            if counts:
                nch = self.comms[g[0]].threshold_chunks(n, code, len(g))
                cnt = torch.zeros(len(g), self.world, nch, dtype=torch.int32, device=dev)
            _H.XgmiComm.allreduce_threshold_local([self.comms[k] for k in g], [inputs[k].data_ptr() for k in g],
                                                  [outputs[k].data_ptr() for k in g], n, code,
                                                  _current_stream(dev.index), th_reduce, th_complete,
                                                  0 if cnt is None else cnt.data_ptr(),
                                                  1.0 / self.world if op == "avg" else 1.0, rescale)
            cnts.append(cnt)
        if not counts:
            return outputs, None
        return outputs, cnts[0] if len(cnts) == 1 else cnts

    def collective(self, op: str, inputs: Sequence[torch.Tensor], outputs: Sequence[torch.Tensor] | None = None, *,
                   scale: float = 1.0) -> list[torch.Tensor]:
        """op: "all_to_all" (in/out [world*m]), "all_gather" (in [m], out [world*m]) or
        "reduce_scatter" (in [world*m], out [m]) for every logical rank (xgmi_coll.hip)."""
        kind = {"all_to_all": _H.Coll.AllToAll, "all_gather": _H.Coll.AllGather,
                "reduce_scatter": _H.Coll.ReduceScatter}[op]
        if len(inputs) != self.world:
            raise ValueError("one input per logical rank")
        n = inputs[0].numel()
        m = n if op == "all_gather" else n // self.world
        out_n = self.world * m if op != "reduce_scatter" else m
        if outputs is None:
            outputs = [torch.empty(out_n, dtype=x.dtype, device=x.device) for x in inputs]
        code = _dtype_code(inputs[0].dtype)
        for g in self.groups:
            dev = self.devices[g[0]]
            _H.XgmiComm.collective_local([self.comms[k] for k in g], kind, [inputs[k].data_ptr() for k in g],
                                         [outputs[k].data_ptr() for k in g], m, code,
                                         torch.cuda.current_stream(dev).cuda_stream, scale)
        return list(outputs)

    def step_adamw(self, grads: Sequence[torch.Tensor], params: Sequence[torch.Tensor], states: Sequence[dict], *,
                   lr: float, betas: tuple[float, float] = (0.9, 0.999), eps: float = 1e-8,
                   weight_decay: float = 0.0, step: int, op: str = "avg") -> None:
        """The fused reduce-scatter + AdamW + all-gather for every logical rank."""
        h = _H.AdamW()
        h.lr, (h.beta1, h.beta2), h.eps, h.weight_decay, h.step = lr, betas, eps, weight_decay, step
        n = params[0].numel()
        code = _dtype_code(params[0].dtype)
        for g in self.groups:
            dev = self.devices[g[0]]
            _H.XgmiComm.step_adamw_local(
                [self.comms[k] for k in g], [grads[k].data_ptr() for k in g], [params[k].data_ptr() for k in g], n,
                code, torch.cuda.current_stream(dev).cuda_stream,
                [(states[k]["master"].data_ptr(), states[k]["exp_avg"].data_ptr(), states[k]["exp_avg_sq"].data_ptr())
                 for k in g], h, 1.0 / self.world if op == "avg" else 1.0)

    def barrier(self) -> None:
        for g in self.groups:
            dev = self.devices[g[0]]
            _H.XgmiComm.barrier_local([self.comms[k] for k in g], torch.cuda.current_stream(dev).cuda_stream)

    def check(self) -> None:
        for d in set(self.devices):
            torch.cuda.synchronize(d)
        errs = [c.error() for c in self.comms]
        if any(errs):
            raise CommError("; ".join(f"rank {k}: {_describe(e)}" for k, e in enumerate(errs) if e))
