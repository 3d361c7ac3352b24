"""The protocol-driven GPU round engine, in one process.

The reference runs one master actor and N worker actors (AllreduceMaster.scala:15-98,
AllreduceWorker.scala:9-270). `PlaneJob` builds exactly that on the native actor runtime,
with every worker a `PlaneWorkerActor` (csrc/runtime/plane_worker.h) over its own xGMI round
plane (csrc/hip/xgmi_plane.h): StartAllreduce(r) from the master becomes ONE threshold-kernel
launch per worker, the sink gets the GPU output tensor and the real per-chunk counts, and
CompleteAllreduce goes back to the master. Registration carries each worker's plane
descriptor (its HBM arena's IPC handle) in MemberUp.meta; the master relays them to all
workers in InitWorkers.planes.

Multi-process deployments use the CLIs instead (`mxar-master` + `mxar-worker --device k`);
the plane descriptor then travels in the cluster join (ClusterConfig.meta).

    job = PlaneJob(3, 1 << 20, max_chunk_size=1 << 14, th_reduce=1.0, th_complete=1.0, max_round=20)
    job.run()
    out, counts = job.outputs[0][20]   # worker 0, round 20
"""
from __future__ import annotations

import itertools
import os
import threading
import time
import warnings
from typing import Callable, Sequence

import numpy as np
import torch

from ._native import C
from .ops.kernels import dtype_code

_HUBS = itertools.count()


def default_plane_grid(device: int, share: int) -> int:
    """Workgroups per round kernel of a plane worker when `share` workers run on `device`.

    One worker per GPU: 2 per CU (the plane's own default). Co-located workers split
    the CUs: together they run about one workgroup per CU, so every worker's kernel stays
    resident beside the others. Their planes also coarsen full-threshold rounds to one chunk
    per workgroup. 2 workers x 128 workgroups beat 2 x 256 by 8-30 % per round at
    16-256 MiB (profiles/round5/protocol_grid_chunk.jsonl). Co-located workers also fit what
    the device's residency budget has left (csrc/hip/residency.h: every spinning kernel of
    the process reserves its workgroups; a second job shares the device with the first)."""
    cus = torch.cuda.get_device_properties(device).multi_processor_count if torch.cuda.is_available() else 256
    if share <= 1:
        return 2 * cus
    st = C.hip.residency_state(device)
    free = st["capacity"] - st["used"]
    return max(0, min(max(8, cus // share), (free - 1) // share))


def iota_source(n: int, device: torch.device, dtype: torch.dtype, offset: float = 0.0) -> Callable:
    """The reference's demo dataSource (AllreduceWorker.scala:285-291), data[i] = i + iteration
    (+ offset), produced on the GPU by the fill_iota kernel on torch's current stream."""
    code = dtype_code(dtype)

    def source(req):
        x = torch.empty(n, dtype=dtype, device=device)
        C.hip.fill_iota(x.data_ptr(), n, float(req.iteration) + offset, code, torch.cuda.current_stream(device).cuda_stream)
        return x

    return source


def host_iota_source(n: int, offset: float = 0.0) -> Callable:
    """The reference's demo dataSource on the host (float32 data[i] = i + iteration + offset)."""
    base = np.arange(n, dtype=np.float32)

    def source(req):
        return base + np.float32(req.iteration + offset)

    return source


class PlaneJob:
    """Master + P plane workers in one process (threaded actor system).

    Workers sharing a GPU form a plane group (csrc/hip/xgmi_plane.cc PlaneGroup): ONE
    resident kernel runs every round of every one of them, a slice of workgroups per worker
    fed from that worker's own door ring (xgmi_threshold.hip
    threshold_group_resident_kernel). Each worker's rounds still run on their own schedule (a
    straggler's slice lags while the others run ahead), and no round can wait in a hardware
    queue behind a co-located peer's spinning round, so any number of workers (<= 16 per GPU)
    runs at the boxes' GPU_MAX_HW_QUEUES = 4 - the reference hosts any number of worker
    actors in one ActorSystem (AllreduceSpec.scala:746-755)."""

    def __init__(self, P: int, data_size: int, *, max_chunk_size: int, th_allreduce: float = 1.0,
                 th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 1, max_round: int = 10,
                 devices: Sequence[int] | None = None, dtype: torch.dtype = torch.float32, grid: int = 0,
                 sources: Sequence[Callable] | None = None, keep_outputs: bool = True, round_timeout_ms: int = 0,
                 timeout_s: float = 60.0, order_ref: bool = True, on_output: Callable | None = None,
                 max_peers: int | None = None, high_priority: bool = True, order_release: bool = True,
                 plane: str = "xgmi", hub: str | None = None, spin_us: int = 1000, reinit_on_loss: bool = False,
                 split: bool = True, keep_last: bool = False, bridge_port: int | None = None,
                 external_rounds: bool = False, min_chunk: int | None = None, lag_wait_us: float | None = None,
                 record: bool = False):
        """plane: "xgmi" (one threshold-kernel launch per round on the GPUs in `devices`) or
        "loopback" (host memory, no GPU: csrc/runtime/loopback_plane.h; `hub` names the
        workers' shared hub, default a fresh one; dtype float32, devices ignored).
        split: chunks fewer than the plane's workgroups are split into slices over several
        workgroups, each chunk still one threshold decision (csrc/hip/xgmi_threshold.hip).
        sources: callables (AllReduceInputRequest -> tensor / array) or GPU tensors; a tensor is
        fetched natively every round (no Python, no GIL).
        keep_last: each worker keeps only its newest round output, natively (`last_output(k)`);
        replaces keep_outputs / on_output, so no Python runs on the round path.
        bridge_port: serve the master's control bridge there (0 = any free port, see
        `bridge_port`; docs/BRIDGE.md). external_rounds: bridge clients drive the rounds.
        min_chunk: the planes keep one flag / count / threshold decision per chunk of at least
        this many elements (xgmi_plane.h); default: max_chunk_size whenever it is finer than the
        1 KiB flag granularity, so every reference chunk is decided on its own (the reference's
        DataBuffer semantics at any maxChunkSize).
        lag_wait_us: a round waits at most this long at its lag gate for a peer still in the
        round that last used its row, then runs without it (XgmiPlaneOptions::lag_wait_us; the
        straggler mode at thresholds < 1). None: wait for the peer (bounded buffers).
        record: with keep_last, the native sinks also keep every round's sink time and count
        totals (`sink_stamps(k)`, `count_stats(k)`)."""
        self.P = P
        self.n = data_size
        self.dtype = dtype
        if plane not in ("xgmi", "loopback"):
            raise ValueError(f"unknown plane {plane!r}")
        self.plane_kind = plane
        if plane == "loopback":
            self.devices = [None] * P
            grid = 0
        else:
            self.devices = list(devices) if devices is not None else [torch.cuda.current_device()] * P
        if len(self.devices) != P:
            raise ValueError("one device per worker")
        self._residency = []
        if plane == "xgmi":
            share = max(self.devices.count(d) for d in set(self.devices))
            if grid <= 0:
                grid = min(default_plane_grid(d, self.devices.count(d)) for d in set(self.devices))
            # co-located workers' group kernels spin: reserve their workgroups (+ the
            # dispatcher wave) in the device budget now, so a job that cannot fit beside what
            # already runs fails HERE, loudly, not as round timeouts (csrc/hip/residency.h)
            for d in sorted(set(self.devices)):
                k = self.devices.count(d)
                if k > 1:
                    if grid < 8:
                        st = C.hip.residency_state(d)
                        raise RuntimeError(f"residency budget: {k} co-located workers on device {d} need >= 8 "
                                           f"workgroups each; {st['capacity'] - st['used']} of {st['capacity']} "
                                           f"free (held: {st['holders']})")
                    self._residency.append(C.hip.residency_reserve(d, k * grid + 1, f"PlaneJob {k} workers x {grid}"))
        self.grid = grid
        self.system = C.ActorSystem("ClusterSystem", False)
        self.finished = threading.Event()
        self.rounds = {"n": 0}
        self.outputs: list[dict[int, tuple]] = [dict() for _ in range(P)]
        self.keep = keep_outputs
        self.on_output = on_output
        if plane == "loopback":
            hub = hub or f"planejob{next(_HUBS)}"
            self.planes = [C.loopback_plane(hub) for _ in range(P)]
            if sources is None:
                sources = [host_iota_source(data_size, 1000.0 * k) for k in range(P)]
        else:
            es = torch.empty(0, dtype=dtype).element_size()
            if min_chunk is None:
                min_chunk = max_chunk_size if max_chunk_size * es < 1024 else 0
            self.planes = [C.hip.xgmi_plane(d, dtype_code(dtype), data_size, max_peers=max_peers or P,
                                            max_lag=max_lag, grid=grid, timeout_s=timeout_s, order_ref=order_ref,
                                            high_priority=high_priority, order_release=order_release,
                                            spin_us=spin_us, split=split, min_chunk=min_chunk,
                                            lag_wait_us=-1.0 if lag_wait_us is None else float(lag_wait_us),
                                            residency_external=self.devices.count(d) > 1)
                           for d in self.devices]
            if sources is None:
                sources = [iota_source(data_size, torch.device("cuda", d), dtype, 1000.0 * k)
                           for k, d in enumerate(self.devices)]
        # a GPU tensor as a source: the same buffer every round, fetched without Python
        # (hip.tensor_source) - no GIL on the round path for persistent gradient buffers
        self.sources = [C.hip.tensor_source(src) if isinstance(src, torch.Tensor) and plane == "xgmi" else src
                        for src in sources]
        self.keep_last = keep_last
        self._final_stamps: list[float] | None = None
        self._last = [C.last_output_sink(record) for _ in range(P)] if keep_last else None

        def fin(r):
            self.rounds["n"] = r
            self.finished.set()

        self.master = self.system.master(P, th_allreduce, th_reduce, th_complete, max_lag, data_size, max_round,
                                         max_chunk_size, on_finished=fin, roundTimeoutMs=round_timeout_ms,
                                         reinitOnLoss=reinit_on_loss, externalRounds=external_rounds,
                                         bridgePort=-1 if bridge_port is None else bridge_port)
        self.workers = [self.system.plane_worker(self.sources[k], self._sink(k), self.planes[k], f"worker{k}")
                        for k in range(P)]

    def _sink(self, k: int):
        if self._last is not None:  # keep_last: a native sink, no Python per round
            return self._last[k]
        if not self.keep and self.on_output is None:
            return None

        def sink(out):
            if self.keep:
                self.outputs[k][out.iteration] = (out.data, list(out.count))
            if self.on_output is not None:
                self.on_output(k, out)
        return sink

    def start(self) -> None:
        """Register the workers with the master (MemberUp carrying the plane descriptor, in
        worker order: worker k gets id k)."""
        for w, p in zip(self.workers, self.planes):
            self.master.tell(C.MemberUp(w, "worker", "", p.descriptor), None)

    def run(self, timeout: float = 120.0) -> float:
        """start() and wait until the master finished every round; returns the wall time."""
        t0 = time.perf_counter()
        self.start()
        if not self.finished.wait(timeout):
            planes = [p.debug_state() for p in self.planes if hasattr(p, "debug_state")]
            msg = f"plane job did not finish in {timeout} s: {self.state()} planes: {planes}"
            print(msg, file=__import__("sys").stderr, flush=True)  # before any teardown that may block
            raise TimeoutError(msg)
        for p in self.planes:  # the last round's sinks run after the master's last barrier
            p.drain()
        self.system.await_idle(10.0)
        return time.perf_counter() - t0

    @property
    def stamps(self) -> list[float]:
        """perf_counter() seconds at which each round reached the master's barrier (recorded
        natively by the master: no Python callback on the round path)."""
        if self._final_stamps is not None:
            return self._final_stamps
        return self.system.master_round_stamps(self.master)

    @property
    def bridge_port(self) -> int:
        """The master's control-bridge port (-1 without a bridge)."""
        return self.system.master_bridge_port(self.master)

    def last_output(self, k: int):
        """keep_last: worker k's newest AllReduceOutput (None before its first round)."""
        if self._last is None:
            raise RuntimeError("PlaneJob(keep_last=True) keeps the last output")
        return self._last[k].last()

    def sink_stamps(self, k: int) -> list[tuple[int, float]]:
        """keep_last + record: worker k's (iteration, perf_counter seconds) per completed round."""
        return self._last[k].stamps()

    def count_stats(self, k: int) -> dict:
        """keep_last + record: worker k's per-chunk count totals over every round."""
        return self._last[k].count_stats()

    def state(self) -> dict:
        return {"master": self.system.master_state(self.master),
                "workers": [self.system.plane_worker_state(w) for w in self.workers]}

    def shutdown(self) -> None:
        """Stop the actors and destroy the planes NOW. A plane's destructor frees device
        memory (hipFree synchronises the whole device); left to a later garbage collection it
        could run while another job's round kernels spin on a worker whose thread is stuck in
        that free - a deadlock until the kernels' deadline."""
        import gc

        if self._final_stamps is None:
            self._final_stamps = self.system.master_round_stamps(self.master)
        self.system.shutdown()
        self.planes = []
        self.workers = []
        gc.collect()
        for t in self._residency:  # after the planes (and their group kernels) are gone
            t.release()
        self._residency = []


def distributed_plane_job(n: int, source, *, max_chunk_size: int, dtype: torch.dtype, rounds: int,
                          th: float = 1.0, max_lag: int = 1, grid: int = 0, timeout_s: float = 300.0,
                          on_output: Callable | None = None, keep_last: bool = False,
                          external_client: bool = False, min_chunk: int | None = None,
                          host_spin_us: int | None = 500) -> dict:
    """One plane worker per torch.distributed rank (one process per GPU), the master on rank 0,
    the reference's cluster shape: workers join rank 0's seed over TCP (127.0.0.1) and
    announce their plane descriptors in the join; the master relays them in InitWorkers and
    drives `rounds` rounds; the data moves over xGMI inside the planes. torch.distributed is
    used only to agree on the seed port and to hold the ranks until the master is done.
    `source`: a callable or a GPU tensor (fetched natively every round); keep_last: a native
    sink keeps the newest output (returned as "last") instead of calling `on_output`.
    external_client: the master runs in externalRounds mode with a control bridge and rank 0
    drives the rounds through it as an outside client would (docs/BRIDGE.md, pipelined
    StartAllreduce); "stamps" are then the client's RoundComplete arrival times.
    host_spin_us: actor dispatchers and cluster readers keep polling this long after their last
    work before sleeping (MXAR_DISPATCH_SPIN_US / MXAR_TCP_SPIN_US unless already set; the
    native executables' --spin-us): every TCP hop of a round then lands on a running thread -
    native 64 MiB rounds 176-198 -> 152-160 us (profiles/round3/native_spin_ab.jsonl).
    Returns (rank 0) {"stamps": round completion times, "state": worker state}."""
    import os

    import torch.distributed as dist

    from .parallel.comm import free_port

    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.cuda.current_device()
    if host_spin_us is not None and host_spin_us >= 0:  # read when the system / readers start
        os.environ.setdefault("MXAR_DISPATCH_SPIN_US", str(host_spin_us))
        os.environ.setdefault("MXAR_TCP_SPIN_US", str(host_spin_us))
    system = C.ActorSystem("ClusterSystem", False)
    if min_chunk is None:  # one flag per reference chunk when maxChunkSize is finer than 1 KiB
        min_chunk = max_chunk_size if max_chunk_size * torch.empty(0, dtype=dtype).element_size() < 1024 else 0
    plane = C.hip.xgmi_plane(dev, dtype_code(dtype), n, max_peers=world, max_lag=max_lag, grid=grid,
                             timeout_s=min(60.0, timeout_s), min_chunk=min_chunk)
    if isinstance(source, torch.Tensor):  # fetched natively every round (no GIL)
        source = C.hip.tensor_source(source)
    last = C.last_output_sink() if keep_last else None
    sink = last if keep_last else (lambda out: on_output(out)) if on_output is not None else None
    worker = system.plane_worker(source, sink, plane, "worker")
    port = [free_port() if rank == 0 else 0]
    dist.broadcast_object_list(port, src=0)
    cc = C.ClusterConfig()
    cc.host = "127.0.0.1"
    cc.port = port[0] if rank == 0 else 0
    cc.roles = ["worker"]
    cc.seed_nodes = [f"mxar.tcp://ClusterSystem@127.0.0.1:{port[0]}"]
    cc.heartbeat_interval_s = 0.2
    cc.acceptable_heartbeat_pause_s = 10.0
    cc.auto_down_unreachable_after_s = -1.0
    cc.meta = plane.descriptor
    fin = threading.Event()
    master = None
    if rank == 0:
        master = system.master(world, 1.0, th, th, max_lag, n, rounds - 1, max_chunk_size,
                               on_finished=lambda r: fin.set(), externalRounds=external_client,
                               bridgePort=0 if external_client else -1)
    node = C.ClusterNode.start(system, cc)
    if master is not None:
        node.subscribe(master)
    ok = [True]
    client_stamps: list[float] = []
    if rank == 0 and external_client:
        from .bridge import BridgeClient

        try:
            with BridgeClient("127.0.0.1", system.master_bridge_port(master), timeout=min(120.0, timeout_s)) as b:
                b.wait_for("InitWorkers")
                b.start(0)
                for r in range(rounds):
                    if r + 1 < rounds:
                        b.start(r + 1)  # queued behind round r
                    b.wait_for("RoundComplete", round=r)
                    client_stamps.append(time.perf_counter())
        except Exception as e:  # noqa: BLE001 - the ranks must still leave together
            ok = [False]
            client_stamps = []
            import warnings

            warnings.warn(f"bridge-driven job failed: {e!r}", RuntimeWarning, stacklevel=2)
    if rank == 0 and ok[0]:
        ok = [fin.wait(timeout_s)]
    dist.broadcast_object_list(ok, src=0)
    plane.drain()
    system.await_idle(5.0)
    stamps = (client_stamps if external_client else system.master_round_stamps(master)) if master is not None else []
    out = {"ok": bool(ok[0]), "stamps": stamps, "state": system.plane_worker_state(worker),
           "plane": {"launches": plane.stats.launches, "chunk_elems": plane.chunk_elems, "chunks": plane.chunks,
                     "resident_rounds": plane.stats.resident_rounds},
           "last": last.last() if last is not None else None}
    dist.barrier()
    node.leave()
    time.sleep(0.3)
    node.shutdown()
    system.shutdown()
    del plane
    return out
