"""xGMI bring-up pack: what the links give the engine's own store path, measured before the
first multi-GPU allreduce is timed (bench.py `xgmi_links`, N > 1).

The reference's data plane is an all-peer fan-out - every worker scatters to and broadcasts
to every other worker directly (/root/reference/src/main/scala/sample/cluster/allreduce/
AllreduceWorker.scala:194-209, :230-238) - which on 8 x MI355X drives all 7 xGMI links of a
GPU at once. The probes (csrc/hip/xgmi_probe.hip) use the two-shot's exact store path
(write-through 16-B pushes into a peer's fine-grained slab, relaxed system-scope flags):

  push_GBps[r][k]  rank r pushing into peer k alone, every rank at once with the same shift
                   d = k - r (a permutation: each GPU sends on one link and receives on one);
  all_GBps[r]      rank r pushing the same bytes into all peers at once (the fan-out);
  fanout_ratio     all_GBps / mean single-peer rate (7 links ideal: 7.0);
  coarse / pull    the same single-peer and all-peer rates for two other paths a two-shot
                   could take: plain stores into the peer's COARSE-grained memory with one
                   system release per workgroup (`coarse`), and remote LOADS of the peer's
                   fine-grained slab (`pull`) - which store path and memory kind the links
                   serve best is then read off the first 8-GPU run;
  flag_us[k]       one-way flag hand-off rank 0 <-> k, bare (relaxed store + poll) and with
                   the kernels' release / acquire fences.

Collective: every rank of the communicator must call probe_links together, with no other
launch of the communicator in flight.
"""
from __future__ import annotations

import torch


def _barrier(comm) -> None:
    import torch.distributed as dist

    torch.cuda.synchronize(comm.device)
    dist.barrier(group=comm.cpu_group)


def probe_links(comm, nbytes: int = 64 << 20, reps: int = 5, iters: int = 2000, grid: int = 0) -> dict:
    """Push rates and flag latencies of `comm` (an XgmiCommunicator, world > 1). `grid`:
    workgroups per destination (0 = 64, enough to saturate one link; the all-peer launch uses
    the same count per peer)."""
    import torch.distributed as dist

    P, r, dev = comm.world, comm.rank, comm.device
    c = comm._c
    nbytes = min(int(nbytes), int(c.probe_max_bytes)) // 4096 * 4096
    g = grid or 64
    src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev).uniform_(-1, 1)
    stream = torch.cuda.current_stream(dev)
    out: dict = {"bytes": nbytes, "reps": reps, "grid_per_peer": g, "store": "st16_wt (two-shot scatter path)",
                 "coarse_store": "plain st16 + system release per workgroup", "pull_load": "remote system-coherent ld16"}

    def timed_push(mask: int, mode: int = 0) -> float:
        c.probe_push(src.data_ptr(), nbytes, mask, g, stream.cuda_stream, mode)  # warm-up
        _barrier(comm)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            c.probe_push(src.data_ptr(), nbytes, mask, g, stream.cuda_stream, mode)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / 1e3 / reps  # s per launch

    def rates(mode: int):
        # one peer at a time, every rank with the same shift d: mine[k] = this rank <-> (r + d) % P
        mine = [0.0] * P
        for d in range(1, P):
            k = (r + d) % P
            mine[k] = round(nbytes / timed_push(1 << k, mode) / 1e9, 2)
        all_rate = round((P - 1) * nbytes / timed_push(((1 << P) - 1) & ~(1 << r), mode) / 1e9, 2)
        rows: list = [None] * P
        dist.all_gather_object(rows, (mine, all_rate), group=comm.cpu_group)
        singles = [v for i, row in enumerate(rows) for k, v in enumerate(row[0]) if k != i]
        return rows, singles

    rows, singles = rates(0)
    out["push_GBps"] = [row[0] for row in rows]
    out["all_GBps"] = [row[1] for row in rows]
    mean_single = sum(singles) / len(singles) if singles else 0.0
    out["single_GBps_min_med_max"] = [min(singles), sorted(singles)[len(singles) // 2], max(singles)]
    out["fanout_ratio"] = round(min(out["all_GBps"]) / mean_single, 2) if mean_single else None
    # the coarse-grained push and the pull: [single-peer min, median, max], [all-peer min, max]
    handles: list = [None] * P
    dist.all_gather_object(handles, c.probe_coarse_handle(), group=comm.cpu_group)
    c.probe_coarse_connect(handles)
    _barrier(comm)
    for mode, key in ((1, "coarse"), (2, "pull")):
        rows_m, singles_m = rates(mode)
        alls = [row[1] for row in rows_m]
        out[key] = {"single_GBps_min_med_max": [min(singles_m), sorted(singles_m)[len(singles_m) // 2], max(singles_m)],
                    "all_GBps_min_max": [min(alls), max(alls)]}

    # flag hand-off rank 0 <-> k (others idle between barriers)
    # (the token nonce is the same on both sides: a per-communicator call count, so a word
    # left by an earlier probe never matches)
    ticks = torch.zeros(1, dtype=torch.int64, device=dev)
    lat = {"bare": [None] * P, "fenced": [None] * P}
    calls = getattr(comm, "_probe_calls", 0) + 1
    comm._probe_calls = calls
    for fenced in (False, True):
        for k in range(1, P):
            _barrier(comm)
            if r in (0, k):
                ticks.zero_()
                nonce = 1 + (calls * 2 * P + 2 * k + int(fenced)) % 65535
                c.probe_pingpong(k if r == 0 else 0, iters, nonce, fenced, ticks.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize(dev)
            if r == 0:
                t = ticks.item()
                # ticks = iters round trips at 100 MHz; one-way = half a round trip
                lat["fenced" if fenced else "bare"][k] = round(t / iters / 2 / 100.0, 3) if t else None
    obj = [lat]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(comm.cpu_group, 0) if comm.cpu_group else 0,
                               group=comm.cpu_group)
    out["flag_us"] = obj[0]
    _barrier(comm)
    comm.check()
    return out

