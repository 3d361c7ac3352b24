"""Command-line entry points, argument-compatible with the reference's mains.

    mxar-master [port totalWorkers dataSize maxChunkSize]      AllreduceMaster.scala:101-137
    mxar-worker [port sourceDataSize]                           AllreduceWorker.scala:272-301

Defaults are the reference's: master port 2551, 2 workers, dataSize = totalWorkers * 5,
maxChunkSize 2, thresholds thAllreduce 1 / thReduce 0.9 / thComplete 0.8, maxLag 1,
maxRound 100; worker port 2553, sourceDataSize 10, data source data[i] = i + iteration.
Everything else comes from the layered config (conf/application.conf, MXAR_* env,
--set key=value). Differences from the reference (documented fixes): the master exits
after the last round and workers exit when the master leaves the cluster.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import threading
import time

import numpy as np

from . import config as mconfig
from ._native import C
from .utils.metrics import (MetricsRegistry, cluster_source, master_source, plane_worker_source, worker_source,
                            write_trace)


def _cluster_cfg(cfg: mconfig.Config, port: int, roles: list[str]) -> "C.ClusterConfig":
    cc = C.ClusterConfig()
    cc.host = str(cfg["mxar.remote.hostname"])
    cc.port = int(port)
    cc.roles = roles
    cc.seed_nodes = cfg.seeds()
    cc.heartbeat_interval_s = float(cfg["mxar.cluster.failure-detector.heartbeat-interval"])
    cc.acceptable_heartbeat_pause_s = float(cfg["mxar.cluster.failure-detector.acceptable-heartbeat-pause"])
    cc.auto_down_unreachable_after_s = float(cfg["mxar.cluster.auto-down-unreachable-after"])
    cc.worker_path = str(cfg["mxar.cluster.worker-path"])
    return cc


def _common(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--config", action="append", default=[], help="HOCON config file (repeatable)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE", help="config override")
    ap.add_argument("--metrics-json", default=None, help="write the metrics snapshot here at exit")
    ap.add_argument("--metrics-port", type=int, default=None, help="serve Prometheus /metrics on this port")
    ap.add_argument("--trace-json", default=None, help="record a Chrome-trace timeline, written at exit")


def _observe(args, cfg, labels: dict) -> MetricsRegistry:
    reg = MetricsRegistry(labels)
    trace = args.trace_json or cfg.get("mxar.trace.json")
    if trace:
        C.trace.enable(True)
    if args.metrics_port is not None:
        port = reg.serve(args.metrics_port)
        print(f"[mxar] metrics on http://127.0.0.1:{port}/metrics", file=sys.stderr, flush=True)
    return reg


def _finish(args, cfg, reg: MetricsRegistry, extra: dict) -> None:
    path = args.metrics_json or cfg.get("mxar.metrics.json")
    if path:
        snap = reg.snapshot()
        snap.update(extra)
        with open(path, "w") as f:
            json.dump(snap, f, indent=1, default=str)
    trace = args.trace_json or cfg.get("mxar.trace.json")
    if trace:
        n = write_trace(trace)
        print(f"[mxar] wrote {n} trace events to {trace}", file=sys.stderr, flush=True)
    reg.close()


def _load(args) -> mconfig.Config:
    cfg = mconfig.load(args.config, args.set)
    C.set_log_level(str(cfg["mxar.loglevel"]))
    return cfg


def _install_signals(stop: threading.Event) -> None:
    for s in (signal.SIGINT, signal.SIGTERM):
        try:
            signal.signal(s, lambda *_: stop.set())
        except ValueError:  # not the main thread
            pass


def master_main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="mxar-master", description=__doc__)
    ap.add_argument("port", nargs="?", type=int, default=2551)
    ap.add_argument("totalWorkers", nargs="?", type=int, default=None)
    ap.add_argument("dataSize", nargs="?", type=int, default=None)
    ap.add_argument("maxChunkSize", nargs="?", type=int, default=None)
    ap.add_argument("--linger", action="store_true", help="keep running after the last round (reference behaviour)")
    ap.add_argument("--checkpoint", default=None, help="write {round, epoch} here after every completed round")
    ap.add_argument("--resume", action="store_true", help="start at the round after the one in --checkpoint")
    ap.add_argument("--bridge", type=int, default=None, metavar="PORT",
                    help="serve the control bridge (JSON lines, docs/BRIDGE.md) on PORT (0 = any free port)")
    ap.add_argument("--external-rounds", action="store_true",
                    help="bridge clients drive the rounds with StartAllreduce (the master only inits workers)")
    ap.add_argument("--akka-port", type=int, default=None, metavar="PORT",
                    help="serve the master as akka.tcp://<system>@host:PORT/user/master (docs/AKKA_WIRE.md)")
    _common(ap)
    args = ap.parse_args(argv)
    if args.bridge is not None:
        args.set.append(f"mxar.bridge.port={args.bridge}")
    if args.akka_port is not None:
        args.set.append(f"mxar.akka.port={args.akka_port}")
    if args.external_rounds:
        args.set.append("mxar.bridge.external-rounds=true")
    cfg = _load(args)
    total = args.totalWorkers if args.totalWorkers is not None else int(cfg["mxar.allreduce.total-workers"])
    data_size = args.dataSize if args.dataSize is not None else (
        total * 5 if cfg.origin.get("mxar.allreduce.data-size") == "default" else int(cfg["mxar.allreduce.data-size"]))
    chunk = args.maxChunkSize if args.maxChunkSize is not None else int(cfg["mxar.allreduce.max-chunk-size"])
    system = C.ActorSystem(str(cfg["mxar.system-name"]), False)
    done = threading.Event()
    stop = threading.Event()
    rounds = {"n": 0}

    def finished(r: int) -> None:
        rounds["n"] = r
        done.set()

    start_round = 0
    if args.resume and args.checkpoint and os.path.exists(args.checkpoint):
        with open(args.checkpoint) as f:
            start_round = int(json.load(f)["round"]) + 1
        print(f"[mxar-master] resuming at round {start_round} from {args.checkpoint}", flush=True)

    stamps: list[float] = []  # completion time of every round: steady-state round rate

    def on_round(r: int, epoch: int) -> None:
        stamps.append(time.perf_counter())
        if args.checkpoint:  # atomic replace: a crash never leaves a torn checkpoint
            tmp = args.checkpoint + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"round": r, "epoch": epoch, "dataSize": data_size, "totalWorkers": total}, f)
            os.replace(tmp, args.checkpoint)

    master = system.master(total, float(cfg["mxar.allreduce.th-allreduce"]), float(cfg["mxar.allreduce.th-reduce"]),
                           float(cfg["mxar.allreduce.th-complete"]), int(cfg["mxar.allreduce.max-lag"]), data_size,
                           int(cfg["mxar.allreduce.max-round"]), chunk,
                           liveBarrier=bool(cfg["mxar.allreduce.live-barrier"]),
                           reinitOnLoss=bool(cfg["mxar.allreduce.reinit-on-loss"]),
                           resumeOnJoin=bool(cfg["mxar.allreduce.resume-on-join"]), on_finished=finished, name="master",
                           startRound=start_round, on_round=on_round,
                           roundTimeoutMs=int(float(cfg["mxar.allreduce.round-timeout"]) * 1000),
                           externalRounds=bool(cfg["mxar.bridge.external-rounds"]),
                           bridgePort=max(int(cfg["mxar.bridge.port"]), 0 if int(cfg["mxar.akka.port"]) >= 0 else -1),
                           bridgeHost=str(cfg["mxar.bridge.host"]))
    bridge_port = system.master_bridge_port(master)
    if bridge_port >= 0:
        print(f"[mxar-master] control bridge on {cfg['mxar.bridge.host']}:{bridge_port}"
              f"{' (external rounds)' if cfg['mxar.bridge.external-rounds'] else ''}", flush=True)
    if int(cfg["mxar.akka.port"]) >= 0:  # a front-end of the bridge (csrc/runtime/akka_endpoint.h)
        akka_ep = C.akka.start_endpoint(master, port=int(cfg["mxar.akka.port"]), host=str(cfg["mxar.bridge.host"]),
                                        system=str(cfg["mxar.system-name"]), package=str(cfg["mxar.akka.package"]),
                                        suid_start=int(cfg["mxar.akka.suid.start-allreduce"]),
                                        suid_complete=int(cfg["mxar.akka.suid.complete-allreduce"]),
                                        cookie=str(cfg["mxar.akka.cookie"]))
        print(f"[mxar-master] akka.tcp endpoint {akka_ep.address} serves {akka_ep.master_path}", flush=True)
    node = C.ClusterNode.start(system, _cluster_cfg(cfg, args.port, ["master"]))
    node.subscribe(master)
    reg = _observe(args, cfg, {"role": "master", "address": node.address})
    reg.register("master", master_source(system, master))
    reg.register("cluster", cluster_source(node))
    print(f"[mxar-master] {node.address} totalWorkers={total} dataSize={data_size} maxChunkSize={chunk}",
          flush=True)
    _install_signals(stop)
    t0 = time.time()
    while not stop.is_set() and not (done.is_set() and not args.linger):
        stop.wait(0.1)
    elapsed = time.time() - t0
    if done.is_set():
        print(f"[mxar-master] finished {rounds['n']} rounds in {elapsed:.2f}s", flush=True)
    steady = (len(stamps) - 1) / (stamps[-1] - stamps[0]) if len(stamps) > 1 and stamps[-1] > stamps[0] else 0.0
    _finish(args, cfg, reg, {"rounds": rounds["n"], "elapsed_s": elapsed, "steady_rounds_per_s": steady})
    node.leave()
    time.sleep(0.2)
    node.shutdown()
    system.shutdown()
    return 0 if done.is_set() or stop.is_set() else 1


def worker_main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="mxar-worker", description=__doc__)
    ap.add_argument("port", nargs="?", type=int, default=2553)
    ap.add_argument("sourceDataSize", nargs="?", type=int, default=10)
    ap.add_argument("--print-outputs", action="store_true", help="one JSON line per AllReduceOutput on stdout")
    ap.add_argument("--max-outputs", type=int, default=0, help="exit after this many outputs (0 = never)")
    ap.add_argument("--device", type=int, default=None,
                    help="run the worker on this GPU: an xGMI round plane (one kernel launch per round, peers' "
                         "HBM mapped over IPC; csrc/hip/xgmi_plane.h) instead of ScatterBlock/ReduceBlock messages")
    ap.add_argument("--dtype", choices=["fp32", "bf16", "fp16"], default=None, help="GPU worker element type")
    ap.add_argument("--source-delay-ms", type=float, default=0.0,
                    help="sleep this long in the data source every round (demos / failure tests: slow rounds)")
    _common(ap)
    args = ap.parse_args(argv)
    cfg = _load(args)
    if args.device is not None:
        # a GPU worker's host threads keep polling through each round (the native mxar-gpu's
        # --spin-us default): every hop of the next round lands on a running thread
        spin = str(int(cfg["mxar.host-spin-us"]))
        os.environ.setdefault("MXAR_DISPATCH_SPIN_US", spin)
        os.environ.setdefault("MXAR_TCP_SPIN_US", spin)
    system = C.ActorSystem(str(cfg["mxar.system-name"]), False)
    n = args.sourceDataSize
    count = {"n": 0}
    stop = threading.Event()
    plane = None

    def sink(out):  # logging sink (AllreduceWorker.scala:295-297)
        count["n"] += 1
        if args.print_outputs:
            data = out.data
            data = data.float().cpu().tolist() if hasattr(data, "cpu") else np.asarray(data).tolist()
            print(json.dumps({"iteration": out.iteration, "data": data, "count": list(out.count)}), flush=True)
        if args.max_outputs and count["n"] >= args.max_outputs:
            stop.set()

    meta = ""
    if args.device is None:
        base = np.arange(n, dtype=np.float32)

        def source(req):  # createDataSource: data[i] = i + iteration (AllreduceWorker.scala:285-291)
            if args.source_delay_ms > 0:
                time.sleep(args.source_delay_ms / 1e3)
            return C.AllReduceInput(base + np.float32(req.iteration))

        wref = system.worker(source, sink, "worker")
    else:
        plane, source = _gpu_worker_plane(args, cfg, n)
        wref = system.plane_worker(source, sink, plane, "worker")
        meta = plane.descriptor  # the master relays it to every peer in InitWorkers.planes
    cc = _cluster_cfg(cfg, args.port, ["worker"])
    cc.meta = meta
    node = C.ClusterNode.start(system, cc)
    reg = _observe(args, cfg, {"role": "worker", "address": node.address})
    if plane is None:
        reg.register("worker", worker_source(system, wref))
    else:
        reg.register("worker", plane_worker_source(system, wref, plane))
    reg.register("cluster", cluster_source(node))
    events = system.probe("membership")
    node.subscribe(events)  # MemberUp events are queued: a short-lived master is never missed
    where = f" device=cuda:{args.device} plane={plane.name}" if plane is not None else ""
    print(f"[mxar-worker] {node.address} sourceDataSize={n}{where}", file=sys.stderr, flush=True)
    _install_signals(stop)
    seen_master = False
    while not stop.is_set():
        ev = events.receive(0.1)
        if ev is not None and isinstance(ev[0], C.MemberUp) and ev[0].role == "master":
            seen_master = True
        if seen_master and not any("master" in m["roles"] for m in node.members()):
            break  # the master left / was downed: the job is over
    _finish(args, cfg, reg, {"outputs": count["n"]})
    node.leave()
    time.sleep(0.1)
    node.shutdown()
    system.shutdown()
    return 0


def _gpu_worker_plane(args, cfg: mconfig.Config, n: int):
    """The GPU worker: an xGMI round plane on cuda:<device> and the reference's demo data
    source, data[i] = i + iteration (AllreduceWorker.scala:285-291), produced on the GPU by
    the fill_iota kernel in the plane's element type."""
    import torch

    from .ops.kernels import dtype_code

    dt = args.dtype or str(cfg["mxar.plane.dtype"])
    tdt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[dt]
    dev = torch.device("cuda", args.device)
    torch.cuda.set_device(dev)
    plane = C.hip.xgmi_plane(args.device, dtype_code(tdt), n, max_peers=int(cfg["mxar.plane.max-peers"]),
                             max_lag=int(cfg["mxar.plane.max-lag"]), grid=int(cfg["mxar.plane.grid"]),
                             timeout_s=float(cfg["mxar.plane.timeout"]), spin_us=int(cfg["mxar.plane.spin-us"]),
                             min_chunk=int(cfg["mxar.plane.min-chunk"]))

    def source(req):
        x = torch.empty(n, dtype=tdt, device=dev)
        C.hip.fill_iota(x.data_ptr(), n, float(req.iteration), dtype_code(tdt),
                        torch.cuda.current_stream(dev).cuda_stream)
        return x

    return plane, source


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("master", "worker", "bench"):
        print("usage: python -m akka_allreduce_1_amd {master|worker|bench} [args...]", file=sys.stderr)
        return 2
    if argv[0] == "bench":
        from .bench_cli import main as bench_main

        return bench_main(argv[1:])
    return master_main(argv[1:]) if argv[0] == "master" else worker_main(argv[1:])


if __name__ == "__main__":
    sys.exit(main())
