"""The reference's deployment (README.md:3-7): one master process + N worker processes
joined through the seed node, over real TCP on 127.0.0.1, via the CLI entry points."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from akka_allreduce_1_amd.parallel.comm import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAST = ["--set", "mxar.cluster.failure-detector.heartbeat-interval=100ms",
        "--set", "mxar.cluster.failure-detector.acceptable-heartbeat-pause=1s",
        "--set", "mxar.cluster.auto-down-unreachable-after=1s", "--set", "mxar.loglevel=WARNING"]


@pytest.mark.slow
def test_master_and_two_worker_processes(tmp_path):
    port = free_port()
    seed = ["--set", f"mxar.cluster.seed-nodes=mxar.tcp://ClusterSystem@127.0.0.1:{port}"]
    exact = ["--set", "mxar.allreduce.th-reduce=1.0", "--set", "mxar.allreduce.th-complete=1.0",
             "--set", "mxar.allreduce.max-round=4"]
    env = dict(os.environ, PYTHONPATH=ROOT)
    py = [sys.executable, "-m", "akka_allreduce_1_amd"]
    ckpt = tmp_path / "ckpt.json"
    master = subprocess.Popen(py + ["master", str(port), "2", "10", "2", "--checkpoint", str(ckpt)] + seed + exact + FAST,
                              env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    workers = [subprocess.Popen(py + ["worker", "0", "10", "--print-outputs", "--metrics-json",
                                      str(tmp_path / f"w{i}.json"), "--trace-json", str(tmp_path / f"t{i}.json")]
                                + seed + FAST, env=env,
                                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for i in range(2)]
    try:
        mout, merr = master.communicate(timeout=60)
        assert master.returncode == 0, merr
        assert "finished 5 rounds" in mout, mout + merr  # rounds 0..maxRound (AllreduceMaster.scala:62)
        for w in workers:
            out, err = w.communicate(timeout=30)
            assert w.returncode == 0, err
            rows = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
            got = {r["iteration"]: r["data"] for r in rows}
            for it in range(5):  # rounds 0..maxRound
                np.testing.assert_array_equal(got[it], 2 * (np.arange(10) + it))
        assert json.loads(ckpt.read_text())["round"] == 4  # last completed round (0..maxRound)
        for i in range(2):
            m = json.loads((tmp_path / f"w{i}.json").read_text())
            assert m["worker"]["rounds_completed"] == 5 and m["cluster"]["frames_in"] > 0
            t = json.loads((tmp_path / f"t{i}.json").read_text())
            assert any(e["name"].startswith("complete r") for e in t["traceEvents"])
    finally:
        for p in [master] + workers:
            if p.poll() is None:
                p.kill()


def test_mxar_bench_gloo_two_ranks(tmp_path):
    """mxar-bench under torchrun (2 gloo ranks on CPU): one JSON row per size, busbw = algbw."""
    out = tmp_path / "rows.jsonl"
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), "-m", "akka_allreduce_1_amd", "bench", "--backend", "gloo",
           "--algos", "torch", "--sizes", "4K..64K", "--dtype", "fp32", "--iters", "3", "--json", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(l) for l in out.read_text().splitlines()]
    assert [x["bytes"] for x in rows] == [4096, 16384, 65536]
    for x in rows:
        assert x["P"] == 2 and x["p50_us"] > 0 and x["busbw_GBps"] == x["algbw_GBps"]


def test_native_master_and_two_workers(tmp_path):
    """The Python-free executables (csrc/tools/mxar_main.cc): the reference's deployment
    (one master + 2 workers, positional args), exact sums at th = 1, every process exits."""
    import socket
    import subprocess

    exe = os.path.join(ROOT, "akka_allreduce_1_amd", "mxar")
    if not os.path.exists(exe):
        pytest.skip("native executable not built (tools/build_native.py)")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    seed = f"mxar.tcp://ClusterSystem@127.0.0.1:{port}"
    common = ["--seeds", seed, "--loglevel", "ERROR"]
    # the master polls its host threads through the rounds (--spin-us), worker 0 sleeps at once
    master = subprocess.Popen([exe, "master", str(port), "2", "12", "2", "--th-reduce", "1", "--th-complete", "1",
                               "--max-round", "15", "--spin-us", "200"] + common, stdout=subprocess.PIPE, text=True)
    workers = [subprocess.Popen([exe, "worker", "0", "12"] + common + (["--spin-us", "0"] if k == 0 else []),
                                stdout=subprocess.PIPE, text=True)
               for k in range(2)]
    try:
        mout, _ = master.communicate(timeout=60)
        wouts = [w.communicate(timeout=60)[0] for w in workers]
    finally:
        for p in [master] + workers:
            if p.poll() is None:
                p.kill()
    assert master.returncode == 0 and "finished 16 rounds" in mout, mout
    for out, w in zip(wouts, workers):
        assert w.returncode == 0, out
        sums = {int(line.split()[3]): float(line.split()[5]) for line in out.splitlines() if " sum " in line}
        assert sorted(sums) == list(range(16)), out
        for r, v in sums.items():  # data[i] = i + r on both workers: sum 2 * (66 + 12 r)
            assert v == 2 * (66 + 12 * r), (r, v)


@pytest.mark.gpu
def test_native_gpu_workers(tmp_path):
    """`mxar-gpu worker --device 0` (csrc/tools/mxar_gpu.cc): the reference's deployment with
    each worker's rounds on the GPU - XgmiRoundPlane + PlaneWorkerActor, source filled by a
    kernel, no Python in any process. Two workers share GPU 0 through the xGMI arena."""
    import socket

    exe_dir = os.path.join(ROOT, "akka_allreduce_1_amd")
    exe, gpu_exe = os.path.join(exe_dir, "mxar"), os.path.join(exe_dir, "mxar-gpu")
    assert os.path.exists(gpu_exe), "mxar-gpu not built (tools/build_native.py)"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    n, rounds = 4096, 40
    common = ["--seeds", f"mxar.tcp://ClusterSystem@127.0.0.1:{port}", "--loglevel", "ERROR"]
    master = subprocess.Popen([exe, "master", str(port), "2", str(n), "512", "--th-reduce", "1", "--th-complete", "1",
                               "--max-lag", "2", "--max-round", str(rounds - 1)] + common,
                              stdout=subprocess.PIPE, text=True)
    workers = [subprocess.Popen([gpu_exe, "worker", "0", str(n), "--device", "0", "--max-peers", "2",
                                 "--plane-timeout", "20"] + common, stdout=subprocess.PIPE, text=True)
               for _ in range(2)]
    try:
        mout, _ = master.communicate(timeout=90)
        wouts = [w.communicate(timeout=60)[0] for w in workers]
    finally:
        for p in [master] + workers:
            if p.poll() is None:
                p.kill()
    assert master.returncode == 0 and f"finished {rounds} rounds" in mout, mout
    for out, w in zip(wouts, workers):
        assert w.returncode == 0, out
        sums = {int(line.split()[3]): float(line.split()[5]) for line in out.splitlines() if " sum " in line}
        assert sorted(sums) == list(range(rounds)), out
        for r, v in sums.items():  # data[i] = i + r on both workers
            assert v == 2 * (n * (n - 1) / 2 + n * r), (r, v)


@pytest.mark.slow
def test_worker_process_killed_survivors_reinitialised(tmp_path):
    """The reference's deployment over TCP, and one worker PROCESS is killed mid-job. The
    failure detector marks it unreachable and auto-downs it; the master's remote DeathWatch
    fires. With mxar.allreduce.reinit-on-loss the master re-initialises the two survivors
    at the current round, and they finish every round with sums of exactly two workers."""
    port = free_port()
    seed = ["--set", f"mxar.cluster.seed-nodes=mxar.tcp://ClusterSystem@127.0.0.1:{port}"]
    conf = ["--set", "mxar.allreduce.th-reduce=1.0", "--set", "mxar.allreduce.th-complete=1.0",
            "--set", "mxar.allreduce.max-round=120", "--set", "mxar.allreduce.reinit-on-loss=true"]
    env = dict(os.environ, PYTHONPATH=ROOT)
    py = [sys.executable, "-m", "akka_allreduce_1_amd"]
    master = subprocess.Popen(py + ["master", str(port), "3", "10", "2"] + seed + conf + FAST, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    outs = [open(tmp_path / f"w{i}.out", "w") for i in range(3)]
    workers = [subprocess.Popen(py + ["worker", "0", "10", "--print-outputs", "--source-delay-ms", "20"] + seed + FAST,
                                env=env, stdout=outs[i], stderr=subprocess.DEVNULL, text=True) for i in range(3)]
    try:
        t0 = time.time()
        while time.time() - t0 < 30:  # wait until rounds are flowing
            if sum(1 for _ in open(tmp_path / "w0.out")) >= 10:
                break
            time.sleep(0.1)
        workers[2].kill()
        mout, merr = master.communicate(timeout=90)
        assert master.returncode == 0, merr[-3000:]
        assert "finished 121 rounds" in mout, mout + merr[-3000:]
        for i in (0, 1):
            workers[i].wait(timeout=30)
            rows = [json.loads(l) for l in open(tmp_path / f"w{i}.out") if l.startswith("{")]
            got = {r["iteration"]: r["data"] for r in rows}
            np.testing.assert_array_equal(got[120], 2 * (np.arange(10) + 120))  # the two survivors
            np.testing.assert_array_equal(got[0], 3 * np.arange(10))            # all three before the loss
    finally:
        for p in [master] + workers:
            if p.poll() is None:
                p.kill()
        for f in outs:
            f.close()
