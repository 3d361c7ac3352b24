"""The examples run end to end (examples/README.md)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240, env=None):
    e = dict(os.environ, **(env or {}))
    return subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=e)


@pytest.mark.parametrize("plane", ["host", "loopback"])
def test_reference_demo(plane):
    extra = ["--th-reduce", "1", "--th-complete", "1"] if plane == "loopback" else []
    r = _run(["examples/reference_demo.py", "--plane", plane, "--rounds", "4"] + extra)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "finished" in r.stdout
    if plane == "loopback":  # exact: worker k's data is i + round + 1000 k
        assert "worker 0 round 3: [1006.0, 1008.0" in r.stdout, r.stdout


def test_train_dp_two_ranks_on_gloo():
    from akka_allreduce_1_amd.parallel.comm import free_port

    r = _run(["-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
              "--master-port", str(free_port()), "examples/train_dp.py", "--cpu", "--steps", "20", "--width", "64"],
             timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "replica max diff 0" in r.stdout, r.stdout


@pytest.mark.gpu
def test_reference_demo_on_the_gpu_round_engine():
    r = _run(["examples/reference_demo.py", "--plane", "gpu", "--rounds", "4", "--th-reduce", "1", "--th-complete", "1"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "worker 1 round 3: [1006.0, 1008.0" in r.stdout, r.stdout


@pytest.mark.gpu
def test_train_dp_one_gpu():
    from akka_allreduce_1_amd.parallel.comm import free_port

    r = _run(["-m", "torch.distributed.run", "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
              "--master-port", str(free_port()), "examples/train_dp.py", "--steps", "30", "--overlap", "auto"],
             timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "replica max diff 0" in r.stdout, r.stdout
    # the reducer measured its candidate schedules in the first steps and kept one
    assert "schedule overlap:" in r.stdout or "schedule serial:" in r.stdout, r.stdout


@pytest.mark.gpu
def test_native_gpu_job_two_workers_on_one_gpu():
    """examples/native_gpu_job.sh: master + 2 `mxar-gpu` worker processes (every worker on GPU 0),
    64 rounds of 1 M floats; the master finishes every round and both workers exit cleanly."""
    r = subprocess.run(["bash", "examples/native_gpu_job.sh", "2", str(1 << 20), "4096", "64"], cwd=ROOT,
                       capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, SHARE_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert '"rounds": 64' in r.stdout, r.stdout
    assert r.stdout.count("64 rounds completed") == 2, r.stdout
