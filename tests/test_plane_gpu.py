"""The protocol-driven GPU round engine (csrc/runtime/plane_worker.*, csrc/hip/xgmi_plane.*,
csrc/hip/xgmi_threshold.hip) on one MI355X.

* exact rounds: master + P plane workers, thresholds 1, the reference's (unaligned) block
  ranges and maxChunkSize chunks: every round's output is the exact sum, every count is P;
* a deterministic straggler at th < 1 gives the SAME outputs and counts as the host
  WorkerCore (the reference's state machine) in the same scenario - including the
  reference's own-block-missing output of the straggler (its own ReduceBlocks are queued
  behind the completion);
* catch-up, GPU analogues of AllreduceSpec T13 (simple) and T14 (cold): rounds complete
  with what arrived when StartAllreduce runs more than maxLag ahead, no error word, no
  reset;
* the reference deployment: mxar-master + P `mxar-worker --device 0` processes, 101 rounds.
Worker k's data is i + iteration + 1000 k, so a chunk's sum identifies its contributors.
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from akka_allreduce_1_amd._native import C  # noqa: E402
from akka_allreduce_1_amd.engine import PlaneJob, iota_source  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = torch.device("cuda", 0)
F = np.float32


def layout(n, P, C_):
    step = -(-n // P)
    return step, -(-step // C_)


def expected(n, it, ranks):
    i = np.arange(n, dtype=np.float64)
    return sum(i + it + 1000.0 * k for k in ranks)


def subset_of(vals, lo, hi, it, cnt, P):
    """Which contributor subset (by sum of ids) produced vals[lo:hi] of round `it`; None if no
    subset of size cnt fits every element."""
    i = np.arange(lo, hi, dtype=np.float64)
    s = (vals[lo:hi].astype(np.float64) - cnt * (i + it)) / 1000.0
    if not np.allclose(s, s[0], atol=1e-3) or abs(s[0] - round(s[0])) > 1e-3:
        return None
    return int(round(s[0]))


@pytest.mark.parametrize("P,n,chunk,dtype", [(2, 10, 2, torch.float32), (2, 10007, 333, torch.float32),
                                             (3, 30000, 1000, torch.float32), (3, 4096, 512, torch.bfloat16)])
def test_plane_rounds_exact_at_threshold_one(P, n, chunk, dtype):
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=1.0, th_complete=1.0, max_lag=1, max_round=12, dtype=dtype,
                   timeout_s=20.0)
    try:
        job.run(timeout=120)
        assert job.rounds["n"] == 13
        step, nch = layout(n, P, chunk)
        for k in range(P):
            st = job.system.plane_worker_state(job.workers[k])
            assert st["stats"]["plane_errors"] == 0 and st["stats"]["rounds_completed"] == 13, st
            for it in range(13):
                data, counts = job.outputs[k][it]
                assert data.dtype == dtype and data.numel() == n
                got = data.float().cpu().numpy()
                if dtype == torch.float32:
                    np.testing.assert_array_equal(got, expected(n, it, range(P)), err_msg=f"worker {k} round {it}")
                else:  # fp32 sum of the bf16 inputs, one rounding
                    ar = torch.arange(n, dtype=torch.float64)
                    ref = sum((ar + it + 1000.0 * j).to(dtype).double() for j in range(P)).numpy()
                    assert np.all(np.abs(got - ref) <= np.abs(ref) * 2.0 ** -8 + 1e-6), (k, it)
                assert len(counts) == P * job.planes[k].chunks
                assert all(c == P for c in counts), counts
        assert job.planes[0].stats.launches == 13
    finally:
        job.shutdown()


def _host_outputs(P, n, chunk, th, straggler, delay, rounds):
    """The same scenario on the host WorkerCore (the reference's state machine)."""
    system = C.ActorSystem("Host", False)
    done = {}
    fin = __import__("threading").Event()
    outs = [dict() for _ in range(P)]

    def src(k):
        base = np.arange(n, dtype=F) + F(1000 * k)

        def f(req):
            if k == straggler:
                time.sleep(delay)
            return C.AllReduceInput(base + F(req.iteration))
        return f

    def sink(k):
        def f(out):
            outs[k][out.iteration] = (np.asarray(out.data).copy(), list(out.count))
        return f

    master = system.master(P, 1.0, th, th, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set())
    ws = [system.worker(src(k), sink(k), f"w{k}") for k in range(P)]
    for w in ws:
        master.tell(C.MemberUp(w, "worker", ""), None)
    assert fin.wait(60)
    system.await_idle(5.0)
    system.shutdown()
    del done
    return outs


def test_straggler_matches_host_worker_core():
    P, n, chunk, rounds = 3, 3000, 250, 4
    th = 2.0 / 3.0
    straggler, delay = 2, 0.3
    host = _host_outputs(P, n, chunk, th, straggler, delay, rounds)

    def slow(source):
        def f(req):
            time.sleep(delay)
            return source(req)
        return f

    srcs = [iota_source(n, DEV, torch.float32, 1000.0 * k) for k in range(P)]
    srcs[straggler] = slow(srcs[straggler])
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=th, th_complete=th, max_lag=1, max_round=rounds - 1,
                   sources=srcs, timeout_s=20.0)
    try:
        job.run(timeout=120)
        for k in range(P):
            for it in range(rounds):
                g, gc = job.outputs[k][it]
                h, hc = host[k][it]
                assert gc == hc, (k, it, gc, hc)
                np.testing.assert_array_equal(g.float().cpu().numpy(), h, err_msg=f"worker {k} round {it}")
        # the shape of the result, as the reference defines it
        step, nch = layout(n, P, chunk)
        g, gc = job.outputs[straggler][1]
        assert gc[straggler * nch:(straggler + 1) * nch] == [0] * nch  # own block missing (queued behind)
        assert not g[straggler * step:].float().abs().sum().item()
        assert gc[:2 * nch] == [2] * (2 * nch)
    finally:
        job.shutdown()


class _Gate:
    """A causal straggler: its fetch of round r waits until every other worker's sink has
    received round r. Its data then arrives strictly after the others completed the round,
    whatever the host or device speed - a deterministic scenario for both engines."""

    def __init__(self, others: int):
        import threading

        self.others = others
        self.cv = threading.Condition()
        self.seen: dict[int, int] = {}

    def sink(self, it: int) -> None:
        with self.cv:
            self.seen[it] = self.seen.get(it, 0) + 1
            self.cv.notify_all()

    def wait(self, it: int) -> None:
        with self.cv:
            assert self.cv.wait_for(lambda: self.seen.get(it, 0) >= self.others, timeout=300), it


def _host_outputs_gated(P, n, chunk, th, straggler, rounds):
    import threading

    system = C.ActorSystem("Host", False)
    fin = threading.Event()
    outs = [dict() for _ in range(P)]
    gate = _Gate(P - 1)

    def src(k):
        base = np.arange(n, dtype=F) + F(1000 * k)

        def f(req):
            if k == straggler:
                gate.wait(req.iteration)
            return C.AllReduceInput(base + F(req.iteration))
        return f

    def sink(k):
        def f(out):
            outs[k][out.iteration] = (np.asarray(out.data).copy(), list(out.count))
            if k != straggler:
                gate.sink(out.iteration)
        return f

    master = system.master(P, 1.0, th, th, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set())
    ws = [system.worker(src(k), sink(k), f"w{k}") for k in range(P)]
    for w in ws:
        master.tell(C.MemberUp(w, "worker", ""), None)
    assert fin.wait(600)
    system.await_idle(5.0)
    system.shutdown()
    return outs


def fine_chunk_parity(n: int, P: int = 3, chunk: int = 2, rounds: int = 2, log=None) -> dict:
    """The GPU round engine vs the host WorkerCore with a maxChunkSize far below the 1 KiB
    flag granularity, a causal straggler and th = 2/3: bit-identical outputs and counts
    (tools/fine_chunk_parity.py runs it at 1 M floats)."""
    th = 2.0 / 3.0
    straggler = 2
    lvl = C.get_log_level()
    C.set_log_level("ERROR")  # the host run logs every outdated 2-float ReduceBlock
    t0 = time.perf_counter()
    try:
        host = _host_outputs_gated(P, n, chunk, th, straggler, rounds)
    finally:
        C.set_log_level(lvl)
    t_host = time.perf_counter() - t0
    if log:
        log(f"host WorkerCore: {t_host:.1f} s")
    gate = _Gate(P - 1)

    def gated(source):
        def f(req):
            gate.wait(req.iteration)
            return source(req)
        return f

    srcs = [iota_source(n, DEV, torch.float32, 1000.0 * k) for k in range(P)]
    srcs[straggler] = gated(srcs[straggler])
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=th, th_complete=th, max_lag=1, max_round=rounds - 1,
                   sources=srcs, timeout_s=60.0,
                   on_output=lambda k, out: gate.sink(out.iteration) if k != straggler else None)
    try:
        t0 = time.perf_counter()
        job.run(timeout=300)
        t_gpu = time.perf_counter() - t0
        if log:
            log(f"GPU round engine: {t_gpu:.1f} s")
        step, nch = layout(n, P, chunk)
        assert job.planes[0].chunks == nch and job.planes[0].stats.coarsened == 0
        for k in range(P):
            for it in range(rounds):
                g, gc = job.outputs[k][it]
                h, hc = host[k][it]
                assert len(gc) == P * nch
                assert gc == hc, (k, it, [i for i in range(len(gc)) if gc[i] != hc[i]][:8])
                np.testing.assert_array_equal(g.float().cpu().numpy(), h, err_msg=f"worker {k} round {it}")
        g, gc = job.outputs[0][0]
        return {"n": n, "P": P, "max_chunk_size": chunk, "chunks_per_block": nch, "rounds": rounds,
                "th": th, "identical": True, "host_s": round(t_host, 1), "gpu_s": round(t_gpu, 1),
                "fast_worker_counts_round0": [int(sum(1 for c in gc[j * nch:(j + 1) * nch] if c)) for j in range(P)]}
    finally:
        job.shutdown()


def test_fine_chunks_keep_reference_semantics():
    """maxChunkSize below the 1 KiB flag granularity (the reference's default 2-float chunk,
    43 691 chunks per block at 256 K floats - tools/fine_chunk_parity.py runs 1 M): the plane
    keeps one flag, count and threshold decision per reference chunk (min_chunk), so a
    causal straggler at th = 2/3 gives bit-identical outputs and counts to the host
    WorkerCore (DataBuffer.scala:12,28-29,69-75; AllreduceWorker.scala:56-57). The fast
    workers complete each round with exactly the two fast blocks."""
    # 3 equal blocks of 87 382 floats: (2/3 * 3 * nch) is exactly the two fast blocks, so the
    # rounds' contents do not depend on which of two simultaneous last arrivals wins
    r = fine_chunk_parity(3 * 87382)
    nch = r["chunks_per_block"]
    assert r["fast_worker_counts_round0"][:2] == [nch, nch] and r["fast_worker_counts_round0"][2] == 0


def test_fine_chunks_coarsen_at_threshold_one():
    """Without a fine flag table (min_chunk=0) a 2-float maxChunkSize runs at thresholds 1 in
    coarse kernel chunks - the sums cannot change - with the counts still reported per
    reference chunk."""
    P, n, chunk = 2, 1 << 20, 2
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=1.0, th_complete=1.0, max_lag=1, max_round=2,
                   timeout_s=20.0, min_chunk=0)
    try:
        job.run(timeout=120)
        step, nch = layout(n, P, chunk)
        assert job.planes[0].chunks == nch and job.planes[0].stats.coarsened == 1
        for k in range(P):
            data, counts = job.outputs[k][2]
            np.testing.assert_array_equal(data.float().cpu().numpy(), expected(n, 2, range(P)))
            assert len(counts) == P * nch and all(c == P for c in counts)
    finally:
        job.shutdown()


def _consistent(job, P, n, chunk, counts_ok):
    """Every chunk of every output is the sum of `count` distinct workers (0 -> zeros)."""
    step, nch = layout(n, P, chunk)
    for k in range(P):
        for it, (data, counts) in job.outputs[k].items():
            v = data.float().cpu().numpy()
            for j in range(P):
                for c in range(nch):
                    lo, hi = j * step + c * chunk, min(n, j * step + min(step, (c + 1) * chunk))
                    if lo >= hi:
                        continue
                    cnt = counts[j * nch + c]
                    assert cnt in counts_ok, (k, it, j, c, cnt)
                    if cnt == 0:
                        assert not np.any(v[lo:hi]), (k, it, j, c)
                    else:
                        assert subset_of(v, lo, hi, it, cnt, P) is not None, (k, it, j, c, cnt)


def test_simple_catchup_forces_rounds_without_errors():
    """T13 analogue (AllreduceSpec.scala:535-559): the straggler stalls, the fast workers'
    reduces fire (thReduce 2/3) but their rounds cannot complete (thComplete 1); the master's
    round deadline keeps starting rounds, StartAllreduce(r) with r - maxLag > round forces the
    stuck round to complete with what arrived (the straggler's block: zeros, count 0). When
    the straggler wakes, the fast workers' FORCE requests complete its stale round at once."""
    P, n, chunk = 3, 6000, 500
    srcs = [iota_source(n, DEV, torch.float32, 1000.0 * k) for k in range(P)]
    base = srcs[2]

    def stall(req):
        if req.iteration == 0:
            time.sleep(2.0)
        return base(req)

    srcs[2] = stall
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=2.0 / 3.0, th_complete=1.0, max_lag=1, max_round=8,
                   sources=srcs, round_timeout_ms=250, timeout_s=30.0)
    try:
        job.run(timeout=180)
        st = job.state()
        for k, w in enumerate(st["workers"]):
            assert w["stats"]["plane_errors"] == 0, (k, w)  # no ERR_TIMEOUT_LAG, no timeouts
            assert w["round"] == 9, (k, w)  # every round 0..maxRound completed
        assert sum(w["stats"]["forced_completions"] for w in st["workers"][:2]) > 0, st
        _consistent(job, P, n, chunk, {0, 1, 2, 3})  # 1: a forced reduce of what had arrived
        step, nch = layout(n, P, chunk)
        # round 0 of a fast worker: forced; the fast blocks made it (count 2), the straggler's not
        data, counts = job.outputs[0][0]
        assert counts[:2 * nch] == [2] * (2 * nch) and counts[2 * nch:] == [0] * nch, counts
    finally:
        job.shutdown()


def test_cold_catchup():
    """T14 analogue (AllreduceSpec.scala:561-584): worker 2 first hears of the job at
    StartAllreduce(4) (maxLag 1): rounds 0..2 are completed cold - nothing of its own, what
    the peers delivered - and 3..4 run normally; the fast workers, held at their lag gate,
    resume as soon as the cold rounds publish progress."""
    P, n, chunk = 3, 6000, 500
    th = 2.0 / 3.0
    system = C.ActorSystem("Cold", False)
    probe = system.probe("master")
    planes = [C.hip.xgmi_plane(0, C.hip.DType.F32, n, max_peers=P, max_lag=1, grid=64, timeout_s=30.0)
              for _ in range(P)]
    outs = [dict() for _ in range(P)]

    def sink(k):
        return lambda out: outs[k].__setitem__(out.iteration, (out.data, list(out.count)))

    ws = [system.plane_worker(iota_source(n, DEV, torch.float32, 1000.0 * k), sink(k), planes[k], f"w{k}")
          for k in range(P)]
    try:
        wmap = {k: ws[k] for k in range(P)}
        descs = {k: planes[k].descriptor for k in range(P)}
        for k in range(P):
            m = C.InitWorkers(wmap, probe, k, th, th, 1, n, chunk, epoch=1)
            m.planes = descs
            ws[k].tell(m, None)
        got = set()

        def collect(want, limit):
            t0 = time.time()
            while not want <= got and time.time() - t0 < limit:
                e = probe.receive(1.0)
                if e is not None and isinstance(e[0], C.CompleteAllreduce):
                    got.add((e[0].srcId, e[0].round))
            return want <= got

        # the fast workers run rounds 0 and 1 one at a time, as the master would start them (a
        # StartAllreduce(r) that arrives while round r - maxLag - 1 is still open forces it -
        # the reference's catch-up rule); round 2 then waits at its lag gate for worker 2
        for r in (0, 1):
            for k in (0, 1):
                ws[k].tell(C.StartAllreduce(r, 1), None)
            assert collect({(0, r), (1, r)}, 30), sorted(got)
        for r in (2, 3, 4):
            for k in (0, 1):
                ws[k].tell(C.StartAllreduce(r, 1), None)
        time.sleep(0.3)
        ws[2].tell(C.StartAllreduce(4, 1), None)  # worker 2's first StartAllreduce
        collect({(k, r) for k in range(P) for r in range(5)}, 60)
        assert got == {(k, r) for k in range(P) for r in range(5)}, sorted(got)
        st = system.plane_worker_state(ws[2])
        assert st["stats"]["cold_rounds"] == 3 and st["stats"]["plane_errors"] == 0, st
        for k in (0, 1):
            assert system.plane_worker_state(ws[k])["stats"]["plane_errors"] == 0
        step, nch = layout(n, P, chunk)
        for it in (0, 1):  # cold rounds whose fast blocks were reduced before worker 2 started
            data, counts = outs[2][it]
            assert counts[:2 * nch] == [2] * (2 * nch), (it, counts)
            assert counts[2 * nch:] == [0] * nch, (it, counts)  # nothing of its own in a cold round
            v = data.float().cpu().numpy()
            np.testing.assert_array_equal(v[:2 * step], expected(n, it, (0, 1))[:2 * step])
            assert not np.any(v[2 * step:])

        class J:
            outputs = outs
        _consistent(J, P, n, chunk, {0, 1, 2, 3})  # 1: a forced reduce of what had arrived
    finally:
        system.shutdown()


def test_plane_stale_epoch_and_reinit():
    """A re-initialisation (new membership epoch, startRound) lays the same arenas out again:
    the new epoch's round epochs start above the old ones (InitWorkers.roundBase), so flags
    the old epoch left behind are never taken for new arrivals."""
    P, n, chunk = 2, 5000, 700
    job = PlaneJob(P, n, max_chunk_size=chunk, max_round=3, timeout_s=20.0)
    try:
        job.run(timeout=60)
        # second epoch by hand: same planes, resume at round 7, round base above epoch 1
        probe = job.system.probe("m2")
        wmap = {k: job.workers[k] for k in range(P)}
        for k in range(P):
            m = C.InitWorkers(wmap, probe, k, 1.0, 1.0, 1, n, chunk, epoch=2, startRound=7)
            m.planes = {j: job.planes[j].descriptor for j in range(P)}
            m.roundBase = 100
            job.workers[k].tell(m, None)
        got = set()
        for r in (7, 8, 9):  # one round at a time, as a master starts them
            for k in range(P):
                job.workers[k].tell(C.StartAllreduce(r, 2), None)
            t0 = time.time()
            while not {(0, r), (1, r)} <= got and time.time() - t0 < 30:
                e = probe.receive(1.0)
                if e is not None and isinstance(e[0], C.CompleteAllreduce):
                    assert e[0].epoch == 2
                    got.add((e[0].srcId, e[0].round))
        assert got == {(k, r) for k in range(P) for r in (7, 8, 9)}
        for k in range(P):
            assert job.system.plane_worker_state(job.workers[k])["stats"]["plane_errors"] == 0
        for it in (7, 8, 9):
            data, counts = job.outputs[0][it]
            np.testing.assert_array_equal(data.cpu().numpy(), expected(n, it, range(P)))
    finally:
        job.shutdown()


@pytest.mark.parametrize("P,n,chunk", [(2, 10, 2), (3, 3000, 100)])
def test_cli_master_and_gpu_worker_processes(tmp_path, P, n, chunk):
    """The reference's deployment (README.md:3-7) on the GPU: mxar-master + P
    `mxar-worker --device 0` processes (plane descriptors in the cluster join, relayed in
    InitWorkers), 101 rounds at th = 1, exact sums on every worker."""
    from akka_allreduce_1_amd.parallel.comm import free_port

    port = free_port()
    fast = ["--set", "mxar.cluster.failure-detector.heartbeat-interval=100ms",
            "--set", "mxar.cluster.failure-detector.acceptable-heartbeat-pause=3s",
            "--set", "mxar.cluster.auto-down-unreachable-after=5s", "--set", "mxar.loglevel=WARNING"]
    seed = ["--set", f"mxar.cluster.seed-nodes=mxar.tcp://ClusterSystem@127.0.0.1:{port}"]
    exact = ["--set", "mxar.allreduce.th-reduce=1.0", "--set", "mxar.allreduce.th-complete=1.0"]
    gpu = ["--device", "0", "--set", "mxar.plane.grid=32", "--set", f"mxar.plane.max-peers={P}",
           "--set", "mxar.plane.timeout=20"]
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    py = [sys.executable, "-m", "akka_allreduce_1_amd"]
    master = subprocess.Popen(py + ["master", str(port), str(P), str(n), str(chunk), "--metrics-json",
                                    str(tmp_path / "m.json")] + seed + exact + fast,
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    # worker output goes to files: ~P x 101 JSON rows of n floats would fill a pipe nobody reads
    wout = [open(tmp_path / f"w{i}.out", "w") for i in range(P)]
    werr = [open(tmp_path / f"w{i}.err", "w") for i in range(P)]
    workers = [subprocess.Popen(py + ["worker", "0", str(n), "--print-outputs", "--metrics-json",
                                      str(tmp_path / f"w{i}.json")] + gpu + seed + fast, env=env,
                                stdout=wout[i], stderr=werr[i], text=True) for i in range(P)]
    try:
        try:
            mout, merr = master.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for p in [master] + workers:
                p.kill()
            logs = [master.communicate()[1][-2500:]] + [(tmp_path / f"w{i}.err").read_text()[-2500:] for i in range(P)]
            pytest.fail("job did not finish; stderr tails:\n" + "\n----\n".join(logs))
        assert master.returncode == 0, merr[-3000:]
        assert "finished 101 rounds" in mout, mout + merr[-3000:]
        for i, w in enumerate(workers):
            w.wait(timeout=60)
            out, err = (tmp_path / f"w{i}.out").read_text(), (tmp_path / f"w{i}.err").read_text()
            assert w.returncode == 0, err[-3000:]
            rows = [json.loads(line) for line in out.splitlines() if line.startswith("{")]
            got = {r["iteration"]: r for r in rows}
            assert sorted(got) == list(range(101)), sorted(got)[:5]
            for it in range(101):  # every worker: data[i] = i + iteration
                np.testing.assert_array_equal(got[it]["data"], P * (np.arange(n) + it))
                assert set(got[it]["count"]) == {P}
            m = json.loads((tmp_path / f"w{i}.json").read_text())
            assert m["worker"]["rounds_completed"] == 101 and m["worker"]["plane_errors"] == 0, m["worker"]
            assert m["worker"]["plane_launches"] == 101
    finally:
        for p in [master] + workers:
            if p.poll() is None:
                p.kill()
        for f in wout + werr:
            f.close()


def test_worker_loss_reinitialises_the_survivors():
    """A plane worker dies mid-job (its actor stops; its plane abandons its rounds). With
    reinitOnLoss the master re-initialises the two survivors at the current round: their
    planes abandon the old epoch's rounds (a round still at its lag gate, waiting for the
    lost worker, delivers nothing instead of waiting out the kernel deadline), lay the
    arena out for P = 2 and finish every round exactly."""
    P, n, chunk, rounds, victim = 3, 3000, 250, 30, 2
    started = __import__("threading").Event()

    def slow(k):
        base = iota_source(n, DEV, torch.float32, 1000.0 * k)

        def f(req):
            time.sleep(0.01)
            if req.iteration >= 5:
                started.set()
            return base(req)
        return f

    job = PlaneJob(P, n, max_chunk_size=chunk, max_round=rounds - 1, sources=[slow(k) for k in range(P)],
                   timeout_s=20.0, reinit_on_loss=True)
    try:
        t0 = time.time()
        job.start()
        assert started.wait(30)
        job.workers[victim].tell(C.PoisonPill(), None)
        assert job.finished.wait(60), job.state()
        assert time.time() - t0 < 20, "a round waited for the lost worker until its kernel deadline"
        for p in job.planes[:2]:
            p.drain()
        st = job.system.master_state(job.master)
        assert st["loss_reinits"] == 1 and st["numWorkers"] == 2, st
        for k in (0, 1):
            w = job.system.plane_worker_state(job.workers[k])
            assert w["stats"]["plane_errors"] == 0, w
            data, counts = job.outputs[k][rounds - 1]
            np.testing.assert_array_equal(data.cpu().numpy(), expected(n, rounds - 1, (0, 1)))
            assert all(c == 2 for c in counts), counts
    finally:
        job.shutdown()


def test_lost_worker_replaced_by_a_new_plane_worker():
    """Elastic membership on the GPU round engine: worker 2 dies, the survivors continue
    (reinitOnLoss), a replacement worker with a NEW plane (arena) joins and everyone is
    re-initialised at the current round (resumeOnJoin); the job finishes exactly with three."""
    P, n, chunk, rounds = 3, 3000, 250, 40
    system = C.ActorSystem("ElasticGpu", False)
    fin = __import__("threading").Event()
    outs = [dict() for _ in range(P + 1)]
    progressed = {"r": -1}

    def src(k):
        base = iota_source(n, DEV, torch.float32, 1000.0 * min(k, 2))

        def f(req):
            time.sleep(0.01)
            progressed["r"] = max(progressed["r"], req.iteration)
            return base(req)
        return f

    planes = []
    master = system.master(P, 1.0, 1.0, 1.0, 1, n, rounds - 1, chunk, on_finished=lambda r: fin.set(),
                           reinitOnLoss=True, resumeOnJoin=True)

    def join(k):
        planes.append(C.hip.xgmi_plane(0, C.hip.DType.F32, n, max_peers=4, max_lag=1, grid=64, timeout_s=20.0))
        w = system.plane_worker(src(k), (lambda k: lambda out: outs[k].__setitem__(out.iteration, (out.data, list(out.count))))(k),
                                planes[-1], f"w{k}")
        master.tell(C.MemberUp(w, "worker", "", planes[-1].descriptor), None)
        return w

    try:
        ws = [join(k) for k in range(P)]
        t0 = time.time()
        while progressed["r"] < 5 and time.time() - t0 < 30:
            time.sleep(0.01)
        ws[2].tell(C.PoisonPill(), None)
        while system.master_state(master)["loss_reinits"] < 1 and time.time() - t0 < 30:
            time.sleep(0.01)
        join(3)
        assert fin.wait(60), system.master_state(master)
        assert time.time() - t0 < 30, "a round waited out a kernel deadline"
        for p in planes:
            p.drain()
        st = system.master_state(master)
        assert st["loss_reinits"] == 1 and st["join_reinits"] == 1 and st["numWorkers"] == 3, st
        data, counts = outs[0][rounds - 1]
        np.testing.assert_array_equal(data.cpu().numpy(), expected(n, rounds - 1, (0, 1, 2)))
        assert all(c == 3 for c in counts), counts
    finally:
        system.shutdown()
        planes.clear()
        __import__("gc").collect()


# ---- split chunks: fewer protocol chunks than workgroups (csrc/hip/xgmi_threshold.hip) ----
# A chunk of >= 2 x 64 KiB is cut into slices, one workgroup each; it stays ONE threshold
# decision (contributor set, take, count), so every property below is per whole chunk.

@pytest.mark.parametrize("P,n,chunk,dtype", [(2, (1 << 20) + 7, (1 << 19) + 9, torch.float32),
                                             (3, 600001, 100000, torch.float32),
                                             (2, 1 << 20, 1 << 18, torch.bfloat16)])
def test_split_chunks_exact_at_threshold_one(P, n, chunk, dtype):
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=1.0, th_complete=1.0, max_lag=1, max_round=7, dtype=dtype,
                   timeout_s=20.0)
    try:
        job.run(timeout=120)
        assert job.rounds["n"] == 8
        for k in range(P):
            st = job.system.plane_worker_state(job.workers[k])
            assert st["stats"]["plane_errors"] == 0, st
            for it in range(8):
                data, counts = job.outputs[k][it]
                got = data.float().cpu().numpy()
                if dtype == torch.float32:
                    np.testing.assert_array_equal(got, expected(n, it, range(P)), err_msg=f"worker {k} round {it}")
                else:
                    ar = torch.arange(n, dtype=torch.float64)
                    ref = sum((ar + it + 1000.0 * j).to(dtype).double() for j in range(P)).numpy()
                    assert np.all(np.abs(got - ref) <= np.abs(ref) * 2.0 ** -8 + 1e-6), (k, it)
                # P for every chunk that exists; 0 past the end of a short last block (600001 / 3:
                # blocks of 3, 3 and 2 chunks), as the host WorkerCore reports it
                step, nch = layout(n, P, chunk)
                want = [P if min(step, n - j * step) > c * chunk else 0 for j in range(P) for c in range(nch)]
                assert list(counts) == want, counts
    finally:
        job.shutdown()


def test_split_straggler_matches_host_worker_core():
    """The reference-order accounting (snapshot, tickets) with split chunks: the same outputs
    and counts as the host WorkerCore for a deterministic straggler."""
    P, n, chunk, rounds = 3, 300000, 50000, 4
    th = 2.0 / 3.0
    straggler, delay = 2, 0.3
    host = _host_outputs(P, n, chunk, th, straggler, delay, rounds)

    def slow(source):
        def f(req):
            time.sleep(delay)
            return source(req)
        return f

    srcs = [iota_source(n, DEV, torch.float32, 1000.0 * k) for k in range(P)]
    srcs[straggler] = slow(srcs[straggler])
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=th, th_complete=th, max_lag=1, max_round=rounds - 1,
                   sources=srcs, timeout_s=20.0)
    try:
        job.run(timeout=120)
        for k in range(P):
            for it in range(rounds):
                g, gc = job.outputs[k][it]
                h, hc = host[k][it]
                assert gc == hc, (k, it, gc, hc)
                np.testing.assert_array_equal(g.float().cpu().numpy(), h, err_msg=f"worker {k} round {it}")
    finally:
        job.shutdown()


def test_split_catchup_keeps_chunks_whole():
    """Forced completions race the slices of a chunk: whatever each round ends with, every
    chunk is the sum of ONE contributor subset of size `count` over all its slices (or zeros
    with count 0) - never half one decision and half another."""
    P, n, chunk = 3, 600000, 50000
    srcs = [iota_source(n, DEV, torch.float32, 1000.0 * k) for k in range(P)]
    base = srcs[2]

    def stall(req):
        if req.iteration in (0, 3):
            time.sleep(1.0)
        return base(req)

    srcs[2] = stall
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=2.0 / 3.0, th_complete=2.0 / 3.0, max_lag=1, max_round=8,
                   sources=srcs, round_timeout_ms=250, timeout_s=30.0)
    try:
        job.run(timeout=180)
        st = job.state()
        for k, w in enumerate(st["workers"]):
            assert w["stats"]["plane_errors"] == 0, (k, w)
            assert w["round"] == 9, (k, w)
        _consistent(job, P, n, chunk, {0, 1, 2, 3})
    finally:
        job.shutdown()


def test_split_matches_unsplit_outputs():
    """Same job, split on and off: identical outputs and counts at thresholds 1."""
    P, n, chunk = 2, 1 << 20, 1 << 18
    res = []
    for split in (True, False):
        job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=1, max_round=3, timeout_s=20.0, split=split)
        try:
            job.run(timeout=120)
            res.append({(k, it): (d.cpu().numpy().copy(), list(c)) for k in range(P)
                        for it, (d, c) in job.outputs[k].items()})
        finally:
            job.shutdown()
    assert res[0].keys() == res[1].keys()
    for key in res[0]:
        np.testing.assert_array_equal(res[0][key][0], res[1][key][0], err_msg=str(key))
        assert res[0][key][1] == res[1][key][1]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_tensor_sources_and_native_keep_last_sink(dtype):
    """GPU tensors as dataSources (hip.tensor_source: fetched natively, ordered after torch's
    stream) and the native keep-last sink: no Python per round, outputs exact."""
    P, n, rounds = 2, (1 << 20) + 3, 7
    xs = [torch.empty(n, dtype=dtype, device=DEV) for _ in range(P)]
    job = PlaneJob(P, n, max_chunk_size=4096, max_lag=1, max_round=rounds - 1, dtype=dtype, sources=xs,
                   keep_outputs=False, keep_last=True, timeout_s=20.0)
    try:
        for k, x in enumerate(xs):  # queued on torch's stream, no sync: the source's event orders it
            x.copy_(torch.arange(n, device=DEV, dtype=torch.float32).remainder_(97).add_(k).to(dtype))
        job.run(timeout=120)
        ref = (xs[0].float() + xs[1].float()).to(dtype)
        for k in range(P):
            o = job.last_output(k)
            assert o.iteration == rounds - 1 and all(c == P for c in o.count)
            assert torch.equal(o.data, ref), k
            st = job.system.plane_worker_state(job.workers[k])
            assert st["stats"]["plane_errors"] == 0 and st["stats"]["rounds_completed"] == rounds, st
        assert len(job.stamps) == rounds
    finally:
        job.shutdown()


def test_bridge_client_drives_gpu_rounds():
    """The control bridge (docs/BRIDGE.md) drives the xGMI round engine: a socket client plays
    AllreduceMaster's round loop (StartAllreduce -> barrier -> next), the plane workers run one
    threshold-kernel launch per round on the GPU, every output exact."""
    from akka_allreduce_1_amd.bridge import BridgeClient

    P, n, chunk, rounds = 2, 10007, 333, 12
    job = PlaneJob(P, n, max_chunk_size=chunk, max_round=rounds - 1, timeout_s=20.0, bridge_port=0,
                   external_rounds=True)
    try:
        job.start()
        with BridgeClient("127.0.0.1", job.bridge_port) as b:
            assert b.wait_for("InitWorkers")["workers"] == [0, 1]
            time.sleep(0.1)
            assert job.planes[0].stats.launches == 0  # nothing launches before the client starts a round
            b.drive(range(rounds), timeout=30)
            b.wait_for("AllreduceFinished", rounds=rounds)
        assert job.finished.wait(10)
        for p in job.planes:
            p.drain()
        job.system.await_idle(10.0)
        for k in range(P):
            for it in range(rounds):
                data, counts = job.outputs[k][it]
                np.testing.assert_array_equal(data.float().cpu().numpy(), expected(n, it, range(P)))
                assert all(c == P for c in counts)
        assert job.planes[0].stats.launches == rounds
    finally:
        job.shutdown()


def test_akka_client_drives_gpu_rounds():
    """The north star's "an existing Akka client can drive it" on the GPU engine: an Akka 2.5
    client (akka_allreduce_1_amd/akka_remote.py) associates with the master's akka.tcp
    endpoint (docs/AKKA_WIRE.md), resolves /user/master with Identify, sends Java-serialized
    StartAllreduce(r) and counts CompleteAllreduce(srcId, r) as AllreduceMaster.scala:58-67
    does; the plane workers run one threshold-kernel launch per round, every output exact."""
    from akka_allreduce_1_amd import akka_remote as ar

    P, n, chunk, rounds = 2, 10007, 333, 10
    job = PlaneJob(P, n, max_chunk_size=chunk, max_round=rounds - 1, timeout_s=20.0, bridge_port=0,
                   external_rounds=True)
    try:
        job.start()
        ep = C.akka.start_endpoint(job.master)
        with ar.AkkaClient("127.0.0.1", ep.port) as cl:
            ref = cl.identify(["user", "master"])
            assert ref == ep.master_path
            for r in range(rounds):
                deadline = time.time() + 20
                while True:  # a start before the workers' InitWorkers is refused: retry
                    cl.start_allreduce(r, to=ref)
                    try:
                        seen = set()
                        while len(seen) < P:
                            src, rr, cls, suid = cl.complete_allreduce(timeout=2 if r == 0 and not seen else 20)
                            assert cls.endswith(".CompleteAllreduce") and suid == ep.suid_complete
                            if rr == r:
                                seen.add(src)
                        break
                    except TimeoutError:
                        assert r == 0 and time.time() < deadline
        assert job.finished.wait(10)
        for p in job.planes:
            p.drain()
        job.system.await_idle(10.0)
        for k in range(P):
            for it in range(rounds):
                data, counts = job.outputs[k][it]
                np.testing.assert_array_equal(data.float().cpu().numpy(), expected(n, it, range(P)))
                assert all(c == P for c in counts)
        assert ep.stats()["suid_mismatches"] == 0
    finally:
        job.shutdown()


def _dist_job_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist

    from akka_allreduce_1_amd.engine import distributed_plane_job

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    try:
        n, rounds = 100_003, 8
        x = torch.arange(n, dtype=torch.float32, device=DEV) + 1000.0 * rank  # exact in fp32
        want = sum(torch.arange(n, dtype=torch.float64) + 1000.0 * k for k in range(world)).float()
        for external in (False, True):
            res = distributed_plane_job(n, x, max_chunk_size=4001, dtype=torch.float32, rounds=rounds,
                                        grid=max(8, 512 // world), keep_last=True, timeout_s=60.0,
                                        external_client=external)
            y = res["last"]
            ok = bool(res["ok"] and y is not None and y.iteration == rounds - 1
                      and torch.equal(y.data.cpu(), want))
            out.append((external, ok, len(res["stamps"]) if rank == 0 else rounds))
    except Exception as e:  # report, never hang the parent
        out.append(("error", False, repr(e)))
    q.put((rank, out))
    dist.destroy_process_group()


def test_distributed_plane_job_master_and_bridge_driven():
    """One plane worker per process (the N > 1 bench's protocol shape, here 2 processes on one
    GPU): the master on rank 0 drives the rounds, then a control-bridge client on rank 0 does
    (docs/BRIDGE.md); every rank's last output is the exact sum both times."""
    import multiprocessing as mp

    from akka_allreduce_1_amd.parallel import free_port

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_dist_job_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    for rank, out in res:
        assert [o[:2] for o in out] == [(False, True), (True, True)], (rank, out)
        assert all(o[2] == 8 for o in out), (rank, out)


# ---------------------------------------------------------------------------------------
# Resident rounds of one worker per process (xgmi_plane.cc launch_resident,
# xgmi_threshold.hip threshold_resident_kernel): rounds of <= 4 MiB (up to 64 workgroups) are
# posted to a kernel that stays on the plane stream between rounds.

def _solo_resident_worker(rank, world, port, q, resident):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    if not resident:
        os.environ["MXAR_PLANE_RESIDENT"] = "0"
    import torch.distributed as dist

    from akka_allreduce_1_amd.engine import distributed_plane_job

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        for n, dtype, chunk in ((10, torch.float32, 2), (4096, torch.bfloat16, 512), (262144, torch.float32, 1024)):
            rounds = 41
            x = (torch.arange(n, dtype=torch.float32, device=DEV) + 1000.0 * rank).to(dtype)
            want = sum((torch.arange(n, dtype=torch.float32) + 1000.0 * k).to(dtype).float()
                       for k in range(world)).to(dtype)
            res = distributed_plane_job(n, x, max_chunk_size=chunk, dtype=dtype, rounds=rounds, grid=64,
                                        keep_last=True, timeout_s=60.0)
            y = res["last"]
            out[n] = (bool(res["ok"] and y is not None and y.iteration == rounds - 1 and torch.equal(y.data.cpu(), want)),
                      res["plane"]["resident_rounds"], rounds)
    except Exception as e:  # report, never hang the parent
        out["error"] = repr(e)
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("resident", [True, False])
def test_one_worker_per_process_resident_and_launched_rounds(resident):
    """One plane worker per process (2 processes on one GPU): exact rounds with resident rounds
    (default) and with one launch per round (MXAR_PLANE_RESIDENT=0); the resident runs took
    their rounds on the resident kernel."""
    import multiprocessing as mp

    from akka_allreduce_1_amd.parallel import free_port

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_solo_resident_worker, args=(r, world, port, q, resident)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    for rank, out in res:
        assert "error" not in out, (rank, out)
        for n, (ok, res_rounds, rounds) in out.items():
            assert ok, (rank, n, out)
            if resident:
                assert res_rounds >= 0.8 * rounds, (rank, n, out)
            else:
                assert res_rounds == 0, (rank, n, out)


# ---------------------------------------------------------------------------------------
# Co-located workers (xgmi_plane.cc PlaneGroup, xgmi_threshold.hip
# threshold_group_resident_kernel): the workers of a job in one process on one GPU run every
# round in ONE resident kernel, a slice of workgroups per worker.

def _bf16_close(data, n, it, P):
    """fp32 sum of the bf16 inputs, one rounding (as test_plane_rounds_exact_at_threshold_one)."""
    ar = torch.arange(n, dtype=torch.float64)
    ref = sum((ar + it + 1000.0 * j).to(torch.bfloat16).double() for j in range(P)).numpy()
    got = data.float().cpu().numpy()
    return bool(np.all(np.abs(got - ref) <= np.abs(ref) * 2.0 ** -8 + 1e-6))


@pytest.mark.parametrize("P,n,chunk,dtype", [(2, 10, 2, torch.float32), (3, 4096, 512, torch.bfloat16),
                                             (4, 16384, 1024, torch.float32), (2, 262144, 1024, torch.float32),
                                             (2, 1 << 20, 4096, torch.bfloat16)])
def test_group_rounds_exact(P, n, chunk, dtype):
    """Co-located workers: every round of every worker runs on the group kernel, outputs are
    the exact sums and every count is P."""
    rounds = 41
    job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=1, max_round=rounds - 1, dtype=dtype, timeout_s=20.0)
    try:
        job.run(timeout=120)
        assert job.rounds["n"] == rounds
        for k in range(P):
            st = job.system.plane_worker_state(job.workers[k])
            assert st["stats"]["plane_errors"] == 0 and st["stats"]["rounds_completed"] == rounds, st
        st = [p.stats for p in job.planes]
        assert all(s.group_size == P and s.group_rounds == rounds for s in st), [(s.group_size, s.group_rounds)
                                                                                 for s in st]
        assert sum(s.group_launches for s in st) >= 1
        for k in range(P):
            for it in range(rounds):
                data, counts = job.outputs[k][it]
                assert list(counts) == [P] * len(counts), (k, it)
                if dtype == torch.float32:
                    np.testing.assert_array_equal(data.cpu().numpy(), expected(n, it, range(P)))
                else:
                    assert _bf16_close(data, n, it, P), (k, it)
    finally:
        job.shutdown()


def test_group_kernel_leaves_when_idle_and_comes_back():
    """Sources slower than the group kernel's idle budget (1 ms): the kernel leaves between
    rounds and the next round launches it again - every round still exact."""
    P, n, chunk, rounds = 2, 1000, 100, 9

    def slow(k):
        def src(req):
            time.sleep(0.005)
            x = torch.arange(n, dtype=torch.float32, device=DEV) + (req.iteration + 1000.0 * k)
            torch.cuda.current_stream(DEV).synchronize()
            return x
        return src

    job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=1, max_round=rounds - 1, timeout_s=20.0,
                   sources=[slow(k) for k in range(P)])
    try:
        job.run(timeout=120)
        assert job.rounds["n"] == rounds
        for k in range(P):
            for it in range(rounds):
                np.testing.assert_array_equal(job.outputs[k][it][0].cpu().numpy(), expected(n, it, range(P)))
        st = [p.stats for p in job.planes]
        assert all(s.group_rounds == rounds for s in st), [s.group_rounds for s in st]
        assert sum(s.group_launches for s in st) >= 2, [s.group_launches for s in st]
    finally:
        job.shutdown()


def test_group_rounds_with_released_outputs():
    """Outputs handed to the sink as tensors and dropped every round go back to the pool
    behind the default stream (an event per batch): sums stay exact and the pool stops
    growing."""
    P, n, chunk, rounds = 2, 2048, 256, 60
    sums = [dict() for _ in range(P)]

    def on_output(k, out):
        sums[k][out.iteration] = float(out.data.double().sum().item())

    job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=1, max_round=rounds - 1, timeout_s=20.0,
                   keep_outputs=False, on_output=on_output)
    try:
        job.run(timeout=120)
        for k in range(P):
            for it in range(rounds):
                assert sums[k][it] == float(expected(n, it, range(P)).sum()), (k, it)
        st = [p.stats for p in job.planes]
        assert all(s.group_rounds == rounds for s in st), [s.group_rounds for s in st]
        assert all(s.pool_grown <= 8 for s in st), [s.pool_grown for s in st]
    finally:
        job.shutdown()


@pytest.mark.parametrize("n,dtype", [(4096, torch.float32), (1 << 20, torch.bfloat16)])
def test_eight_co_located_workers_beyond_the_hardware_queues(n, dtype):
    """More co-located workers than the process has hardware queues (GPU_MAX_HW_QUEUES = 4 on
    the boxes): an 8-worker PlaneJob in one process on one GPU runs exact rounds - one group
    kernel serves every worker, so no round waits in a queue behind a peer's spinning round
    (verdict r4 #6; the reference hosts any number of workers in one ActorSystem,
    AllreduceSpec.scala:746-755)."""
    P, rounds = 8, 30
    queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    assert P > queues
    chunk = 256 if n < 65536 else 4096
    job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=1, max_round=rounds - 1, dtype=dtype, timeout_s=20.0)
    try:
        job.run(timeout=120)
        assert job.rounds["n"] == rounds
        st = [p.stats for p in job.planes]
        assert all(s.group_size == P and s.group_rounds == rounds for s in st), [(s.group_size, s.group_rounds)
                                                                                 for s in st]
        for k in range(P):
            for it in (0, rounds // 2, rounds - 1):
                data, counts = job.outputs[k][it]
                assert list(counts) == [P] * len(counts), (k, it)
                if dtype == torch.float32:
                    np.testing.assert_array_equal(data.cpu().numpy(), expected(n, it, range(P)))
                else:
                    assert _bf16_close(data, n, it, P), (k, it)
    finally:
        job.shutdown()


def test_co_located_planes_construct_beyond_the_hardware_queues():
    """Building more planes than the process has hardware queues no longer refuses (the
    queue-probing heuristic is gone): 3 x GPU_MAX_HW_QUEUES planes on one GPU."""
    queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    planes = [C.hip.xgmi_plane(0, C.hip.DType.F32, 1024, max_peers=2, max_lag=1, grid=8, timeout_s=5.0)
              for _ in range(3 * queues)]
    assert len({p.descriptor for p in planes}) == 3 * queues
    planes.clear()


def test_two_jobs_share_the_device_budget_and_a_third_fails_loudly():
    """Two 4-worker PlaneJobs in ONE process, rounds interleaved, with a GEMM loop on a third
    stream: each job's group kernel reserved its workgroups in the device budget
    (csrc/hip/residency.h), the second took what the first left, every round of both is exact.
    A third job cannot fit and fails at construction with the budget named - never as round
    timeouts on the device."""
    import threading

    P, n, chunk, rounds = 4, 40000, 1000, 40
    jobs = []
    try:
        for j in range(2):
            srcs = [iota_source(n, DEV, torch.float32, 1000.0 * k + 10.0 * j) for k in range(P)]
            jobs.append(PlaneJob(P, n, max_chunk_size=chunk, max_round=rounds - 1, sources=srcs, timeout_s=20.0))
        st = C.hip.residency_state(0)
        assert st["used"] <= st["capacity"], st
        with pytest.raises(RuntimeError, match="residency budget"):
            PlaneJob(P, n, max_chunk_size=chunk, max_round=1, timeout_s=5.0)
        stop = threading.Event()

        def gemms():  # a third stream keeps the CUs busy with work that does not spin
            s = torch.cuda.Stream()
            a = torch.randn(2048, 2048, device=DEV)
            with torch.cuda.stream(s):
                while not stop.is_set():
                    a = torch.tanh(a @ a * 1e-3)
                    s.synchronize()

        th = threading.Thread(target=gemms)
        th.start()
        try:
            for job in jobs:
                job.start()
            for job in jobs:
                assert job.finished.wait(120), job.state()
        finally:
            stop.set()
            th.join()
        for j, job in enumerate(jobs):
            for p in job.planes:
                p.drain()
            for k in range(P):
                for it in (0, rounds // 2, rounds - 1):
                    data, counts = job.outputs[k][it]
                    exp = sum(np.arange(n, dtype=np.float64) + it + 1000.0 * q + 10.0 * j for q in range(P))
                    np.testing.assert_array_equal(data.float().cpu().numpy(), exp, err_msg=f"job {j} worker {k} round {it}")
                    assert all(c == P for c in counts)
    finally:
        for job in jobs:
            job.shutdown()
    assert C.hip.residency_state(0)["used"] == 0
