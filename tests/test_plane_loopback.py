"""The round engine's control logic on a CPU: PlaneWorkerActor (csrc/runtime/plane_worker.h)
over LoopbackRoundPlane (csrc/runtime/loopback_plane.h), the host twin of the xGMI round
plane. The same scenarios as tests/test_plane_gpu.py, no GPU:

* th = 1: every round exact, every chunk counts P (AllreduceWorker.scala:240-251);
* T13 analogue (AllreduceSpec.scala:535-559): a stalled worker, the master's round deadline,
  StartAllreduce(r) with r - maxLag > round forces the stuck rounds (catch-up, :91-97);
* T14 analogue (AllreduceSpec.scala:561-584): a worker whose first StartAllreduce is round
  4 completes rounds 0..2 cold (nothing of its own);
* re-initialisation (new membership epoch, startRound, roundBase) on the same planes;
* a stash before InitWorkers and descriptor checks.
"""
import threading
import time

import numpy as np
import pytest

from akka_allreduce_1_amd._native import C
from akka_allreduce_1_amd.engine import PlaneJob, host_iota_source

F = np.float32


def layout(n, P, C_):
    step = -(-n // P)
    return step, -(-step // C_)


def expected(n, it, ranks):
    i = np.arange(n, dtype=np.float64)
    return sum(i + it + 1000.0 * k for k in ranks)


def subset_ok(vals, lo, hi, it, cnt):
    i = np.arange(lo, hi, dtype=np.float64)
    s = (vals[lo:hi].astype(np.float64) - cnt * (i + it)) / 1000.0
    return np.allclose(s, s[0], atol=1e-3) and abs(s[0] - round(s[0])) <= 1e-3


def consistent(outputs, P, n, chunk, counts_ok):
    """Every chunk of every output is the sum of `count` distinct workers (0 -> zeros)."""
    step, nch = layout(n, P, chunk)
    for k in range(P):
        for it, (data, counts) in outputs[k].items():
            v = np.asarray(data, dtype=np.float64)
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
                        assert subset_ok(v, lo, hi, it, cnt), (k, it, j, c, cnt)


@pytest.mark.parametrize("P,n,chunk", [(2, 10, 2), (3, 10007, 333), (4, 4096, 100)])
def test_loopback_rounds_exact_at_threshold_one(P, n, chunk):
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=1.0, th_complete=1.0, max_lag=1, max_round=12,
                   plane="loopback")
    try:
        job.run(timeout=60)
        assert job.rounds["n"] == 13
        for k in range(P):
            st = job.system.plane_worker_state(job.workers[k])
            assert st["stats"]["plane_errors"] == 0 and st["stats"]["rounds_completed"] == 13, st
            for it in range(13):
                data, counts = job.outputs[k][it]
                np.testing.assert_array_equal(np.asarray(data), expected(n, it, range(P)).astype(F))
                assert len(counts) == P * job.planes[k].chunks and all(c == P for c in counts), counts
        assert job.planes[0].stats["launches"] == 13 and job.planes[0].stats["forced_rounds"] == 0
    finally:
        job.shutdown()


def test_loopback_reference_defaults_101_rounds():
    """The reference's default deployment shape (AllreduceMaster.scala:105-114): 2 workers,
    dataSize 10, maxChunkSize 2, 101 rounds, thReduce 0.9 (f32(0.9 * 2) = 1 contribution per
    reduce) / thComplete 0.8 (f32(0.8 * 2 * 3) = 4 of 6 chunks), maxLag 1: every round
    completes and every chunk is a consistent partial sum."""
    P, n, chunk = 2, 10, 2
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=0.9, th_complete=0.8, max_lag=1, max_round=100,
                   plane="loopback")
    try:
        job.run(timeout=60)
        assert job.rounds["n"] == 101
        consistent(job.outputs, P, n, chunk, {0, 1, 2})
    finally:
        job.shutdown()


def test_loopback_simple_catchup():
    """T13 analogue: worker 2 stalls 1 s in round 0; the master's round deadline keeps
    starting rounds, the fast workers' stuck rounds are forced (catch-up) and nothing errs."""
    P, n, chunk = 3, 600, 50
    srcs = [host_iota_source(n, 1000.0 * k) for k in range(P)]
    base = srcs[2]

    def stall(req):
        if req.iteration == 0:
            time.sleep(1.0)
        return base(req)

    srcs[2] = stall
    job = PlaneJob(P, n, max_chunk_size=chunk, th_reduce=2.0 / 3.0, th_complete=1.0, max_lag=1, max_round=8,
                   sources=srcs, round_timeout_ms=150, plane="loopback")
    try:
        job.run(timeout=60)
        st = job.state()
        for k, w in enumerate(st["workers"]):
            assert w["stats"]["plane_errors"] == 0, (k, w)
            assert w["round"] == 9, (k, w)
        assert sum(w["stats"]["forced_completions"] for w in st["workers"][:2]) > 0, st
        consistent(job.outputs, P, n, chunk, {0, 1, 2, 3})  # 1: a forced reduce of what had arrived
        step, nch = layout(n, P, chunk)
        data, counts = job.outputs[0][0]  # forced: the fast blocks made it (count 2), the straggler's not
        assert counts[:2 * nch] == [2] * (2 * nch) and counts[2 * nch:] == [0] * nch, counts
    finally:
        job.shutdown()


def test_loopback_cold_catchup():
    """T14 analogue: worker 2's first StartAllreduce is round 4 (maxLag 1): rounds 0..2 are
    cold on worker 2 (count 0 for its own block), 3..4 run normally."""
    P, n, chunk = 3, 600, 50
    th = 2.0 / 3.0
    system = C.ActorSystem("Cold", False)
    probe = system.probe("master")
    planes = [C.loopback_plane("cold-hub") for _ in range(P)]
    outs = [dict() for _ in range(P)]

    def sink(k):
        return lambda out: outs[k].__setitem__(out.iteration, (np.asarray(out.data).copy(), list(out.count)))

    ws = [system.plane_worker(host_iota_source(n, 1000.0 * k), sink(k), planes[k], f"w{k}") for k in range(P)]
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
                e = probe.receive(0.5)
                if e is not None and isinstance(e[0], C.CompleteAllreduce):
                    got.add((e[0].srcId, e[0].round))
            return want <= got

        for r in (0, 1):
            for k in (0, 1):
                ws[k].tell(C.StartAllreduce(r, 1), None)
            assert collect({(0, r), (1, r)}, 10), sorted(got)
        for r in (2, 3, 4):
            for k in (0, 1):
                ws[k].tell(C.StartAllreduce(r, 1), None)
        time.sleep(0.2)
        ws[2].tell(C.StartAllreduce(4, 1), None)  # worker 2's first StartAllreduce
        assert collect({(k, r) for k in range(P) for r in range(5)}, 20), sorted(got)
        st = system.plane_worker_state(ws[2])
        assert st["stats"]["cold_rounds"] == 3 and st["stats"]["plane_errors"] == 0, st
        step, nch = layout(n, P, chunk)
        for it in (0, 1):  # cold on worker 2: the fast blocks (count 2), nothing of its own
            data, counts = outs[2][it]
            assert counts[:2 * nch] == [2] * (2 * nch), (it, counts)
            assert counts[2 * nch:] == [0] * nch, (it, counts)
            np.testing.assert_array_equal(data[:2 * step], expected(n, it, (0, 1))[:2 * step].astype(F))
            assert not np.any(data[2 * step:])
        consistent(outs, P, n, chunk, {0, 1, 2, 3})  # 1: a forced reduce of what had arrived
    finally:
        system.shutdown()


def test_loopback_stash_before_init_and_reinit():
    """StartAllreduce before InitWorkers is stashed and replayed; a second
    membership epoch (startRound 7, roundBase 100) on the same planes runs exact rounds and
    drops the old epoch's messages."""
    P, n, chunk = 2, 500, 60
    system = C.ActorSystem("Reinit", False)
    probe = system.probe("master")
    planes = [C.loopback_plane("reinit-hub") for _ in range(P)]
    outs = [dict() for _ in range(P)]
    ws = [system.plane_worker(host_iota_source(n, 1000.0 * k),
                              (lambda k: lambda out: outs[k].__setitem__((out.iteration), np.asarray(out.data).copy()))(k),
                              planes[k], f"w{k}") for k in range(P)]
    try:
        wmap = {k: ws[k] for k in range(P)}
        descs = {k: planes[k].descriptor for k in range(P)}
        got = set()

        def collect(want, limit=10):
            t0 = time.time()
            while not want <= got and time.time() - t0 < limit:
                e = probe.receive(0.5)
                if e is not None and isinstance(e[0], C.CompleteAllreduce):
                    got.add((e[0].epoch, e[0].srcId, e[0].round))
            return want <= got

        for k in range(P):  # Start first: stashed until Init
            ws[k].tell(C.StartAllreduce(0, 1), None)
        for k in range(P):
            m = C.InitWorkers(wmap, probe, k, 1.0, 1.0, 1, n, chunk, epoch=1)
            m.planes = descs
            ws[k].tell(m, None)
        assert collect({(1, k, 0) for k in range(P)}), sorted(got)
        assert system.plane_worker_state(ws[0])["stats"]["stashed"] >= 1
        for k in range(P):
            m = C.InitWorkers(wmap, probe, k, 1.0, 1.0, 1, n, chunk, epoch=2, startRound=7)
            m.planes = descs
            m.roundBase = 100
            ws[k].tell(m, None)
        for k in range(P):
            ws[k].tell(C.StartAllreduce(3, 1), None)  # an old epoch's Start: dropped
        for r in (7, 8, 9):
            for k in range(P):
                ws[k].tell(C.StartAllreduce(r, 2), None)
            assert collect({(2, k, r) for k in range(P)}), sorted(got)
        for it in (0, 7, 8, 9):
            for k in range(P):
                np.testing.assert_array_equal(outs[k][it], expected(n, it, range(P)).astype(F))
        assert 3 not in outs[0]
        assert system.plane_worker_state(ws[0])["stats"]["stale_dropped"] >= 1
    finally:
        system.shutdown()


def test_loopback_descriptors_must_share_a_hub():
    system = C.ActorSystem("Desc", False)
    probe = system.probe("master")
    a, b = C.loopback_plane("hub-a"), C.loopback_plane("hub-b")
    w = system.plane_worker(host_iota_source(8), None, a, "w0")
    errors = []
    try:
        m = C.InitWorkers({0: w, 1: probe}, probe, 0, 1.0, 1.0, 1, 8, 2, epoch=1)
        m.planes = {0: a.descriptor, 1: b.descriptor}
        w.tell(m, None)
        time.sleep(0.3)
        st = system.plane_worker_state(w)
        errors.append(st["initialized"])
    finally:
        system.shutdown()
    assert errors == [False]  # the InitWorkers was refused: the worker stays uninitialised
    assert a.descriptor.startswith("loop1 hub=hub-a ")


def test_loopback_planes_are_independent_across_hubs():
    """Two jobs in one process, each on its own hub, run side by side."""
    jobs = [PlaneJob(2, 64, max_chunk_size=8, max_round=20, plane="loopback") for _ in range(2)]
    ts = [threading.Thread(target=j.run, kwargs={"timeout": 60}) for j in jobs]
    try:
        for t in ts:
            t.start()
        for t in ts:
            t.join(90)
        for j in jobs:
            assert j.rounds["n"] == 21
            np.testing.assert_array_equal(np.asarray(j.outputs[1][20][0]), expected(64, 20, range(2)).astype(F))
    finally:
        for j in jobs:
            j.shutdown()


def test_make_plane_worker_with_a_loopback_hub():
    """actors.make_plane_worker builds the worker + plane; the master relays the descriptors
    announced in MemberUp.meta."""
    from akka_allreduce_1_amd.actors import make_master, make_plane_worker
    from akka_allreduce_1_amd.protocol import MemberUp

    n, P = 12, 3
    system = C.ActorSystem("Api", False)
    fin = threading.Event()
    outs = [dict() for _ in range(P)]
    try:
        pairs = [make_plane_worker(system, host_iota_source(n, 1000.0 * k),
                                   (lambda k: lambda o: outs[k].__setitem__(o.iteration, np.asarray(o.data).copy()))(k),
                                   data_size=n, name=f"w{k}", hub="api-hub") for k in range(P)]
        master = make_master(system, P, 1.0, 1.0, 1.0, 1, n, 5, 2, on_finished=lambda r: fin.set())
        for w, plane in pairs:
            master.tell(MemberUp(w, "worker", "", plane.descriptor), None)
        assert fin.wait(30)
        for p in (pl for _, pl in pairs):
            p.drain()
        for k in range(P):
            np.testing.assert_array_equal(outs[k][5], expected(n, 5, range(P)).astype(F))
        with pytest.raises(ValueError):
            make_plane_worker(system, host_iota_source(n), data_size=n)
    finally:
        system.shutdown()


def test_loopback_native_keep_last_sink_and_master_stamps():
    """keep_last: a native dataSink per worker keeps only the newest round output (no Python
    on the round path); the master stamps every round barrier natively."""
    P, n, chunk, rounds = 3, 1001, 50, 9
    job = PlaneJob(P, n, max_chunk_size=chunk, max_lag=1, max_round=rounds - 1, plane="loopback",
                   keep_outputs=False, keep_last=True)
    try:
        job.run(timeout=60)
        st = job.stamps
        assert len(st) == rounds and all(b >= a for a, b in zip(st, st[1:])), st
        assert abs(st[-1] - __import__("time").perf_counter()) < 60  # perf_counter timebase
        for k in range(P):
            o = job.last_output(k)
            assert o.iteration == rounds - 1 and all(c == P for c in o.count)
            np.testing.assert_array_equal(np.asarray(o.data), expected(n, rounds - 1, range(P)).astype(F))
        assert not any(job.outputs[k] for k in range(P))  # nothing kept by Python
    finally:
        job.shutdown()
    assert len(job.stamps) == rounds  # still readable after shutdown


def test_tensor_source_rejects_host_tensors_and_loopback_keeps_callables():
    """hip.tensor_source takes GPU tensors only (checked before any HIP call); on the
    loopback plane PlaneJob leaves sources as they are."""
    import torch

    with pytest.raises(TypeError):
        C.hip.tensor_source(torch.zeros(8))
    with pytest.raises(TypeError):
        C.hip.tensor_source([1.0, 2.0])
    src = host_iota_source(16, 0.0)
    job = PlaneJob(2, 16, max_chunk_size=4, max_round=1, plane="loopback", sources=[src, src], keep_last=True)
    try:
        assert job.sources[0] is src
        job.run(timeout=30)
        assert job.last_output(1).iteration == 1
    finally:
        job.shutdown()
