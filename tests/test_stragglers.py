"""Straggler tolerance end to end (the reference's reason to exist: thReduce / thComplete /
thAllreduce / maxLag, AllreduceWorker.scala:15-17, AllreduceMaster.scala:17-20), driven by
the fault-injection decorator on a threaded in-process cluster."""
import threading

import numpy as np
import pytest

from akka_allreduce_1_amd._native import C
from akka_allreduce_1_amd.protocol import AllReduceInput, MemberUp


DONE_AT = [0.0]  # perf_counter() at which the last run_cluster's master finished


def run_cluster(P, N, chunk, thA, thR, thC, lag, rounds, data=None, wrap=None, stop_after=None, timeout=30):
    """Master + P workers; returns ({k: {iteration: (data, counts)}}, master_state, worker_states)."""
    import time

    system = C.ActorSystem("ClusterSystem", False)
    done = threading.Event()

    def finished(r):
        DONE_AT[0] = time.perf_counter()
        done.set()

    master = system.master(P, thA, thR, thC, lag, N, rounds - 1, chunk, on_finished=finished)
    outs = {k: {} for k in range(P)}
    lock = threading.Lock()
    data = data or (lambda k, it: (np.arange(N, dtype=np.float32) + it) * (k + 1))
    workers = []

    def make(k):
        def src(req):
            return AllReduceInput(data(k, req.iteration))

        def sink(o):
            with lock:
                outs[k][o.iteration] = (np.asarray(o.data).copy(), list(o.count))
            if stop_after and k == stop_after[0] and o.iteration == stop_after[1]:
                threading.Thread(target=lambda: system.stop(workers[k])).start()

        return src, sink

    for k in range(P):
        src, sink = make(k)
        workers.append(system.worker(src, sink, f"worker{k}"))
    refs = [wrap(k, w, system) if wrap else w for k, w in enumerate(workers)]
    for r in refs:
        master.tell(MemberUp(r, "worker", ""), None)
    ok = done.wait(timeout)
    system.await_idle(5.0)
    mstate = system.master_state(master)
    wstates = [system.worker_state(w) for w in workers]
    system.shutdown()
    assert ok, f"cluster did not finish: {mstate}"
    return outs, mstate, wstates


def counts_per_element(N, P, chunk, counts):
    lay = C.BlockLayout(N, P, chunk)
    maxc = max(lay.num_chunks(b) for b in range(P))
    per = np.zeros(N, dtype=np.int64)
    for b in range(P):
        for i in range(lay.start[b], lay.end[b]):
            per[i] = counts[b * maxc + (i - lay.start[b]) // chunk]
    return per


@pytest.mark.parametrize("P,N,chunk", [(4, 10, 2), (4, 6, 2), (3, 4, 2), (3, 7, 2)])
def test_reference_crash_configs_now_exact(P, N, chunk):
    """these (P, N, C) crash the reference (ArrayIndexOutOfBounds); here they run."""
    outs, _, _ = run_cluster(P, N, chunk, 1.0, 1.0, 1.0, 1, 4)
    for k in range(P):
        for it in range(4):
            exp = (np.arange(N) + it) * sum(range(1, P + 1))
            np.testing.assert_array_equal(outs[k][it][0], exp)


def test_lossy_scatter_partial_sums_are_consistent():
    """25 % of the scatter traffic to worker 1 is lost; thresholds 0.75 let every round finish.
    With all-ones inputs each output element equals the number of contributions summed into
    its chunk, which must equal the count the worker reports for that chunk."""
    P, N, chunk, rounds = 4, 64, 4, 12

    def wrap(k, ref, system):
        return C.faulty(system, ref, drop=0.25, kinds=["ScatterBlock"], seed=7) if k == 1 else ref

    outs, mstate, ws = run_cluster(P, N, chunk, 0.75, 0.75, 0.75, 1, rounds, data=lambda k, it: np.ones(N, np.float32),
                                   wrap=wrap)
    assert mstate["finished"]
    partial = 0
    for k in range(P):
        for it, (vals, counts) in outs[k].items():
            per = counts_per_element(N, P, chunk, counts)
            nz = per > 0
            np.testing.assert_array_equal(vals[nz], per[nz].astype(np.float32))
            assert np.all(vals[~nz] == 0)
            partial += int((per[nz] < P).sum())
    assert partial > 0, "expected some partial (threshold-fired) sums"


def test_master_advances_without_a_silent_worker():
    """thAllreduce = thReduce = thComplete = 0.75: from round 3 on worker 3 receives nothing
    (a hung or partitioned node); the other three keep completing rounds with partial sums
    and the master's barrier advances on 3 of 4 completions."""
    P, N, chunk, rounds = 4, 16, 4, 10

    def wrap(k, ref, system):
        return C.faulty(system, ref, drop=1.0, round_lo=3, seed=5) if k == 3 else ref

    outs, mstate, ws = run_cluster(P, N, chunk, 0.75, 0.75, 0.75, 1, rounds, wrap=wrap)
    assert mstate["finished"]
    assert max(outs[3]) <= 3
    for k in range(3):
        assert rounds - 1 in outs[k]
        vals, counts = outs[k][rounds - 1]
        assert max(counts) <= 3  # worker 3's contribution is missing from every late sum


def test_delays_reorder_but_exact_sums_hold():
    """Half of all scatters/reduces delayed by 5 ms (reordered across rounds): with exact
    thresholds and maxLag 3 the future-round path absorbs the reordering and every sum is
    exact."""
    P, N, chunk, rounds = 3, 12, 2, 8

    def wrap(k, ref, system):
        return C.faulty(system, ref, delay_ms=5, delay_prob=0.5, kinds=["ScatterBlock", "ReduceBlock"], seed=k + 1)

    outs, mstate, ws = run_cluster(P, N, chunk, 1.0, 1.0, 1.0, 3, rounds, wrap=wrap)
    for k in range(P):
        for it in range(rounds):
            np.testing.assert_array_equal(outs[k][it][0], (np.arange(N) + it) * 6)


def test_duplicates_are_detected():
    """The reference double-counts a duplicated message (kept); the worker reports
    it in its stats."""
    P, N, chunk, rounds = 2, 8, 2, 4

    def wrap(k, ref, system):
        return C.faulty(system, ref, duplicate=1.0, kinds=["ReduceBlock"], seed=3) if k == 0 else ref

    _, _, ws = run_cluster(P, N, chunk, 1.0, 1.0, 0.5, 1, rounds, wrap=wrap)
    assert ws[0]["stats"]["duplicate_arrivals"] > 0


def test_resume_from_checkpointed_round():
    """Checkpoint/resume of the control state: the master reports every
    completed round; a new job started at round R re-initialises workers there (InitWorkers
    startRound) and they fetch round R first - no replay of rounds 0..R-1."""
    P, N, chunk = 2, 8, 2
    system = C.ActorSystem("ClusterSystem", False)
    done = threading.Event()
    seen_rounds, fetched = [], []
    master = system.master(P, 1.0, 1.0, 1.0, 1, N, 9, chunk, on_finished=lambda r: done.set(), startRound=6,
                           on_round=lambda r, e: seen_rounds.append(r))
    outs = {}

    def src(req):
        fetched.append(req.iteration)
        return AllReduceInput(np.arange(N, dtype=np.float32) + req.iteration)

    def sink(o):
        outs.setdefault(o.iteration, np.asarray(o.data).copy())

    ws = [system.worker(src, sink, f"w{k}") for k in range(P)]
    for w in ws:
        master.tell(MemberUp(w, "worker", ""), None)
    assert done.wait(20)
    system.await_idle(5.0)
    system.shutdown()
    assert seen_rounds == [6, 7, 8, 9]
    assert min(fetched) == 6
    for r in range(6, 10):
        np.testing.assert_array_equal(outs[r], 2 * (np.arange(N) + r))


def test_master_round_deadline_advances_past_a_hung_worker():
    """thAllreduce = 1 would stall forever on a worker that never completes; a
    round deadline at the master advances such rounds, and the healthy workers still finish
    every round (the hung worker's share is missing from their partial sums)."""
    P, N, chunk, rounds = 3, 12, 2, 6
    system = C.ActorSystem("ClusterSystem", False)
    done = threading.Event()
    master = system.master(P, 1.0, 0.6, 0.6, 1, N, rounds - 1, chunk, on_finished=lambda r: done.set(),
                           roundTimeoutMs=100)
    outs = {k: {} for k in range(P)}
    ws = []
    for k in range(P):
        ws.append(system.worker(lambda req: AllReduceInput(np.ones(N, np.float32)),
                                (lambda o, k=k: outs[k].setdefault(o.iteration, 1)), f"w{k}"))
    hung = C.faulty(system, ws[2], drop=1.0, round_lo=2, seed=1)  # deaf from round 2 on
    for r in [ws[0], ws[1], hung]:
        master.tell(MemberUp(r, "worker", ""), None)
    assert done.wait(20)
    st = system.master_state(master)
    system.shutdown()
    assert st["round_timeouts"] >= 1
    assert all(len(outs[k]) == rounds for k in (0, 1))


def test_blocking_straggler_does_not_hold_the_master():
    """A worker whose dataSource blocks (10 ms per round) must not slow the rounds the fast
    worker drives at thAllreduce 0.5. Its CompleteAllreduce schedules the master on the
    straggler's dispatcher thread (the run-next slot); while the straggler's turn goes on with
    more blocking messages the master must run elsewhere (csrc/runtime/actor_system.cc), not
    wait for the turn to end - that held every round of the job behind up to 64 blocking
    messages (profiles/round6/README.md section 6)."""
    import time


    def timed(delay):
        def data(k, it):
            if k == 1 and delay:
                time.sleep(delay)
            return np.arange(10, dtype=np.float32) + it

        t0 = time.perf_counter()
        outs, mstate, _ = run_cluster(2, 10, 2, 0.5, 0.5, 0.5, 1, 3000, data=data, timeout=60)
        assert mstate["round"] >= 2999, mstate
        return DONE_AT[0] - t0, outs  # to the master's last round (the backlog drains after)

    base, _ = timed(0.0)
    wall, outs = timed(0.01)
    assert len(outs[0]) >= 2900  # the fast worker completed (nearly) every round itself
    assert 0 < len(outs[1]) < 2900  # the straggler completed some rounds during the job (its
    # CompleteAllreduce is what scheduled the master on its thread)
    assert wall < 3 * base + 0.25, (wall, base)
