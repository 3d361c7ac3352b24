"""Conformance vectors T1-T16: the reference's worker spec scenarios
(`src/test/scala/AllreduceSpec.scala`, catalogued in SURVEY §4.3) replayed against the
native WorkerCore through the deterministic TestKit. The probe impersonates every peer
and the master; the test injects the other peers' traffic by hand.
"""
import numpy as np

from akka_allreduce_1_amd.protocol import (CompleteAllreduce, InitWorkers, ReduceBlock, ScatterBlock,
                                           StartAllreduce)
from akka_allreduce_1_amd.testkit import (assertive_data_sink, create_basic_data_source,
                                          create_custom_data_source)

F = np.float32


def arr(*xs):
    return np.array(xs, dtype=F)


def init(tk, worker, workers, idx, thR, thC, lag, n, c):
    tk.tell(worker, InitWorkers(workers, tk.test_actor, idx, thR, thC, lag, n, c))


# --------------------------------------------------------------------------- T1
def test_t1_flushed_output_sums_all_correct_data(tk):
    """AllreduceSpec.scala:45-88 - uneven blocks (2, 1), real self-loopback, batch mode."""
    idx, n, c, actors = 1, 3, 2, 2
    gen = lambda i, it: float(i + it)
    source = create_custom_data_source(n, gen)
    out1 = [gen(i, 0) * actors for i in range(n)]
    out2 = [gen(i, 1) * actors for i in range(n)]
    seen = []
    sink = assertive_data_sink([out1, out2], [0, 1], seen)
    worker = tk.create_new_worker(source, sink)
    workers = tk.initialize_workers_as_self(actors)
    workers[idx] = worker
    init(tk, worker, workers, idx, 1.0, 1.0, 5, n, c)
    tk.tell(worker, StartAllreduce(0))
    tk.tell(worker, ScatterBlock(arr(2), 0, 1, 0, 0))
    tk.tell(worker, ReduceBlock(arr(0, 2), 0, 1, 0, 0, 2))
    tk.tell(worker, StartAllreduce(1))
    tk.tell(worker, ScatterBlock(arr(3), 0, 1, 0, 1))
    tk.tell(worker, ReduceBlock(arr(2, 4), 0, 1, 0, 1, 2))
    tk.fish_for_message(lambda m: m == CompleteAllreduce(1, 0))
    tk.expect_msg(CompleteAllreduce(1, 1))
    assert seen == [0, 1]


# --------------------------------------------------------------------------- T2/T3
def test_t2_t3_early_receiving_reduce(tk):
    """AllreduceSpec.scala:90-132 - reduce blocks of a future round trigger Start(3);
    completion after (0.8*4*1).toInt = 3 blocks; later scatters for it are ignored."""
    worker = tk.create_new_worker(create_basic_data_source(8))
    workers = tk.initialize_workers_as_self(4)
    future = 3
    init(tk, worker, workers, 0, 1.0, 0.8, 5, 8, 2)
    tk.tell(worker, StartAllreduce(0))
    tk.tell(worker, ReduceBlock(arr(12, 15), 0, 0, 0, future, 4))
    tk.tell(worker, ReduceBlock(arr(11, 10), 1, 0, 0, future, 4))
    tk.tell(worker, ReduceBlock(arr(10, 20), 2, 0, 0, future, 4))
    tk.tell(worker, ReduceBlock(arr(9, 10), 3, 0, 0, future, 4))

    def pred(m):
        if isinstance(m, CompleteAllreduce):
            assert m.round == future and m.srcId == 0
            return True
        assert isinstance(m, ScatterBlock), m
        return False

    tk.fish_for_message(pred)
    # T3: no longer act on completed scatter for that round
    for i in range(4):
        tk.tell(worker, ScatterBlock(arr(2 * i, 2 * i), i, 0, 0, future))
    tk.expect_no_msg()


# --------------------------------------------------------------------------- T4
def test_t4_single_round_allreduce(tk):
    """AllreduceSpec.scala:136-173."""
    worker = tk.create_new_worker(create_basic_data_source(8))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 1.0, 0.75, 5, 8, 2)
    tk.tell(worker, StartAllreduce(0))
    for i in range(4):
        tk.expect_scatter(ScatterBlock(arr(2 * i, 2 * i + 1), 0, i, 0, 0))
    for i in range(4):
        tk.tell(worker, ScatterBlock(arr(2 * i, 2 * i), i, 0, 0, 0))
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(12, 12), 0, d, 0, 0, 4))
    tk.tell(worker, ReduceBlock(arr(12, 15), 0, 0, 0, 0, 4))
    tk.tell(worker, ReduceBlock(arr(11, 10), 1, 0, 0, 0, 4))
    tk.tell(worker, ReduceBlock(arr(10, 20), 2, 0, 0, 0, 4))
    tk.tell(worker, ReduceBlock(arr(9, 10), 3, 0, 0, 0, 4))
    tk.expect_msg(CompleteAllreduce(0, 0))


# --------------------------------------------------------------------------- T5
def test_t5_nasty_chunk_size(tk):
    """AllreduceSpec.scala:176-220 - chunks [0,1],[2] / [3,4],[5]; minRequired = 1."""
    n = 6
    worker = tk.create_new_worker(create_basic_data_source(n))
    init(tk, worker, tk.initialize_workers_as_self(2), 0, 0.9, 0.8, 5, n, 2)
    tk.tell(worker, StartAllreduce(0))
    tk.expect_scatter(ScatterBlock(arr(0, 1), 0, 0, 0, 0))
    tk.expect_scatter(ScatterBlock(arr(2), 0, 0, 1, 0))
    tk.expect_scatter(ScatterBlock(arr(3, 4), 0, 1, 0, 0))
    tk.expect_scatter(ScatterBlock(arr(5), 0, 1, 1, 0))
    tk.tell(worker, ScatterBlock(arr(0, 1), 0, 0, 0, 0))
    tk.tell(worker, ScatterBlock(arr(2), 0, 0, 1, 0))
    tk.tell(worker, ScatterBlock(arr(0, 1), 1, 0, 0, 0))
    tk.tell(worker, ScatterBlock(arr(2), 1, 0, 1, 0))
    tk.expect_reduce(ReduceBlock(arr(0, 1), 0, 0, 0, 0, 1))
    tk.expect_reduce(ReduceBlock(arr(0, 1), 0, 1, 0, 0, 1))
    tk.expect_reduce(ReduceBlock(arr(2), 0, 0, 1, 0, 1))
    tk.expect_reduce(ReduceBlock(arr(2), 0, 1, 1, 0, 1))
    tk.tell(worker, ReduceBlock(arr(0, 2), 0, 0, 0, 0, 1))
    tk.tell(worker, ReduceBlock(arr(4), 0, 0, 1, 0, 1))
    tk.tell(worker, ReduceBlock(arr(6, 8), 1, 0, 0, 0, 1))
    tk.expect_msg(CompleteAllreduce(0, 0))
    tk.tell(worker, ReduceBlock(arr(10), 1, 0, 1, 0, 1))
    tk.expect_no_msg()


# --------------------------------------------------------------------------- T6
def test_t6_nasty_chunk_size_contd(tk):
    """AllreduceSpec.scala:222-285 - 3 chunks per block; reduce at 2 arrivals."""
    n = 9
    worker = tk.create_new_worker(create_basic_data_source(n))
    init(tk, worker, tk.initialize_workers_as_self(3), 0, 0.7, 0.7, 5, n, 1)
    tk.tell(worker, StartAllreduce(0))
    for d in range(3):
        for k in range(3):
            tk.expect_scatter(ScatterBlock(arr(3 * d + k), 0, d, k, 0))
    for s in range(3):
        for k in range(3):
            tk.tell(worker, ScatterBlock(arr(k), s, 0, k, 0))
    for k in range(3):
        for d in range(3):
            tk.expect_reduce(ReduceBlock(arr(2 * k), 0, d, k, 0, 2))
    vals = [0, 3, 6, 9, 12, 15, 18]
    for j, v in enumerate(vals):
        tk.tell(worker, ReduceBlock(arr(v), j // 3, 0, j % 3, 0, 2))
    tk.expect_msg(CompleteAllreduce(0, 0))
    tk.tell(worker, ReduceBlock(arr(21), 2, 0, 1, 0, 2))
    tk.tell(worker, ReduceBlock(arr(24), 2, 0, 2, 0, 2))
    tk.expect_no_msg()


# --------------------------------------------------------------------------- T7
def test_t7_multi_round_allreduce(tk):
    """AllreduceSpec.scala:287-320 - 10 rounds; reduce count (0.8*4)=3; complete at 2."""
    worker = tk.create_new_worker(create_basic_data_source(8))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 0.8, 0.5, 5, 8, 2)
    for i in range(10):
        tk.tell(worker, StartAllreduce(i))
        for d in range(4):
            tk.expect_scatter(ScatterBlock(arr(2 * d + i, 2 * d + 1 + i), 0, d, 0, i))
        for s in range(4):
            tk.tell(worker, ScatterBlock(arr(0 + i, 1 + i), s, 0, 0, i))
        for d in range(4):
            tk.expect_reduce(ReduceBlock(arr(0 + 3 * i, 3 + 3 * i), 0, d, 0, i, 3))
        tk.tell(worker, ReduceBlock(arr(1, 2), 0, 0, 0, i, 3))
        tk.tell(worker, ReduceBlock(arr(1, 2), 1, 0, 0, i, 3))
        tk.expect_msg(CompleteAllreduce(0, i))
        tk.tell(worker, ReduceBlock(arr(1, 2), 2, 0, 0, i, 3))
        tk.tell(worker, ReduceBlock(arr(1, 2), 3, 0, 0, i, 3))
        tk.expect_no_msg()


# --------------------------------------------------------------------------- T8
def test_t8_multi_round_allreduce_v2(tk):
    """AllreduceSpec.scala:322-356 - 2 chunks per block; reduce at first arrival."""
    worker = tk.create_new_worker(create_basic_data_source(8))
    init(tk, worker, tk.initialize_workers_as_self(2), 0, 0.6, 0.8, 5, 8, 2)
    for i in range(10):
        tk.tell(worker, StartAllreduce(i))
        tk.expect_scatter(ScatterBlock(arr(0 + i, 1 + i), 0, 0, 0, i))
        tk.expect_scatter(ScatterBlock(arr(2 + i, 3 + i), 0, 0, 1, i))
        tk.expect_scatter(ScatterBlock(arr(4 + i, 5 + i), 0, 1, 0, i))
        tk.expect_scatter(ScatterBlock(arr(6 + i, 7 + i), 0, 1, 1, i))
        tk.tell(worker, ScatterBlock(arr(0 + i, 1 + i), 0, 0, 0, i))
        tk.tell(worker, ScatterBlock(arr(2 + i, 3 + i), 0, 0, 1, i))
        tk.tell(worker, ScatterBlock(arr(10 + i, 11 + i), 1, 0, 0, i))
        tk.tell(worker, ScatterBlock(arr(12 + i, 13 + i), 1, 0, 1, i))
        tk.expect_reduce(ReduceBlock(arr(i, 1 + i), 0, 0, 0, i, 1))
        tk.expect_reduce(ReduceBlock(arr(i, 1 + i), 0, 1, 0, i, 1))
        tk.expect_reduce(ReduceBlock(arr(2 + i, 3 + i), 0, 0, 1, i, 1))
        tk.expect_reduce(ReduceBlock(arr(2 + i, 3 + i), 0, 1, 1, i, 1))
        tk.tell(worker, ReduceBlock(arr(1, 2), 0, 0, 0, i, 1))
        tk.tell(worker, ReduceBlock(arr(1, 2), 0, 0, 1, i, 1))
        tk.tell(worker, ReduceBlock(arr(1, 2), 1, 0, 0, i, 1))
        tk.expect_msg(CompleteAllreduce(0, i))
        tk.tell(worker, ReduceBlock(arr(1, 2), 1, 0, 1, i, 1))
        tk.expect_no_msg()


# --------------------------------------------------------------------------- T9
def test_t9_missed_scatter(tk):
    """AllreduceSpec.scala:358-392 - block size 1; reduce [6] after 3 of 4."""
    n = 4
    worker = tk.create_new_worker(create_basic_data_source(n))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 0.75, 0.75, 5, n, 2)
    tk.tell(worker, StartAllreduce(0))
    for d in range(4):
        tk.expect_scatter(ScatterBlock(arr(d), 0, d, 0, 0))
    tk.tell(worker, ScatterBlock(arr(0), 0, 0, 0, 0))
    tk.expect_no_msg()
    tk.tell(worker, ScatterBlock(arr(2), 1, 0, 0, 0))
    tk.expect_no_msg()
    tk.tell(worker, ScatterBlock(arr(4), 2, 0, 0, 0))
    tk.tell(worker, ScatterBlock(arr(6), 3, 0, 0, 0))
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(6), 0, d, 0, 0, 3))
    tk.tell(worker, ReduceBlock(arr(12), 0, 0, 0, 0, 3))
    tk.tell(worker, ReduceBlock(arr(11), 1, 0, 0, 0, 3))
    tk.tell(worker, ReduceBlock(arr(10), 2, 0, 0, 0, 3))
    tk.expect_msg(CompleteAllreduce(0, 0))
    tk.tell(worker, ReduceBlock(arr(9), 3, 0, 0, 0, 3))
    tk.expect_no_msg()


# --------------------------------------------------------------------------- T10
def test_t10_future_scatter(tk):
    """AllreduceSpec.scala:394-445 - round 1 reduces before round 0; a delayed round-0
    scatter then triggers the round-0 reduce; its duplicate is ignored."""
    n = 4
    worker = tk.create_new_worker(create_basic_data_source(n))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 0.75, 0.75, 5, n, 2)
    tk.tell(worker, StartAllreduce(0))
    for d in range(4):
        tk.expect_scatter(ScatterBlock(arr(d), 0, d, 0, 0))
    tk.tell(worker, ScatterBlock(arr(2), 1, 0, 0, 0))
    tk.tell(worker, ScatterBlock(arr(4), 2, 0, 0, 0))
    tk.tell(worker, ReduceBlock(arr(11), 1, 0, 0, 0, 3))
    tk.tell(worker, ReduceBlock(arr(10), 2, 0, 0, 0, 3))
    tk.tell(worker, StartAllreduce(1))
    tk.tell(worker, ScatterBlock(arr(2), 1, 0, 0, 1))
    tk.tell(worker, ScatterBlock(arr(4), 2, 0, 0, 1))
    tk.tell(worker, ScatterBlock(arr(6), 3, 0, 0, 1))
    for d in range(4):
        tk.expect_scatter(ScatterBlock(arr(d + 1), 0, d, 0, 1))
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(12), 0, d, 0, 1, 3))
    tk.tell(worker, ScatterBlock(arr(0), 3, 0, 0, 0))
    tk.tell(worker, ScatterBlock(arr(6), 3, 0, 0, 0))  # duplicate: count 4 != 3, no fire
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(6), 0, d, 0, 0, 3))
    tk.tell(worker, ReduceBlock(arr(9), 3, 0, 0, 0, 3))
    tk.expect_msg(CompleteAllreduce(0, 0))
    tk.tell(worker, ReduceBlock(arr(11), 1, 0, 0, 1, 3))
    tk.tell(worker, ReduceBlock(arr(10), 2, 0, 0, 1, 3))
    tk.tell(worker, ReduceBlock(arr(9), 3, 0, 0, 1, 3))
    tk.expect_msg(CompleteAllreduce(0, 1))


# --------------------------------------------------------------------------- T11
def test_t11_missed_reduce(tk):
    """AllreduceSpec.scala:447-479 - complete with 3 of 4 reduce blocks."""
    n = 4
    worker = tk.create_new_worker(create_basic_data_source(n))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 1.0, 0.75, 5, n, 100)
    tk.tell(worker, StartAllreduce(0))
    for d in range(4):
        tk.expect_scatter(ScatterBlock(arr(d), 0, d, 0, 0))
    for s in range(4):
        tk.tell(worker, ScatterBlock(arr(2 * s), s, 0, 0, 0))
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(12), 0, d, 0, 0, 4))
    tk.tell(worker, ReduceBlock(arr(12), 0, 0, 0, 0, 4))
    tk.expect_no_msg()
    tk.tell(worker, ReduceBlock(arr(11), 1, 0, 0, 0, 4))
    tk.expect_no_msg()
    tk.tell(worker, ReduceBlock(arr(10), 2, 0, 0, 0, 4))
    tk.expect_msg(CompleteAllreduce(0, 0))


# --------------------------------------------------------------------------- T12
def test_t12_delayed_future_reduce(tk):
    """AllreduceSpec.scala:481-529 - interleaved round 0/1 reduce blocks; relies on
    per-(sender, receiver) FIFO."""
    worker = tk.create_new_worker(create_basic_data_source(4))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 0.75, 0.75, 5, 4, 100)
    tk.tell(worker, StartAllreduce(0))
    for d in range(4):
        tk.expect_scatter(ScatterBlock(arr(d), 0, d, 0, 0))
    tk.tell(worker, ScatterBlock(arr(2), 1, 0, 0, 0))
    tk.tell(worker, ScatterBlock(arr(4), 2, 0, 0, 0))
    tk.tell(worker, ScatterBlock(arr(6), 3, 0, 0, 0))
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(12), 0, d, 0, 0, 3))
    tk.tell(worker, StartAllreduce(1))
    tk.tell(worker, ScatterBlock(arr(3), 1, 0, 0, 1))
    tk.tell(worker, ScatterBlock(arr(5), 2, 0, 0, 1))
    tk.tell(worker, ScatterBlock(arr(7), 3, 0, 0, 1))
    for d in range(4):
        tk.expect_scatter(ScatterBlock(arr(d + 1), 0, d, 0, 1))
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(15), 0, d, 0, 1, 3))
    for s, v in ((1, 11), (2, 10), (3, 9)):
        tk.tell(worker, ReduceBlock(arr(v), s, 0, 0, 0, 3))
        tk.tell(worker, ReduceBlock(arr(v), s, 0, 0, 1, 3))
    tk.expect_msg(CompleteAllreduce(0, 0))
    tk.expect_msg(CompleteAllreduce(0, 1))


# --------------------------------------------------------------------------- T13/T14
def _expect_basic_scatter(tk, i):
    """AllreduceSpec.scala:688-693."""
    for d in range(4):
        tk.expect_scatter(ScatterBlock(arr(2 * d + i, 2 * d + 1 + i), 0, d, 0, i))


def _simulate_scatter_from_peers(tk, worker, i):
    """AllreduceSpec.scala:682-686."""
    tk.tell(worker, ScatterBlock(arr(1.0 * (i + 1), 1.0 * (i + 1)), 1, 0, 0, i))
    tk.tell(worker, ScatterBlock(arr(2.0 * (i + 1), 2.0 * (i + 1)), 2, 0, 0, i))
    tk.tell(worker, ScatterBlock(arr(4.0 * (i + 1), 4.0 * (i + 1)), 3, 0, 0, i))


def _test_catchup(tk, worker, max_lag, catchup_round):
    """AllreduceSpec.scala:695-712."""
    tk.tell(worker, StartAllreduce(catchup_round))
    cr = catchup_round - (max_lag + 1)
    for d in range(4):
        tk.expect_reduce(ReduceBlock(arr(7.0 * (cr + 1), 7.0 * (cr + 1)), 0, d, 0, cr, 3))
    tk.expect_msg(CompleteAllreduce(0, cr))
    _expect_basic_scatter(tk, catchup_round)


def test_t13_simple_catchup(tk):
    """AllreduceSpec.scala:535-559 - Start(6/7/8) force-completes rounds 0/1/2."""
    worker = tk.create_new_worker(create_basic_data_source(8))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 1.0, 1.0, 5, 8, 2)
    for i in range(6):
        tk.tell(worker, StartAllreduce(i))
        _expect_basic_scatter(tk, i)
        _simulate_scatter_from_peers(tk, worker, i)
        for s in (1, 2, 3):
            tk.tell(worker, ReduceBlock(arr(12.0, 12.0), s, 0, 0, i, 4))
    _test_catchup(tk, worker, 5, 6)
    _test_catchup(tk, worker, 5, 7)
    _test_catchup(tk, worker, 5, 8)


def test_t14_cold_catchup(tk):
    """AllreduceSpec.scala:561-584 - Start(10) at once: rounds 0-4 force-completed with
    zero reduce blocks and count 0, then rounds 0-10 scattered."""
    worker = tk.create_new_worker(create_basic_data_source(8))
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 1.0, 1.0, 5, 8, 2)
    tk.tell(worker, StartAllreduce(10))
    for i in range(5):
        for d in range(4):
            tk.expect_reduce(ReduceBlock(arr(0, 0), 0, d, 0, i, 0))
        tk.expect_msg(CompleteAllreduce(0, i))
    for i in range(11):
        _expect_basic_scatter(tk, i)


# --------------------------------------------------------------------------- T15
def test_t15_multi_round_allreduce_v3(tk):
    """AllreduceSpec.scala:610-679 - minChunks (0.75*3*2)=4; round 1 completes first."""
    n = 9
    worker = tk.create_new_worker(create_basic_data_source(n))
    init(tk, worker, tk.initialize_workers_as_self(3), 0, 0.75, 0.75, 5, n, 2)
    tk.tell(worker, StartAllreduce(0))
    for d in range(3):
        tk.expect_scatter(ScatterBlock(arr(3 * d, 3 * d + 1), 0, d, 0, 0))
        tk.expect_scatter(ScatterBlock(arr(3 * d + 2), 0, d, 1, 0))
    for s in range(3):
        tk.tell(worker, ScatterBlock(arr(0, 1), s, 0, 0, 0))
    for s in range(3):
        tk.tell(worker, ScatterBlock(arr(2), s, 0, 1, 0))
    for d in range(3):
        tk.expect_reduce(ReduceBlock(arr(0, 2), 0, d, 0, 0, 2))
    for d in range(3):
        tk.expect_reduce(ReduceBlock(arr(4), 0, d, 1, 0, 2))
    tk.tell(worker, StartAllreduce(1))
    tk.tell(worker, ScatterBlock(arr(10, 11), 1, 0, 0, 1))
    tk.tell(worker, ScatterBlock(arr(12), 1, 0, 1, 1))
    tk.tell(worker, ScatterBlock(arr(10, 11), 2, 0, 0, 1))
    tk.tell(worker, ScatterBlock(arr(12), 2, 0, 1, 1))
    for d in range(3):
        tk.expect_scatter(ScatterBlock(arr(3 * d + 1, 3 * d + 2), 0, d, 0, 1))
        tk.expect_scatter(ScatterBlock(arr(3 * d + 3), 0, d, 1, 1))
    for d in range(3):
        tk.expect_reduce(ReduceBlock(arr(20, 22), 0, d, 0, 1, 2))
    for d in range(3):
        tk.expect_reduce(ReduceBlock(arr(24), 0, d, 1, 1, 2))
    tk.tell(worker, ReduceBlock(arr(11, 11), 1, 0, 0, 0, 2))
    tk.tell(worker, ReduceBlock(arr(11), 1, 0, 1, 1, 2))
    tk.tell(worker, ReduceBlock(arr(11, 11), 1, 0, 0, 1, 2))
    tk.tell(worker, ReduceBlock(arr(11), 1, 0, 1, 0, 2))
    tk.tell(worker, ReduceBlock(arr(11, 11), 2, 0, 0, 0, 2))
    tk.tell(worker, ReduceBlock(arr(11), 2, 0, 1, 1, 2))
    tk.expect_no_msg()
    tk.tell(worker, ReduceBlock(arr(11, 11), 2, 0, 0, 1, 2))
    tk.expect_msg(CompleteAllreduce(0, 1))
    tk.tell(worker, ReduceBlock(arr(11), 2, 0, 1, 0, 2))
    tk.expect_msg(CompleteAllreduce(0, 0))
    st = tk.system.worker_state(worker)
    assert st["round"] == 2  # round advances 0 -> 2 once both are complete


# --------------------------------------------------------------------------- T16
def test_t16_buffer_when_uninitialized(tk):
    """AllreduceSpec.scala:586-603 (commented out in the reference, the intended
    behaviour): a Start before Init is stashed and replayed after Init."""
    worker = tk.create_new_worker(create_basic_data_source(8))
    tk.tell(worker, StartAllreduce(0))
    tk.expect_no_msg()
    init(tk, worker, tk.initialize_workers_as_self(4), 0, 1.0, 1.0, 5, 8, 2)
    _expect_basic_scatter(tk, 0)


def test_conformance_threaded_mode():
    """T4 under the threaded dispatcher (eager scheduling), with real timeouts."""
    from akka_allreduce_1_amd.testkit import TestKit

    with TestKit("Threaded", deterministic=False, timeout=5.0) as tk:
        test_t4_single_round_allreduce(tk)
        test_t9_missed_scatter(tk)
