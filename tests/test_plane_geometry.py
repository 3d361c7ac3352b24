"""The round geometry is a function of the membership alone (csrc/runtime/plane_geometry.h):
every worker of a job - co-located or alone on its GPU - computes the same kernel chunk, so
peers' slot offsets and per-chunk flags line up (advisor r5: mixed placement)."""
from akka_allreduce_1_amd._native import C

H = "00" * 64  # a well-formed (dummy) IPC handle


def desc(pid, dev, grid=128, wgc=1, coarsen=1):
    return f"xgmi1 pid={pid} dev={dev} bytes=1 id={pid * 10 + dev} grid={grid} wgc={wgc} coarsen={coarsen} h={H}"


def test_mixed_placement_agrees_on_the_chunk():
    # devices [0, 0, 1] in one process: two workers share GPU 0's group kernel, one is alone
    mixed = {0: desc(100, 0), 1: desc(100, 0), 2: desc(100, 1)}
    g = C.plane_geometry(3, 4 << 20, 1024, 1.0, 1.0, mixed)
    # the co-located cap (one kernel chunk per workgroup of 128) applies to the WHOLE job:
    # 1366 reference chunks per block -> 11 per kernel chunk, for the lone worker on GPU 1 too
    assert g["colocation"] == 2 and g["coarse"] == 11 and g["chunk"] == 11 * 1024 and g["nch"] == 125
    # the result cannot depend on which worker asks: the function sees only the membership
    # (a worker's own id is not an input); the same job laid out one worker per GPU chunks finer
    alone = {0: desc(100, 0), 1: desc(101, 1), 2: desc(102, 2)}
    g1 = C.plane_geometry(3, 4 << 20, 1024, 1.0, 1.0, alone)
    assert g1["colocation"] == 1 and g1["coarse"] == 8


def test_job_wide_knobs_take_the_strictest_plane():
    # planes built with different grids / knobs: the smallest grid, coarsening only if all allow
    d = {0: desc(1, 0, grid=256), 1: desc(2, 1, grid=64)}
    assert C.plane_geometry(2, 1 << 22, 1024, 1.0, 1.0, d)["grid"] == 64
    d = {0: desc(1, 0), 1: desc(2, 1, coarsen=0)}
    assert C.plane_geometry(2, 1 << 22, 1024, 1.0, 1.0, d)["coarse"] == 1
    # below full thresholds the reference chunk is the decision unit: never coarsened
    d = {0: desc(1, 0), 1: desc(1, 0)}
    g = C.plane_geometry(2, 1 << 22, 1024, 0.75, 0.75, d)
    assert g["coarse"] == 1 and g["nch"] == g["nch_ref"] == 2048


def test_descriptors_without_geometry_fields_still_parse():
    # a round-5 descriptor (no grid / wgc / coarsen): defaults, no error
    old = {0: f"xgmi1 pid=1 dev=0 bytes=1 id=1 h={H}", 1: f"xgmi1 pid=2 dev=1 bytes=1 id=2 h={H}"}
    g = C.plane_geometry(2, 1000, 2, 1.0, 1.0, old)
    assert g["block"] == 500 and g["nch"] == 1  # a block of <= 32 KiB is one kernel chunk
