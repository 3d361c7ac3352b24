"""The launch-size grid rule (csrc/hip/xgmi_comm.h size_grid_rule, XgmiComm::launch_grid) on
the CPU: the workgroup counts the measured table in profiles/round4/README.md section 9 asks
for (grid sweep: 8 logical ranks x 1 MiB best at 128, x 4 MiB / 16 MiB at 256, 256 MiB at the
full grid; one-shot over P x bytes)."""
from akka_allreduce_1_amd._native import C

R = C.hip.size_grid_rule
KiB, MiB = 1 << 10, 1 << 20


def test_two_shot_one_workgroup_per_64_kib_between_64_and_256():
    assert R(8 * 256 * KiB, 512, 8, False) == 64      # 2 MiB in the launch: the floor
    assert R(8 * MiB, 512, 8, False) == 128           # 8 ranks x 1 MiB
    assert R(32 * MiB, 512, 8, False) == 256          # 8 x 4 MiB: the cap
    assert R(128 * MiB, 512, 8, False) == 256         # 8 x 16 MiB
    assert R(2 * MiB, 512, 2, False) == 64            # 2 x 1 MiB
    assert R(8 * MiB, 512, 2, False) == 128           # 2 x 4 MiB


def test_full_grid_from_the_limit():
    assert R(512 * MiB, 512, 2, False) == 512         # 2 x 256 MiB
    assert R(2048 * MiB, 512, 8, False) == 512        # 8 x 256 MiB
    assert R(256 * MiB, 512, 4, False, 256 * MiB) == 512   # threshold kernel: full from 256 MiB
    assert R(256 * MiB, 512, 4, False) == 256


def test_one_shot_counts_every_input_and_may_use_the_full_grid():
    assert R(2 * 256 * KiB, 512, 2, True) == 64       # 2 x (2 x 256 KiB) = 1 MiB
    assert R(2 * 4 * MiB, 512, 2, True) == 256        # 2 x 8 MiB = 16 MiB
    assert R(8 * MiB, 512, 8, True) == 512            # 8 x 8 MiB = 64 MiB: the full grid


def test_never_above_the_device_grid():
    assert R(64 * MiB, 128, 8, False) == 128
    assert R(64 * MiB, 32, 8, True) == 32
    assert R(1 * KiB, 32, 2, False) == 32


def test_shared_launches_cap_each_rank_at_half_the_cus():
    """Several logical ranks in one launch: at most 128 workgroups per rank at the default
    grid of 512 (profiles/round5/README.md section 13: 2 x 256 MiB two-shot 426-436 -> 389-395
    us; 4 ranks at 128 beat 64; 8 ranks indifferent)."""
    S = C.hip.shared_launch_rule
    assert S(1, 512) == 0                      # a rank alone on its GPU: launch_grid's rule
    assert S(2, 512) == 128
    assert S(8, 512) == 128                    # 512 / 8 = 64 is below the cap anyway
    assert min(R(512 * MiB, 512, 2, False) // 2, S(2, 512)) == 128


def test_co_located_plane_workers_share_the_cus():
    """engine.default_plane_grid: co-located workers together run about one workgroup per
    CU; a worker alone on its GPU keeps two per CU (section 12)."""
    from akka_allreduce_1_amd.engine import default_plane_grid

    cus = 256  # no GPU here: the MI355X count
    assert default_plane_grid(0, 1) == 2 * cus
    assert default_plane_grid(0, 2) == cus // 2
    assert default_plane_grid(0, 8) == cus // 8
    assert default_plane_grid(0, 16) == 16
    # the device residency budget (2 x CUs spinning workgroups, csrc/hip/residency.h) caps it:
    # 64 co-located workers x 8 + the dispatcher wave would not fit
    assert default_plane_grid(0, 64) == (2 * cus - 1) // 64
    from akka_allreduce_1_amd._native import C

    tok = C.hip.residency_reserve(0, 300, "another job")
    try:
        assert default_plane_grid(0, 4) == (2 * cus - 300 - 1) // 4  # what the first job left
        with __import__("pytest").raises(RuntimeError, match="residency budget"):
            C.hip.residency_reserve(0, 2 * cus, "too big")
    finally:
        tok.release()
    assert C.hip.residency_state(0)["used"] == 0
