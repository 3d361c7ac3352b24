"""Algorithm classes shared by the communicator's tuner (parallel/comm.py) and the bench
line (benchmarks/summary.py) - one definition, no dependencies (importable without the
native module)."""

# library paths: timed next to the kernels as comparison columns, never picked by tune() and
# never the automatic headline
LIBRARY_ALGOS = ("rccl", "rsag", "p2p")
# kernels that round more than once (ring_native: every reduce-scatter hop's partial is rounded
# to the element type): timed by tune() as comparison columns but adopted only with
# exact_only=False - by default every tuned choice sums in fp32 and rounds once, as precise as
# the reference's fp32 sums
LOSSY_ALGOS = ("ring_native",)
