#!/usr/bin/env python3
"""VERDICT r2 item 5 at full size: the GPU round engine with the reference's 2-float
maxChunkSize on a 1 M-float vector (P = 3, th = 2/3, causal straggler) vs the host
WorkerCore - bit-identical outputs and counts (tests/test_plane_gpu.py, fine_chunk_parity).

    python tools/fine_chunk_parity.py --n 1048576 > gpurun_out/fine_chunk_parity.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3 * 349526)  # 1 M floats in 3 equal blocks
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import threading
    import time

    import test_plane_gpu as t  # noqa: E402

    t0 = time.time()

    def beat():  # progress for the long host run (gpurun kills a run silent for 3 min)
        while True:
            time.sleep(30)
            print(f"... {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()

    r = t.fine_chunk_parity(a.n, rounds=a.rounds, log=lambda m: print(m, file=sys.stderr, flush=True))
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
