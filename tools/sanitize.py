#!/usr/bin/env python3
"""Build and run the host-runtime stress program under a sanitizer.

The protocol cores, actor runtime and cluster layer (csrc/core, csrc/runtime, csrc/cluster;
no HIP, no Python) are compiled with -fsanitize=<thread|address|undefined> together with
csrc/tests/runtime_stress.cc and run; any sanitizer report fails the run.

    python tools/sanitize.py --sanitize thread
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "csrc"


def build(kind: str) -> Path:
    out = ROOT / "build" / f"runtime_stress_{kind}"
    out.parent.mkdir(parents=True, exist_ok=True)
    srcs = [CSRC / "tests" / "runtime_stress.cc"]
    for sub in ("core", "runtime", "cluster"):
        srcs += sorted((CSRC / sub).glob("*.cc"))
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={kind}", "-fno-omit-frame-pointer", f"-I{CSRC}",
           "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-DMXAR_NO_ROCTX", "-o", str(out)]
    cmd += [str(s) for s in srcs] + ["-lpthread"]
    subprocess.run(cmd, check=True)
    return out


def run(binary: Path, kind: str) -> int:
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 exitcode=66 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([str(binary)], env=env, capture_output=True, text=True, timeout=600)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[-20000:])
    return r.returncode


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sanitize", choices=["thread", "address", "undefined"], default="thread")
    a = ap.parse_args()
    return run(build(a.sanitize), a.sanitize)


if __name__ == "__main__":
    sys.exit(main())
