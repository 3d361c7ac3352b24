"""Loader for the in-tree native module `_C` (C++ runtime + HIP/CDNA4 kernels).

The module is built in-tree by `tools/build_native.py` (or `__graft_entry__.build()`).
If it is missing we build it on first import when a toolchain is present; otherwise the
import fails loudly - there is no pure-Python fallback for the runtime or the kernels.
"""
from __future__ import annotations

import importlib
import os
import sys
from pathlib import Path

_ROOT = Path(__file__).resolve().parents[1]


def _load():
    try:
        return importlib.import_module("akka_allreduce_1_amd._C")
    except ImportError as first:
        if os.environ.get("MXAR_NO_AUTOBUILD") == "1":
            raise
        builder = _ROOT / "tools" / "build_native.py"
        if not builder.exists():
            raise
        sys.path.insert(0, str(builder.parent))
        try:
            import build_native  # type: ignore

            build_native.build(verbose=False)
        except Exception as e:  # pragma: no cover - only when the toolchain is broken
            raise ImportError(f"native module _C missing and build failed: {e}") from first
        finally:
            sys.path.pop(0)
        return importlib.import_module("akka_allreduce_1_amd._C")


C = _load()
