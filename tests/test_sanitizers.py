"""Race / memory-error detection for the host runtime: the protocol cores,
threaded actor system, TCP cluster and fault injector built with ThreadSanitizer and
AddressSanitizer (+LeakSanitizer) and driven by csrc/tests/runtime_stress.cc."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["thread", "address", "undefined"])
def test_runtime_under_sanitizer(kind):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sanitize.py"), "--sanitize", kind],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "runtime_stress: OK" in r.stdout
