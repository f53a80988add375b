"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer + LeakSanitizer (CPU only).

tools/sanitize_host.sh rebuilds every host translation unit of libecg with -fsanitize=address,undefined
(the HIP kernels keep their device code; host flags go through -Xarch_host) and runs
tests/sanitize/host_fuzz.cpp.  The driver exercises these parts over randomly drawn parameters of
every code family:
- the matrix builders and Gauss-Jordan;
- the decode planners;
- partitions and repair plans;
- the index helpers;
- the partial-coding matrices.
It makes no GPU call: execution steps fail cleanly with ECG_EHIP after planning.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_host_code_sanitizers():
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh")], capture_output=True, text=True,
                       timeout=900)
    tail = (p.stdout + p.stderr)[-4000:]
    assert p.returncode == 0, tail
    assert "host fuzz done" in p.stdout, tail
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, tail
