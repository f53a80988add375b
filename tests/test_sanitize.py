"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer + LeakSanitizer, and the engine's
concurrency under ThreadSanitizer (CPU only; the TSan tests are at the end).

tools/sanitize_host.sh rebuilds every host translation unit of libecg with -fsanitize=address,undefined
(the kernel file for its host side only: nothing here launches a kernel) and runs
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


def _tsan(variant, threads, ops, seed=1):
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "tsan_host.sh"), variant, str(threads), str(ops), str(seed)],
                       capture_output=True, text=True, timeout=900)
    return p.returncode, p.stdout, p.stderr


@pytest.mark.skipif(not shutil.which("/opt/rocm/lib/llvm/bin/clang++"), reason="needs ROCm clang (TSan runtime)")
def test_engine_concurrency_under_thread_sanitizer():
    """the engine's concurrency under ThreadSanitizer, on the CPU.  tools/tsan_host.sh
    links libecg's host code (and gf_kernels.hip's host side) against tests/tsan/hip_stub.cpp -- a CPU
    stand-in for the HIP runtime that emulates the library's kernels bit-exactly and checks that no table a
    pending launch reads is rewritten from another stream -- and runs tests/tsan/engine_race.cpp: a
    hipStreamPerThread eviction scenario, then 8 threads of random proxy-like calls (device tier on own /
    per-thread / null streams, scopes with scratch partials, deferred and synchronous host tier, host
    pipelines, the ErasureCode facade, stream churn, reclaims) with a program cache of 4, every result
    against the oracle.  Zero reports, zero hazards, every check passed."""
    rc, out, err = _tsan("product", 8, 150, 7)
    tail = (out + err)[-4000:]
    assert rc == 0, tail
    assert "WARNING: ThreadSanitizer" not in err, tail
    assert "0 failed, 0 device-time hazards" in out, tail


@pytest.mark.skipif(not shutil.which("/opt/rocm/lib/llvm/bin/clang++"), reason="needs ROCm clang (TSan runtime)")
def test_thread_sanitizer_reports_a_seeded_race():
    """The harness can see a race: the ECG_TEST_TSAN_SEEDED_RACE build pushes evicted program sets onto the
    retirement list without its lock (engine.cpp Engine::retire), and ThreadSanitizer must say so."""
    rc, out, err = _tsan("seeded", 8, 100)
    assert rc != 0
    assert "WARNING: ThreadSanitizer: data race" in err, (out + err)[-3000:]
    assert "Engine::retire" in err, err[-3000:]


@pytest.mark.skipif(not shutil.which("/opt/rocm/lib/llvm/bin/clang++"), reason="needs ROCm clang (TSan runtime)")
def test_per_thread_stream_cover_hazard_is_detected_on_the_round4_keying():
    """round 4 covered a program set noted on hipStreamPerThread from whichever thread
    swept, on that thread's own per-thread stream.  The ECG_TEST_PER_THREAD_SHARED_KEY build restores that
    keying; the harness's per-thread scenario must then report a device-time hazard (a pool block rewritten
    from thread B's stream while thread A's queued launch still reads it), and the product build must not
    (test_engine_concurrency_under_thread_sanitizer)."""
    rc, out, err = _tsan("sharedkey", 2, 10)
    assert rc != 0
    assert "DEVICE-TIME HAZARD" in err, (out + err)[-3000:]
    assert "per-thread scenario: 0 device-time hazards" not in out
