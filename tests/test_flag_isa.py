"""The completion-flag epilogue, pinned in the ISA.

Host-tier calls complete by polling per-workgroup flags.  Correctness rests on an
explicit `s_waitcnt vmcnt(0)` between the L2 write-back and the flag store that the compiler once dropped
(3 of 2617 rebuilt blocks read stale in round 2).  The GPU test for it is probabilistic; this one is not:
every flag-posting kernel in the shipped libecg.so is disassembled and its epilogue checked
(tools/check_flag_isa.py), and a probe built with the wait removed must fail the same check.  CPU only."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_flag_isa as C  # noqa: E402

LIB = os.path.join(ROOT, "erasure-codes-prototype_amd", "lib", "libecg.so")


def test_every_flag_kernel_of_libecg_has_the_full_release_sequence():
    ks, flagged, bad = C.check(C.disassemble(LIB))
    # gf_lat_dword_kernel: 8 row tiles x 2 flavours x 6 input buckets x 2 (eager or not) = 192,
    # gf_vec_kernel in INLINE_LAT mode (mode 3): 8 x 2 x 4 NT policies = 64, plus the wide BINARY tiles
    # (9-16 rows, default NT policy only) = 8
    lat = [n for n in ks if "gf_lat_dword_kernel" in n]
    assert len(lat) == 192 and all(n in flagged for n in lat)
    inline_lat = re.compile(r"gf_vec_kernel<\d+, 3, \d+, (true|false)>")
    vec_lat = [n for n in ks if inline_lat.search(n)]
    assert len(vec_lat) == 72 and all(n in flagged for n in vec_lat)
    # and the resident call worker (ECG_OPT_CALL_WORKER), which posts the same flags per call
    worker = [n for n in ks if "gf_call_worker_kernel" in n]
    assert len(worker) == 1 and worker[0] in flagged
    assert len(flagged) == 265
    assert not bad, {n: p for n, p in list(bad.items())[:3]}
    # no other kernel writes the L2 back to the host (the batched kernels never post flags)
    assert all("gf_lat_dword_kernel" in n or inline_lat.search(n) or n in worker for n in flagged)


def _probe(tmp_path, drop):
    out = tmp_path / ("drop.o" if drop else "keep.o")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-c",
           "-I", os.path.join(ROOT, "erasure-codes-prototype_amd", "csrc"),
           os.path.join(ROOT, "tests", "isa", "flag_probe.hip"), "-o", str(out)]
    if drop:
        cmd.insert(1, "-DECG_TEST_DROP_FLAG_WAIT")
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return C.check(C.disassemble(str(out)))


def test_checker_rejects_the_epilogue_without_its_wait(tmp_path):
    _, flagged, bad = _probe(tmp_path, drop=False)
    assert len(flagged) == 1 and not bad
    _, flagged, bad = _probe(tmp_path, drop=True)
    assert len(flagged) == 1 and len(bad) == 1
    (problems,) = bad.values()
    assert any("not preceded by s_waitcnt vmcnt(0) after buffer_wbl2" in p for p in problems), problems


def test_checker_on_synthetic_sequences():
    good = ["global_store_dword v[2:3], v1, off nt", "s_waitcnt vmcnt(0)", "s_barrier", "s_and_saveexec_b64 s[8:9], vcc",
            "buffer_wbl2 sc0 sc1", "s_waitcnt vmcnt(0)", "s_load_dword s8, s[0:1], 0x5b0",
            "global_store_dword v0, v1, s[0:1] sc0 sc1", "s_endpgm"]
    assert C.check_kernel(good) == []
    no_first_wait = [x for i, x in enumerate(good) if i != 1]
    assert any("s_barrier not preceded" in p for p in C.check_kernel(no_first_wait))
    no_second_wait = [x for i, x in enumerate(good) if i != 5]
    assert any("after buffer_wbl2" in p for p in C.check_kernel(no_second_wait))
    not_system = [x.replace(" sc0 sc1", "") if x.startswith("global_store_dword v0") else x for x in good]
    assert any("not system scope" in p for p in C.check_kernel(not_system))
    store_after_barrier = good[:3] + ["global_store_dword v[4:5], v2, off"] + good[3:]
    assert C.check_kernel(store_after_barrier)
    # an agent-scope write-back (the call worker publishing a descriptor to its other workgroups) is not a
    # host flag: not checked, and a kernel with only such write-backs posts no flags
    agent = ["global_store_dword v[2:3], v1, off", "buffer_wbl2 sc1", "global_store_dword v4, v5, s[2:3] sc1"]
    assert C.check_kernel(agent) == []
    assert not C.check("00000000 <k>:\n" + "\n".join("\t" + x for x in agent))[1]
