"""Register budgets of the shipped kernels, read from libecg.so's gfx950 code-object metadata (CPU only).

The latency kernel's coefficient tables go through LDS and are read input by input, an order pinned by an
empty asm per input (csrc/gf_kernels.hip, lat_fold_lds).  Without it the compiler hoists every table into
VGPRs: 243 VGPRs for RS(10,4) (two waves per SIMD) and scratch spills for a 16-input, 8-output tile
(profiles/r04/lat_tables/).  These checks keep that from coming back unnoticed with a compiler change, and
check that no kernel uses scratch memory at all.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "erasure-codes-prototype_amd", "lib", "libecg.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _metadata():
    """{kernel symbol: {field: int}} from the code object's AMDGPU metadata note."""
    with tempfile.TemporaryDirectory() as d:
        bundle, co = os.path.join(d, "fatbin.bin"), os.path.join(d, "gfx950.co")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={bundle}", LIB, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={bundle}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out = {}
    for blk in re.split(r"\n\s+- \.", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name:
            continue
        fields = {k: int(v) for k, v in re.findall(r"\.(\w+):\s+(\d+)\s*$", blk, re.M)}
        out[name.group(1)] = fields
    return out


@pytest.fixture(scope="module")
def meta():
    if not os.path.exists(LIB):
        pytest.skip("libecg.so not built")
    return _metadata()


def test_no_kernel_uses_scratch(meta):
    assert len(meta) > 400
    bad = {n: f for n, f in meta.items() if f.get("private_segment_fixed_size", 0) or f.get("vgpr_spill_count", 0)}
    assert not bad, list(bad)[:5]


def test_latency_kernels_fit_four_waves_per_simd(meta):
    lat = {n: f for n, f in meta.items() if "gf_lat_dword_kernel" in n}
    assert len(lat) == 192
    assert all(f["sgpr_spill_count"] == 0 for f in lat.values()), [n for n, f in lat.items() if f["sgpr_spill_count"]][:3]
    worst = max(f["vgpr_count"] for f in lat.values())
    assert worst <= 128, worst  # 512 VGPRs per SIMD lane / 4 waves


def test_headline_kernels_do_not_spill(meta):
    # gf_vec_kernel<MT, STRIDED (2), NT 3, BIN>: the encode (MT = 4) and decode (MT = 1) of the bench line
    head = {n: f for n, f in meta.items() if re.search(r"gf_vec_kernelILi[1-4]ELi2ELi3ELb[01]E", n)}
    assert len(head) == 8
    assert all(f["sgpr_spill_count"] == 0 for f in head.values())


def test_call_worker_tables_in_lds(meta):
    (w,) = [f for n, f in meta.items() if "gf_call_worker_kernel" in n]
    assert w["sgpr_spill_count"] < 200, w  # 1324 with its tables in SGPRs
    assert w["group_segment_fixed_size"] >= 4 * 64 * 32  # the per-wave table slices
