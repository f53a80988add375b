#!/usr/bin/env python3
"""Check the completion-flag epilogue in the gfx950 ISA of libecg.so (or of any HIP object / bundle).

A host-tier call polls per-workgroup flags in mapped host memory instead of synchronising the stream
(DESIGN.md §4b).  A flag may be posted only after the workgroup's output is visible to the host, i.e. in
every kernel that posts flags (it contains `buffer_wbl2`), the instruction stream must read

    s_waitcnt vmcnt(0)      every wave: its own output stores have completed
    s_barrier               the workgroup has met (no vector memory op in between)
    buffer_wbl2 sc0 sc1     lane 0: L2 written back, system scope
    s_waitcnt vmcnt(0)      the write-back has completed            <- the wait the compiler once dropped
    global_store ... sc0 sc1  the flag (system scope; the first vector store after the write-back)

(csrc/gf_done_flag.hpp).  Without the second wait the host read 3 of 2617 rebuilt blocks stale in round 2.
Only system-scope write-backs count (`buffer_wbl2 sc0 sc1`); agent-scope ones stay on the device.
The code object is taken from the library's .hip_fatbin section with objcopy + clang-offload-bundler in a
temporary directory and disassembled with llvm-objdump; nothing is written into the repository.

usage: tools/check_flag_isa.py [path/to/libecg.so | object.o]   (exit 0 = every flag kernel passes)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
VMEM = re.compile(r"^(global|flat|buffer|scratch)_(load|store|atomic)")
STORE = re.compile(r"^(global|flat|buffer|scratch)_(store|atomic)")
WAIT_VM0 = re.compile(r"^s_waitcnt\b.*\bvmcnt\(0\)")


def disassemble(path):
    """gfx950 disassembly (text) of a shared library with a .hip_fatbin section, or of an offload bundle."""
    with tempfile.TemporaryDirectory() as d:
        bundle = os.path.join(d, "fatbin.bin")
        if subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={bundle}", path, os.path.join(d, "x")],
                          capture_output=True).returncode != 0:
            bundle = path  # not an ELF with a fat binary: take the file itself as the bundle
        co = os.path.join(d, "gfx950.co")
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={bundle}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "-C", co], check=True,
                              capture_output=True, text=True).stdout


def kernels(text):
    """{symbol: [instruction mnemonics + operands]} from llvm-objdump output."""
    out, name = {}, None
    for ln in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            name = m.group(1)
            out[name] = []
            continue
        if name is None:
            continue
        ins = ln.split("//")[0].strip()
        if ins and not ins.endswith(":"):
            out[name].append(ins)
    return out


SYS_WBL2 = re.compile(r"^buffer_wbl2\b.*\bsc0\b.*\bsc1\b")


def check_kernel(ins):
    """Problems with the flag epilogues of one kernel's instruction list (empty = ok).  An epilogue is a
    system-scope write-back (`buffer_wbl2 sc0 sc1`, what a release to the host compiles to); an agent-scope
    one (`buffer_wbl2 sc1`, e.g. the call worker publishing a descriptor to its other workgroups) stays
    on the device and is not a host flag."""
    probs = []
    wbl = [i for i, x in enumerate(ins) if SYS_WBL2.match(x)]
    for w in wbl:
        # the flag store: the first vector store after the write-back, with a vmcnt(0) wait before it
        f = next((i for i in range(w + 1, len(ins)) if STORE.match(ins[i])), None)
        if f is None:
            probs.append(f"@{w} no store after buffer_wbl2")
            continue
        if not any(WAIT_VM0.match(x) for x in ins[w + 1:f]):
            probs.append(f"@{w} flag store @{f} not preceded by s_waitcnt vmcnt(0) after buffer_wbl2")
        if "sc0" not in ins[f] or "sc1" not in ins[f]:
            probs.append(f"@{f} flag store is not system scope: {ins[f]}")
        # before it: s_barrier, with no vector memory op between the barrier and the write-back, and a
        # vmcnt(0) wait after the wave's last vector memory op and before the barrier
        b = next((i for i in range(w - 1, -1, -1) if ins[i].startswith("s_barrier")), None)
        if b is None:
            probs.append(f"@{w} no s_barrier before buffer_wbl2")
            continue
        if any(VMEM.match(x) for x in ins[b + 1:w]):
            probs.append(f"@{w} vector memory op between s_barrier @{b} and buffer_wbl2")
        last_vm = next((i for i in range(b - 1, -1, -1) if VMEM.match(ins[i])), -1)
        if not any(WAIT_VM0.match(x) for x in ins[last_vm + 1:b]):
            probs.append(f"@{b} s_barrier not preceded by s_waitcnt vmcnt(0) after the last vector memory op @{last_vm}")
    return probs


def check(text):
    """(flag-posting kernels, {kernel: problems}) for a disassembly."""
    ks = kernels(text)
    flagged = {n: ins for n, ins in ks.items() if any(SYS_WBL2.match(x) for x in ins)}
    bad = {n: p for n, ins in flagged.items() if (p := check_kernel(ins))}
    return ks, flagged, bad


def main(argv):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = argv[1] if len(argv) > 1 else os.path.join(root, "erasure-codes-prototype_amd", "lib", "libecg.so")
    ks, flagged, bad = check(disassemble(path))
    print(f"{path}: {len(ks)} kernels, {len(flagged)} post completion flags, {len(bad)} with a bad epilogue")
    for n, p in list(bad.items())[:10]:
        print(f"  {n}:\n    " + "\n    ".join(p))
    return 0 if flagged and not bad else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv))
