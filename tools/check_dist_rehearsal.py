#!/usr/bin/env python3
"""Compare bench.py JSON lines of the N=1 and N=2 rehearsal runs (tools/gpu_dist_rehearsal.sh)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "erasure-codes-prototype_amd"))
import ecg_dist as D  # noqa: E402


def line(path):
    for ln in reversed(open(path).read().splitlines()):
        if ln.startswith("{"):
            return json.loads(ln)
    raise SystemExit(f"no JSON line in {path}")


d = sys.argv[1]
rs1, rs2 = line(f"{d}/rs_n1.log"), line(f"{d}/rs_n2.log")
w1, w2 = line(f"{d}/waves_n1.log"), line(f"{d}/waves_n2.log")
ok = True
c1 = D.combine(int(x, 16) for x in rs1["parity_checksums"])
c2 = D.combine(int(x, 16) for x in rs2["parity_checksums"])
print(f"rs-encode-decode: N=1 512 stripes {c1:016x}; N=2 x 256 {c2:016x}; n_gpus={rs2['n_gpus']}")
ok &= c1 == c2 and rs2["n_gpus"] == 2 and len(rs2["parity_checksums"]) == 2
for nm, x in (("N=1", rs1), ("N=2", rs2)):  # the default line's config5 object (full 65536 x 4 MiB batch)
    c5 = x["config5"]
    print(f"config5 {nm}: {c5['parity_checksum']} (N=1 reference {c5['parity_checksum_n1']}), "
          f"stripes per rank {c5['stripes_per_rank']}, hbm_frac per rank {c5['hbm_frac_per_rank']}")
    ok &= c5["checksum_equals_n1"] is True and len(c5["hbm_frac_per_rank"]) == x["n_gpus"]
print("per_rank", rs2["per_rank"])
print("ring_repair N=2", rs2.get("ring_repair"))
ok &= rs2.get("ring_repair", {}).get("verified_all_ranks") is True
for nm, x in (("N=1", rs1), ("N=2", rs2)):  # RCCL self-exchange at N = 1, gloo in the shared-GPU N = 2
    if nm == "N=1":
        print("ring_repair N=1", x.get("ring_repair"))
        ok &= x.get("ring_repair", {}).get("verified_all_ranks") is True
    print(f"global_ring_repair {nm}", x.get("global_ring_repair"))
    ok &= x.get("global_ring_repair", {}).get("verified_all_ranks") is True
    print(f"merge_ring {nm}", x.get("merge_ring"))
    ok &= x.get("merge_ring", {}).get("verified_all_ranks") is True
    print(f"host_path {nm}", x.get("host_path"))
    ok &= x.get("host_path", {}).get("verified_all_ranks") is True
ok &= len(rs2["per_rank"]["encode_frac"]) == 2 and len(rs2["per_rank"]["decode_frac"]) == 2
spawn = f"{d}/rs_n2_selfspawn.log"
if os.path.exists(spawn):  # bench.py --gpus 2 started its own ranks (torch.distributed.run child)
    rs2s = line(spawn)
    c2s = D.combine(int(x, 16) for x in rs2s["parity_checksums"])
    print(f"rs-encode-decode self-spawned: N=2 x 256 {c2s:016x}; n_gpus={rs2s['n_gpus']}")
    ok &= c2s == c1 and rs2s["n_gpus"] == 2
print(f"rs4m-waves: N=1 {w1['parity_checksum']}; N=2 {w2['parity_checksum']}")
ok &= w1["parity_checksum"] == w2["parity_checksum"]
for f in ("lrc_n2", "pc_n2", "ring_n2"):
    x = line(f"{d}/{f}.log")
    print(f, "n_gpus", x["n_gpus"], "verified", x.get("verified", "-"))
    ok &= x["n_gpus"] == 2 and x.get("verified", True) is True
print("REHEARSAL", "OK" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
