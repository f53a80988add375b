#!/usr/bin/env python3
"""Check a bench.py line at world N against the N = 1 line over the same global stripes
(tools/gpu_dist_rehearsal8.sh): combined headline parity checksum and config-5 checksum equal, every
cross-GPU object verified on all ranks, per-rank arrays of length N.
usage: check_rehearsal_n.py N1_LOG NN_LOG N"""
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


one, many, n = line(sys.argv[1]), line(sys.argv[2]), int(sys.argv[3])
checks = []


def check(what, ok, detail=""):
    checks.append(ok)
    print(f"{'ok ' if ok else 'BAD'} {what} {detail}")


c1 = D.combine(int(x, 16) for x in one["parity_checksums"])
cn = D.combine(int(x, 16) for x in many["parity_checksums"])
check("n_gpus", many["n_gpus"] == n, many["n_gpus"])
check("headline checksum N=1 == N", c1 == cn and len(many["parity_checksums"]) == n, f"{c1:016x} / {cn:016x}")
for key in ("encode_frac", "decode_frac", "encode_ms", "decode_ms"):
    check(f"per_rank.{key} has {n} entries", len(many["per_rank"][key]) == n, many["per_rank"][key])
c5a, c5b = one["config5"], many["config5"]
check("config5 checksum N=1 == N", c5a["parity_checksum"] == c5b["parity_checksum"],
      f"{c5a['parity_checksum']} / {c5b['parity_checksum']}")
check("config5 per-rank shares", len(c5b["stripes_per_rank"]) == n and sum(c5b["stripes_per_rank"]) ==
      sum(c5a["stripes_per_rank"]), c5b["stripes_per_rank"])
check("config5 hbm_frac_per_rank", len(c5b["hbm_frac_per_rank"]) == n, c5b["hbm_frac_per_rank"])
for obj in ("ring_repair", "global_ring_repair", "merge_ring", "host_path", "config3", "config4", "families"):
    for nm, x in (("N=1", one), (f"N={n}", many)):
        o = x.get(obj, {})
        check(f"{obj} {nm} verified_all_ranks", o.get("verified_all_ranks") is True,
              {k: v for k, v in o.items() if k in ("backend", "n_gpus", "repairs_per_s", "merges_per_s",
                                                      "encode_GiBps", "decode_GiBps", "error")})
print("REHEARSAL", "OK" if all(checks) else "MISMATCH", f"({sum(checks)}/{len(checks)} checks)")
sys.exit(0 if all(checks) else 1)
