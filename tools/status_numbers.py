#!/usr/bin/env python3
"""The status numbers DESIGN.md §0, README.md and BASELINE.md quote, read from one final pass.

    python tools/status_numbers.py [profiles/r05/final7]

Prints the bench line's headline figures, the committed headline profile and PMC traffic, config 5, the
host path, configs 3 and 4 (with the committed per-form profile when present) and the GPU-suite tally, each
with the precision the docs use."""
import json
import os
import re
import sys


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r05/final7"
    line = json.loads(open(os.path.join(d, "bench.log")).read().strip().splitlines()[-1])
    prof = json.load(open(os.path.join(d, "headline_profile.json")))
    pmc = json.load(open(os.path.join(d, "pmc_traffic.json")))
    r = line["roofline"]
    c5, hp, cpu = line["config5"], line["host_path"], line["cpu_baseline"]
    e, dc = prof["encode"], prof["decode"]
    print(f"value {line['value']:.0f} GiB/s, {line['ms_per_step']:.3f} ms/step")
    print(f"encode HIP events {r['frac']:.3f} ({line['encode_ms']:.3f} ms); decode {r['decode_frac']:.3f} "
          f"({line['decode_ms']:.3f} ms)")
    print(f"encode rocprof avg {e['avg_ms']:.3f} ms = {e['frac_avg']:.3f} (median {e['median_ms']:.3f} ms = "
          f"{e['frac_median']:.3f}); decode avg {dc['avg_ms']:.3f} ms = {dc['frac_avg']:.3f}")
    print(f"PMC traffic: encode {pmc['encode_hbm_bytes_per_launch'] / e['algorithmic_bytes_per_launch']:.6f} x, "
          f"decode {pmc['decode_hbm_bytes_per_launch'] / dc['algorithmic_bytes_per_launch']:.5f} x algorithmic; "
          f"libecg {pmc['libecg_sha16']} (profile {prof['libecg_sha16']})")
    print(f"cpu_baseline {cpu['value']:.1f} {cpu['unit']} ({cpu['cores']} threads): GPU line {line['value'] / cpu['value']:.0f}x")
    print(f"config5 {c5['aggregate_GiBps']:.0f} GiB/s, frac {c5['hbm_frac_max']:.3f}, checksum {c5['parity_checksum']} "
          f"equal to N=1: {c5['checksum_equals_n1']}")
    print(f"host_path {hp['encode_GiBps']:.1f} / {hp['decode_GiBps']:.1f} GiB/s")
    for key in ("config3", "config4"):
        c = line.get(key, {})
        if "forms" not in c:
            print(f"{key}: {c}")
            continue
        forms = ", ".join(f"{n} {v['algorithmic_frac']:.3f}" + (f" [{v['kernel']} {v['profile_kernel_avg_us']} us]"
                                                                 if v.get("kernel") else "")
                          for n, v in c["forms"].items())
        cb = c.get("cpu_baseline", {})
        print(f"{key}: {forms}; verified all ranks {c.get('verified_all_ranks')}; cpu {cb.get('value')} {cb.get('unit')}")
    if "build" in line:
        b = line["build"]
        print(f"build: libecg {b.get('libecg_sha16')} sources {b.get('sources_sha16')} "
              f"built by build() from these sources: {b.get('built_by_build_from_these_sources')}")
    log = open(os.path.join(d, "pytest_gpu.log")).read()
    m = re.search(r"(\d+) passed(?:, (\d+) skipped)?", log)
    print(f"GPU suite: {m.group(1)} passed, {m.group(2) or 0} skipped")


if __name__ == "__main__":
    main()
