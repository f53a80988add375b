"""GPU parity of bench.py's `families` workload: every ErasureCode class (ec_factory, metadata.cpp:48-77) through
the facade as the proxies call it -- per-stripe encode, single- and two-block repairs planned by the class's own
generate_repair_plan (helper / main partial decodes + perform_addition, partials declared scratch), and the
two-erasure degraded-read decode -- issued from C++ (loopback/replay.cpp ecg_replay_calls) in batch scopes, so
the scheduler's multi-program launches (single-op plans of one shape) and earliest-group placement run.

Small blocks with byte-path tails.  Every stripe's rebuilt blocks must equal the encoded ones (poisoned first), and
the oracle's class restatement (oracle/ec_ref.py) run on sampled stripes -- the workload's CPU leg -- must produce
the GPU's bytes for every operation.
"""
import os
import sys
import types

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench_mod():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    sys.path.insert(0, ROOT)
    import bench
    return bench


CLASSES = ["RS(12,4)", "ERS(12,4|x=2,seri_num=1)", "Azure_LRC(12,2,2)", "Azure_LRC+1(12,3,2)", "Optimal_LRC(12,2,2)",
           "Optimal_Cauchy_LRC(12,2,2)", "Uniform_Cauchy_LRC(12,2,2)", "PC(4,1,4,1)", "HPC(4,1,4,1|x=2,seri_num=0)",
           "HVPC(4,1,4,1)", "RS(20,4)", "RS(30,4)"]


@pytest.mark.parametrize("cls", CLASSES)
def test_family_vs_oracle(bench_mod, ecg, cls):
    import ecg_dist as D
    assert [f[0] for f in bench_mod.FAMILIES] == CLASSES
    # stripes=1: one stripe per pattern (families rounds S up to whole rounds of the n single-block patterns)
    a = types.SimpleNamespace(block_size=4096 + 48, steps=1, warmup=1, forms=cls, no_cpu_baseline=False,
                              stripes=1, working_set_gib=0.0)
    r = D.from_env()
    line = bench_mod.families(a, r)
    assert list(line["classes"]) == [cls]
    cv = line["classes"][cls]
    assert "error" not in cv, cv
    for op, row in cv["ops"].items():
        assert row["verified"], (cls, op)
        assert row["executed_over_algorithmic"] == 1.0, (cls, op, row["executed_over_algorithmic"])
        assert row["launches_per_batch"] <= 8, (cls, op, row["launches_per_batch"])  # <= 4 products, + byte tails
    chk = cv["cpu_check"]
    assert "error" not in chk, chk
    for op in cv["ops"]:
        assert chk[op]["matches_gpu"], (cls, op)
