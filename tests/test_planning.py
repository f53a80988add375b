"""Partitioning and repair planning (csrc/planning.cpp via the C ABI) against the oracle restatement
(oracle/plan_ref.py) and hand-derived expectations.  Host logic only: no GPU needed."""
import itertools
import json
import os
import random
import zlib

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))["codes"]
TYPE_NAMES = {0: "RS", 1: "ERS", 2: "AZURE_LRC", 3: "AZURE_LRC_1", 4: "OPTIMAL_LRC", 5: "OPTIMAL_CAUCHY_LRC",
              6: "UNIFORM_CAUCHY_LRC", 7: "PC", 8: "Hierachical_PC", 9: "HV_PC"}
# golden codes + the BASELINE configurations' codes + a few shapes with ragged groups
EXTRA = [("RS", {"k": 6, "m": 3}), ("AZURE_LRC", {"k": 12, "l": 3, "g": 3}), ("AZURE_LRC", {"k": 10, "l": 3, "g": 2}),
         ("AZURE_LRC_1", {"k": 12, "l": 4, "g": 2}), ("OPTIMAL_LRC", {"k": 10, "l": 3, "g": 2}),
         ("OPTIMAL_CAUCHY_LRC", {"k": 12, "l": 3, "g": 2}), ("UNIFORM_CAUCHY_LRC", {"k": 10, "l": 3, "g": 3}),
         ("PC", {"k1": 3, "m1": 2, "k2": 3, "m2": 2}), ("HV_PC", {"k1": 4, "m1": 1, "k2": 4, "m2": 1})]
CODES = [(TYPE_NAMES[c["type"]], c["params"]) for c in GOLDEN] + EXTRA
IDS = [f"{n}{tuple(p.values())}" for n, p in CODES]


def make(ecg, name, params, rule, seed=None):
    from oracle import plan_ref as P
    p = ecg.ec_factory(ecg.ECTYPE[name], ecg.CodingParameters(**params))
    o = P.planner_for(name, params)
    p.placement_rule = rule
    o.placement_rule = int(rule)
    if seed is not None:
        p.set_random_seed(seed)
        o.set_random_seed(seed)
    return p, o


def failure_sets(n, rng):
    sets = [[i] for i in range(n)] + [list(c) for c in itertools.combinations(range(n), 2)]
    for size in (3, 4, 5):
        combos = list(itertools.combinations(range(n), size))
        sets += [list(c) for c in rng.sample(combos, min(40, len(combos)))]
    return sets


def plans_tuple(plans):
    return [(bool(p.local_or_column), list(p.failure_idxs), [list(h) for h in p.help_blocks]) for p in plans]


@pytest.mark.parametrize("name,params", CODES, ids=IDS)
def test_partitions_match_oracle(ecg, name, params):
    rules = [ecg.PlacementRule.FLAT, ecg.PlacementRule.OPTIMAL] + (
        [ecg.PlacementRule.SUB_OPTIMAL] if name == "AZURE_LRC" else [])
    for rule in rules:
        p, o = make(ecg, name, params, rule)
        assert p.generate_partition() == o.generate_partition(), rule
    for seed in range(12):
        p, o = make(ecg, name, params, ecg.PlacementRule.RANDOM, seed)
        assert p.generate_partition() == o.generate_partition(), seed


@pytest.mark.parametrize("name,params", CODES, ids=IDS)
def test_partitions_cover_every_block_once(ecg, name, params):
    for rule, seed in [(ecg.PlacementRule.FLAT, None), (ecg.PlacementRule.OPTIMAL, None)] + \
                      [(ecg.PlacementRule.RANDOM, s) for s in range(20)]:
        p, o = make(ecg, name, params, rule, seed)
        plan = p.generate_partition()
        blocks = sorted(b for part in plan for b in part)
        assert blocks == list(range(p.k + p.m)), (rule, plan)
        if rule == ecg.PlacementRule.RANDOM:  # single-region fault tolerance bounds (rs.cpp:86, lrc.cpp:226)
            if name in ("RS", "ERS"):
                assert max(len(x) for x in plan) <= params["m"]
            elif "LRC" in name:
                assert max(len(x) for x in plan) <= params["g"] + 1


@pytest.mark.parametrize("name,params", CODES, ids=IDS)
@pytest.mark.parametrize("rule", ["FLAT", "OPTIMAL", "RANDOM"])
def test_repair_plans_match_oracle(ecg, name, params, rule):
    rng = random.Random(zlib.crc32(repr((name, sorted(params.items()), rule)).encode()))
    p, o = make(ecg, name, params, ecg.PlacementRule[rule], seed=7)
    assert p.generate_partition() == o.generate_partition()
    n = p.k + p.m
    for fs in failure_sets(n, rng):
        if name not in ("RS", "ERS", "PC", "Hierachical_PC", "HV_PC"):
            assert p.check_if_decodable(fs) == o.check_if_decodable(fs), fs
        dec_p, plans_p = p.generate_repair_plan(fs)
        dec_o, plans_o = o.generate_repair_plan(fs)
        assert dec_p == dec_o, fs
        if dec_p:
            assert plans_tuple(plans_p) == plans_tuple(plans_o), fs


def test_survey_config3_partition_and_repair(ecg):
    """Azure-LRC(12,2,2) OPTIMAL partition {0,1,2},{3,4,5},{6,7,8},{9,10,11},
    {14,15,12,13}; repairing data block 0 locally reads its group (1..5 + local parity 14), partition by
    partition (lrc.cpp:249-262)."""
    az = ecg.ec_factory(ecg.ECTYPE.AZURE_LRC, ecg.CodingParameters(k=12, l=2, g=2))
    assert az.generate_partition() == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10, 11], [14, 15, 12, 13]]
    assert az.grouping_information() == [[0, 1, 2, 3, 4, 5, 14], [6, 7, 8, 9, 10, 11, 15], [12, 13]]
    dec, plans = az.generate_repair_plan([0])
    assert dec and len(plans) == 1 and plans[0].local_or_column
    assert plans[0].help_blocks == [[1, 2], [3, 4, 5], [14]]
    dec, plans = az.generate_repair_plan([12])  # a global parity: k survivors, own partition first
    assert dec and not plans[0].local_or_column
    assert plans[0].help_blocks == [[13], [0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10]]
    assert sum(len(h) for h in plans[0].help_blocks) == 12
    assert az.self_information() == "Azure_LRC(12,2,2)"


def test_rs_repair_reads_k_blocks(ecg):
    """RS(10,4) OPTIMAL: partitions of m = 4; every single repair reads exactly k helpers, the failed
    block's partition first (rs.cpp:118-180)."""
    rs = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=10, m=4))
    assert rs.generate_partition() == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13]]
    for f in range(14):
        dec, plans = rs.generate_repair_plan([f])
        h = plans[0].help_blocks
        assert dec and sum(len(x) for x in h) == 10 and f not in sum(h, [])
        assert set(h[0]) <= set(rs.partition_plan[f // 4])
    _, plans = rs.generate_repair_plan([3, 11])
    assert plans[0].help_blocks == [[0, 1, 2], [8, 9, 10], [4, 5, 6, 7]]


def test_pc_iterative_plan(ecg):
    """PC(4,1,4,1): failures {0, 1, 5}: column 0 first, then row 0 (via the row code's partitions), then
    column 1 (pc.cpp:451-551), worked by hand."""
    pc = ecg.ec_factory(ecg.ECTYPE.PC, ecg.CodingParameters(k1=4, m1=1, k2=4, m2=1))
    pc.generate_partition()
    dec, plans = pc.generate_repair_plan([0, 1, 5])
    assert dec
    assert [(p.local_or_column, p.failure_idxs, p.help_blocks) for p in plans] == [
        (True, [0], [[4, 8, 12, 20]]), (False, [1], [[0], [2], [3], [16]]), (True, [5], [[1, 9, 13, 21]])]
    dec, _ = pc.generate_repair_plan([0, 1, 4, 5])  # a 2x2 square: undecodable
    assert not dec


def test_planning_bad_arguments(ecg):
    rs = ecg.ec_factory(ecg.ECTYPE.RS, ecg.CodingParameters(k=4, m=2))
    with pytest.raises(ecg.EcgError):
        rs.placement_rule = 7
    with pytest.raises(ecg.EcgError):
        rs.placement_rule = ecg.PlacementRule.SUB_OPTIMAL
        rs.generate_partition()
    rs.placement_rule = ecg.PlacementRule.OPTIMAL
    rs.generate_partition()
    with pytest.raises(ecg.EcgError):
        rs.generate_repair_plan([6])
    with pytest.raises(ecg.EcgError):
        rs.grouping_information()


def test_get_coding_parameters_per_family(ecg):
    """get_coding_parameters writes the fields each class owns (erasure_code.cpp:12-17, lrc.cpp:14-21,
    pc.cpp:20-29) and init_coding_parameters copies local_or_column where the reference does
    (erasure_code.cpp:5-10, lrc.cpp:5-12) and not where it does not (ERS, rs.cpp:282-288)."""
    E = ecg.ECTYPE
    cp = ecg.CodingParameters
    rs = ecg.ec_factory(E.RS, cp(k=10, m=4))
    g = rs.get_coding_parameters()
    assert (g.k, g.m, g.local_or_column) == (10, 4, False)
    rs.init_coding_parameters(cp(k=6, m=3, local_or_column=True))
    g = rs.get_coding_parameters()
    assert (g.k, g.m, g.local_or_column, rs.k, rs.m) == (6, 3, True, 6, 3)
    ers = ecg.ec_factory(E.ERS, cp(k=4, m=2, x=2, seri_num=1))
    ers.init_coding_parameters(cp(k=4, m=2, x=2, seri_num=1, local_or_column=True))
    assert ers.get_coding_parameters().local_or_column is False
    az = ecg.ec_factory(E.AZURE_LRC, cp(k=12, l=2, g=2))
    g = az.get_coding_parameters()
    assert (g.k, g.l, g.g, g.m) == (12, 2, 2, 4)
    az.init_coding_parameters(cp(k=12, l=2, g=2, local_or_column=True))
    assert az.get_coding_parameters().local_or_column is True
    pc = ecg.ec_factory(E.PC, cp(k1=4, m1=1, k2=4, m2=1))
    g = pc.get_coding_parameters()
    assert (g.k1, g.m1, g.k2, g.m2, g.k, g.m) == (4, 1, 4, 1, 16, 9)
    hv = ecg.ec_factory(E.HV_PC, cp(k1=4, m1=1, k2=4, m2=1))
    assert (hv.k, hv.m) == (16, 8)
