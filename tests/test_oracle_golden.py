"""The oracle (oracle/hj3d_oracle.c) against the golden fixtures made by the REAL reference.

Pins: the bit-exact input generators (mt19937 + libstdc++ shuffle / uniform_int /
generate_canonical + the reference's Zipf sampler and vec_permute), and every counter,
statistic and output checksum of the six experiment-1 plans and the two experiment-4 plans.
CPU only.
"""
import os
import numpy as np
import pytest

import oracle as O
from conftest import load_golden

EXP1 = [x for x in load_golden("exp1_*.json") if x[1]["nS"] <= 100_000_000]  # config D: GPU box only
EXP4 = load_golden("exp4_*.json")
STAT_KEYS = ("nb", "empty", "entries", "distinct", "cc0_min", "cc0_max", "cc0_sum", "cc0_cnt",
             "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")


def exp1_inputs(g):
    _, nR, nS, skew, theta, t, b = g["generator_args"][:7]
    Rk, Sa, fk = O.gen_exp1(nR, nS, bool(skew), theta, t)
    return Rk, Sa, fk, b


@pytest.mark.parametrize("name,g", EXP1, ids=[n for n, _ in EXP1])
def test_exp1_generator_bit_exact(name, g):
    Rk, Sa, fk, _ = exp1_inputs(g)
    assert fk == g["fkMax"]
    assert Rk[:16].tolist() == g["head_Rk"]
    assert Sa[:16].tolist() == g["head_Sa"]
    assert O.colsum(Rk) == g["colsum_Rk"]
    assert O.colsum(Sa) == g["colsum_Sa"]
    if "Rk" in g:
        assert Rk.tolist() == g["Rk"] and Sa.tolist() == g["Sa"]
    assert O.num_distinct(Sa) == g["numDvSa"]


@pytest.mark.parametrize("name,g", EXP1, ids=[n for n, _ in EXP1])
def test_exp1_plans_match_reference(name, g):
    if g["nS"] > 2_000_000:
        pytest.skip("large fixture covered by the GPU parity suite")
    Rk, Sa, _, b = exp1_inputs(g)
    nR, nS = len(Rk), len(Sa)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    nbR, nbS = max(nR // b, 1), max(g["numDvSa"] // b, 1)
    runs = {
        "Csr": O.chain_plan(R, 0, S, 1, nbR, True), "CsrUU": O.chain_plan(R, 0, S, 1, nbR, False),
        "Crs": O.chain_plan(S, 1, R, 0, nbS, False), "Nsr": O.nested_plan(R, 0, S, 1, nbR, True),
        "Nrs": O.nested_plan(S, 1, R, 0, nbS, True), "NrsNU": O.nested_plan(S, 1, R, 0, nbS, False),
    }
    for plan, r in runs.items():
        ref = g["plans"][plan]
        assert r.c_probe == ref["c_probe"], plan
        assert r.c_cmp == ref["c_cmp"], plan
        assert r.c_top == ref["c_top"], plan
        assert r.c_unnest == ref.get("c_unnest", 0), plan
        assert {k: r.stats[k] for k in STAT_KEYS} == {k: ref["stats"][k] for k in STAT_KEYS}, plan
        assert r.out == ref["out"], plan


@pytest.mark.parametrize("name,g", EXP4, ids=[n for n, _ in EXP4])
def test_exp4_generator_and_plans(name, g):
    log2R, a, A, b, B = g["generator_args"][1:6]
    Sa, Ta = O.gen_exp4(log2R, a, A, b, B)
    assert O.colsum(Sa) == g["colsum_Sa"] and O.colsum(Ta) == g["colsum_Ta"]
    if "Sa" in g:
        assert Sa.tolist() == g["Sa"] and Ta.tolist() == g["Ta"]
    n, cardR = len(Sa), 1 << log2R
    R = O.tuples2(np.arange(cardR, dtype=np.uint32), np.zeros(cardR, np.uint32))
    S = O.tuples2(np.arange(n, dtype=np.uint32), Sa)
    T = O.tuples2(np.arange(n, dtype=np.uint32), Ta)
    for plan, nested in (("Ndu", True), ("Chj", False)):
        r = O.exp4_plan(R, S, T, g["nb"], nested)
        ref = g["plans"][plan]
        for k in ("c_probe_RS", "c_probe_RS_cmp", "c_probe_RT", "c_probe_RT_cmp", "c_top"):
            assert r[k.lower()] == ref[k], (plan, k)
        if nested:
            assert r["c_unnest_1"] == ref["c_unnest_1"] and r["c_unnest_2"] == ref["c_unnest_2"]
        assert r["out"] == ref["out"], plan
    assert g["plans"]["Ndu"]["c_top"] == g["join_card2"]  # calcJoinCard2 (main_experiment4.cc:593-597)


def test_survey_known_answers():
    """the reference's own printed relations for -R 3 -S 4."""
    Rk, Sa, _ = O.gen_exp1(8, 16, False)
    assert Rk.tolist() == [2, 3, 0, 5, 4, 6, 7, 1]
    assert Sa.tolist() == [7, 4, 1, 5, 2, 1, 2, 7, 7, 7, 7, 0, 4, 7, 1, 7]
    _, Sz, _ = O.gen_exp1(8, 16, True, 1.0)
    assert Sz.tolist() == [1, 0, 7, 0, 4, 7, 3, 0, 0, 0, 7, 7, 7, 0, 2, 0]
    Sa4, Ta4 = O.gen_exp4(3, 2, 2, 2, 1)
    assert Sa4.tolist() == [0, 0, 1, 1, 2, 3]
    assert Ta4.tolist() == [0, 0, 1, 1, 5, 4]


def test_empty_and_tiny_relations():
    """Edge cases the reference cannot run (its vec_permute underflows on an empty FK vector):
    the oracle treats empty inputs as empty joins."""
    R = O.tuples3(np.array([3, 1, 2], np.uint32), np.zeros(3, np.uint32))
    S = O.tuples3(np.zeros(0, np.uint32), np.zeros(0, np.uint32))
    r = O.chain_plan(R, 0, S, 1, 3, True)
    assert (r.c_probe, r.c_cmp, r.c_top) == (0, 0, 0)
    r = O.nested_plan(S, 1, R, 0, 1, True)
    assert (r.c_probe, r.c_cmp, r.c_top, r.stats["empty"]) == (0, 0, 0, 1)


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "ref_golden.out")),
                    reason="reference harness not built")
def test_reference_cpu_baseline_timer_counts():
    """bench.py's cpu_baseline (kind "reference") runs the reference Csr plan through
    oracle/_ref/ref_golden.out time_csr; its counters must be those of the oracle's Csr plan on
    the same generator sequence (uniform key/FK: every probe matches once)."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "ref_golden.out")
    out = subprocess.run([exe, "time_csr", "4096", "20000", "2"], capture_output=True, text=True, check=True)
    r = json.loads(out.stdout)
    Rk, Sa, _ = O.gen_exp1(4096, 20000, False, 0.0, 0)
    exp = O.chain_plan(O.tuples3(Rk, np.zeros_like(Rk)), 0, O.tuples3(np.arange(20000, dtype=np.uint32), Sa), 1,
                       4096, True)
    assert (r["c_probe"], r["c_cmp"], r["c_top"]) == (exp.c_probe, exp.c_cmp, exp.c_top)
    assert r["reps"] >= 2 and r["probe_ns"] > 0  # repeat_mintime: >= min reps, doubled below 300 ms
    # a probe prefix of the same relation: the counters of the first 5000 S tuples
    r = json.loads(subprocess.run([exe, "time_csr", "4096", "20000", "8", "5000"], capture_output=True, text=True,
                                  check=True).stdout)
    exp = O.chain_plan(O.tuples3(Rk, np.zeros_like(Rk)), 0, O.tuples3(np.arange(5000, dtype=np.uint32), Sa[:5000]), 1,
                       4096, True)
    assert (r["probe_prefix"], r["c_probe"], r["c_cmp"]) == (5000, exp.c_probe, exp.c_cmp) and r["reps"] >= 8


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "ref_golden.out")),
                    reason="reference harness not built")
def test_reference_cpu_baseline_nrs_timer_counts():
    """bench.py --workload C's cpu_baseline runs the reference Nrs plan (ref_golden.out time_nrs);
    its counters must be those of the oracle's Nrs plan on the same Zipf generator sequence."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "ref_golden.out")
    out = subprocess.run([exe, "time_nrs", "4096", "20000", "0.8", "2"], capture_output=True, text=True, check=True)
    r = json.loads(out.stdout)
    Rk, Sa, _ = O.gen_exp1(4096, 20000, True, 0.8, 0)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(20000, dtype=np.uint32), Sa)
    dv = O.num_distinct(Sa)
    exp = O.nested_plan(S, 1, R, 0, dv, True)
    assert r["nb"] == dv
    assert (r["c_probe"], r["c_cmp"], r["c_unnest"], r["c_top"]) == (exp.c_probe, exp.c_cmp, exp.c_unnest, exp.c_top)
    assert r["reps"] >= 2 and r["probe_ns"] > 0  # repeat_mintime: >= min reps, doubled below 300 ms


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "ref_golden.out")),
                    reason="reference harness not built")
def test_reference_cpu_baseline_ndu_timer_counts():
    """bench.py --workload E's cpu_baseline runs the reference Ndu plan (ref_golden.out time_ndu);
    its counters must be those of the oracle's Ndu plan on the same generator sequence."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "ref_golden.out")
    out = subprocess.run([exe, "time_ndu", "12", "3", "4", "2", "2", "2"], capture_output=True, text=True, check=True)
    r = json.loads(out.stdout)
    Sa, Ta = O.gen_exp4(12, 3, 4, 2, 2)
    cardR, n = 1 << 12, len(Sa)
    nb = (cardR >> 3) + (cardR >> 2)  # numFkCommon + numFkExclusive (main_experiment4.cc:855)
    R = O.tuples2(np.arange(cardR, dtype=np.uint32), np.zeros(cardR, np.uint32))
    S = O.tuples2(np.arange(n, dtype=np.uint32), Sa)
    T = O.tuples2(np.arange(n, dtype=np.uint32), Ta)
    exp = O.exp4_plan(R, S, T, nb, True)
    assert r["nb"] == nb
    assert (r["c_probe_rs"], r["c_probe_rt"], r["c_unnest_1"], r["c_unnest_2"], r["c_top"]) == (
        exp["c_probe_rs"], exp["c_probe_rt"], exp["c_unnest_1"], exp["c_unnest_2"], exp["c_top"])
