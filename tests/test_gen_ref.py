"""The engine's reference input generator (hj3d_gen_exp1_ref / hj3d_gen_exp4_ref, csrc/gen_ref.cpp)
against the fixtures the REAL reference wrote (tests/golden/*.json), at every fixture size up to
the headline configs B / C (1e7 / 1e8, uniform and Zipf 0.8) and E (log2R = 22). Host code only:
runs on CPU (libhj3d.so loads without a GPU; the generator touches none)."""
import numpy as np
import pytest

import oracle as O
from conftest import load_golden

# config D (|S| = 1e9) is left to the GPU box (tests/test_gpu_headline.py): 4.4 GB and ~25 s here
EXP1 = [x for x in load_golden("exp1_*.json") if x[1]["nS"] <= 100_000_000]
EXP4 = load_golden("exp4_*.json")


@pytest.mark.parametrize("name,g", EXP1, ids=[n for n, _ in EXP1])
def test_exp1_ref_generator_matches_reference(name, g):
    import hj3d
    _, nR, nS, skew, theta, t = g["generator_args"][:6]
    Rk, Sa = hj3d.gen_exp1_ref(nR, nS, bool(skew), theta, t)
    assert Rk[:16].tolist() == g["head_Rk"] and Sa[:16].tolist() == g["head_Sa"]
    assert O.colsum(Rk) == g["colsum_Rk"]
    assert O.colsum(Sa) == g["colsum_Sa"]
    if "Rk" in g:
        assert Rk.tolist() == g["Rk"] and Sa.tolist() == g["Sa"]
    if nS <= 10_000_000:
        assert len(np.unique(Sa)) == g["numDvSa"]


@pytest.mark.parametrize("name,g", EXP4, ids=[n for n, _ in EXP4])
def test_exp4_ref_generator_matches_reference(name, g):
    import hj3d
    log2R, a, A, b, B = g["generator_args"][1:6]
    Sa, Ta = hj3d.gen_exp4_ref(log2R, a, A, b, B)
    assert len(Sa) == g["cardS"]
    assert O.colsum(Sa) == g["colsum_Sa"] and O.colsum(Ta) == g["colsum_Ta"]
    if "Sa" in g:
        assert Sa.tolist() == g["Sa"] and Ta.tolist() == g["Ta"]


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_zipf_threads_do_not_change_the_stream(threads):
    """The Zipf attempts are evaluated in parallel blocks; the values, and the twister position the
    permutation continues from, must not depend on the worker count (block boundaries included:
    more than one 2^22-attempt block)."""
    import hj3d
    ref = hj3d.gen_exp1_ref(1 << 16, 5_000_000, True, 0.8, 0, threads=1)
    got = hj3d.gen_exp1_ref(1 << 16, 5_000_000, True, 0.8, 0, threads=threads)
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])
    Rk, Sa, _ = O.gen_exp1(1 << 16, 5_000_000, True, 0.8, 0)
    assert np.array_equal(Sa, got[1]) and np.array_equal(Rk, got[0])


def test_generator_edge_cases():
    import hj3d
    # one key: every FK is 0; t shifts fkMax (main_experiment1.cc:190)
    Rk, Sa = hj3d.gen_exp1_ref(1, 7)
    assert Rk.tolist() == [0] and Sa.tolist() == [0] * 7
    Rk, Sa = hj3d.gen_exp1_ref(4096, 0)
    assert sorted(Rk.tolist()) == list(range(4096)) and len(Sa) == 0
    for nR, nS, skew, t in ((1000, 333, False, 3), (65536, 70000, True, 2), (65537, 1000, False, 0)):
        Rk, Sa = hj3d.gen_exp1_ref(nR, nS, skew, 1.0, t)
        eRk, eSa, fk = O.gen_exp1(nR, nS, skew, 1.0, t)
        assert np.array_equal(Rk, eRk) and np.array_equal(Sa, eSa)
        assert int(Sa.max()) < fk
    with pytest.raises(hj3d.Hj3dError):
        hj3d.gen_exp1_ref(0, 10)
    with pytest.raises(hj3d.Hj3dError):
        hj3d.gen_exp1_ref(8, 10, t=4)  # fkMax = 0
