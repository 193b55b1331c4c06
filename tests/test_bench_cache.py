"""bench.py's per-node cache of the reference's relations for N > 1 ranks (CPU): the mapped columns
equal the generator's output, a second call reuses the files, and a rank that is not the maker
finds them after the barrier."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_columns_cached(tmp_path, monkeypatch):
    monkeypatch.setenv("HJ3D_REL_CACHE", str(tmp_path))
    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    import hj3d
    nR, nS = 1000, 20000
    Rk, Sa = hj3d.gen_exp1_ref(nR, nS)
    calls = []
    r1, s1 = bench.reference_columns_cached(nR, nS, True, lambda: calls.append(1))
    assert (np.asarray(r1) == Rk).all() and (np.asarray(s1) == Sa).all() and calls == [1]
    files = sorted(os.listdir(tmp_path))
    mtimes = [os.path.getmtime(tmp_path / f) for f in files]
    r2, s2 = bench.reference_columns_cached(nR, nS, False, lambda: None)  # a non-maker rank
    assert (np.asarray(r2[10:20]) == Rk[10:20]).all() and (np.asarray(s2[-5:]) == Sa[-5:]).all()
    bench.reference_columns_cached(nR, nS, True, lambda: None)  # valid cache: not regenerated
    assert [os.path.getmtime(tmp_path / f) for f in files] == mtimes
