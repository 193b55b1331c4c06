"""Selection pushdown (AlgSelection / AlgDynSelection, reference algebra.hh:278-358).

CPU: the oracle's selection restatement (oracle.select) and the oracle joins downstream of it
reproduce the reference's own main_algebra_example plans (tests/golden/algebra_example.json,
made by tests/golden/make_algebra_golden.py from the reference binary): operator counts and the
output tuples. GPU (-m gpu): hj3d_select against oracle.select bit-exactly (pairs in scan order)
on seeded relations and edge cases, and the example plans through hj3d_select + hj3d_build /
hj3d_probe against the reference's outputs.
"""
import json
import os

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
EX = json.load(open(os.path.join(HERE, "golden", "algebra_example.json")))["tests"]
PRED = [(1, "<", 40)]  # SelectionL / DynSelectionL: L.b < 40 (main_algebra_example.cc)
NB = 4


def rel_u32(rows):
    return np.array(rows, dtype=np.int64).astype(np.int32).view(np.uint32).reshape(len(rows), -1)


def expected_pairs(t, unnest_or_chain=True):
    """Reference output tuples (a, b, c, d) as (L row, R row) pairs."""
    L, R = [tuple(x) for x in t["L"]], [tuple(x) for x in t["R"]]
    return sorted((L.index(tuple(o[:2])), R.index(tuple(o[2:]))) for o in t["output"])


def pair_checksums(pairs):
    h = [O.mix64((a << 32) | b) for a, b in pairs]
    x = 0
    for v in h:
        x ^= v
    M = (1 << 64) - 1
    return {"n": len(pairs), "sum_a": sum(a for a, _ in pairs), "sum_b": sum(b for _, b in pairs),
            "sum_h": sum(h) & M, "xor_h": x}


def test_oracle_selection_matches_reference_example():
    for name, t in EX.items():
        sel = O.select(rel_u32(t["L"]), 0, PRED)
        assert len(sel) == t["counts"]["probe_Sel"], name
        assert t["counts"]["probe_Scan"] == len(t["L"]), name
    t0 = EX["algebra_test0"]
    sel = O.select(rel_u32(t0["L"]), 0, PRED)
    assert [t0["L"][r] for r in sel[:, 1]] == t0["output"]


@pytest.mark.parametrize("name", ["algebra_test1", "algebra_test2", "algebra_test3"])
def test_oracle_join_after_selection_matches_reference_example(name):
    t = EX[name]
    L, R = rel_u32(t["L"]), rel_u32(t["R"])
    sel = O.select(L, 0, PRED)
    c = t["counts"]
    if name == "algebra_test3":
        res = O.chain_plan(R, 0, sel, 0, NB, False, prow=1)
        assert (res.c_probe, res.c_top) == (c["probe_Probe"], c["probe_Top"])
        exp = pair_checksums(expected_pairs(t))
    else:
        res = O.nested_plan(R, 0, sel, 0, NB, name == "algebra_test2", prow=1)
        assert res.c_probe == c["probe_Probe"] and res.c_top == c["probe_Top"]
        exp = pair_checksums(expected_pairs(t))
    assert res.c_build == c["build_Build"]
    for k, v in exp.items():
        assert res.out[k] == v, (name, k)


def test_oracle_selection_ops():
    rng = np.random.default_rng(7)
    t = rng.integers(0, 2**32, size=(1000, 3), dtype=np.uint64).astype(np.uint32)
    v = t[:, 2].view(np.int32).astype(np.int64)
    assert len(O.select(t, 0, [(2, "<", 0)])) == int((v < 0).sum())
    assert len(O.select(t, 0, [(2, ">=", 5, None, False)])) == int((t[:, 2] >= 5).sum())
    got = O.select(t, 1, [(2, "range", -10**9, 10**9), (0, "!=", int(t[0, 0]), None, False)])
    exp_rows = np.nonzero((v >= -10**9) & (v < 10**9) & (t[:, 0] != t[0, 0]))[0]
    assert (got[:, 1] == exp_rows).all() and (got[:, 0] == t[exp_rows, 1]).all()
    assert O.select(t[:0], 0, PRED).shape == (0, 2)


# ---------------------------------------------------------------- GPU
def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


CASES = [
    ("lt_signed", 100_003, [(2, "<", 0)]),
    ("range_two_preds", 1_000_000, [(1, "range", -5 * 10**8, 10**9), (2, "!=", 3, None, False)]),
    ("eq_rare", 65_536, [(2, "==", 12345, None, False)]),
    ("none_pass", 4_097, [(1, ">", 2**31 - 1)]),
    ("all_pass", 4_095, [(1, ">=", -2**31)]),
    ("no_predicate", 10_000, []),
    ("single", 1, [(0, "<=", 2**32, None, False)]),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,preds", CASES, ids=[c[0] for c in CASES])
def test_gpu_select_bit_exact(ctx, name, n, preds):
    import hj3d
    rng = np.random.default_rng(abs(hash(name)) % 2**32)
    t = rng.integers(0, 2**32, size=(n, 3), dtype=np.uint64).astype(np.uint32)
    if name == "eq_rare":
        t[::97, 2] = 12345
    exp = O.select(t, 0, preds)
    pairs, rel, cnt = ctx.select(hj3d.Rel(dev(t), 0), preds)
    assert cnt == len(exp) and rel.n == cnt
    got = pairs[:cnt].cpu().numpy().view(np.uint32)
    assert (got == exp).all()


@pytest.mark.gpu
def test_gpu_select_empty_relation(ctx):
    import hj3d
    import torch
    t = torch.zeros((0, 3), dtype=torch.int32, device="cuda")
    _, rel, cnt = ctx.select(hj3d.Rel(t, 0), PRED)
    assert cnt == 0 and rel.n == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["algebra_test1", "algebra_test2", "algebra_test3"])
def test_gpu_selection_join_matches_reference_example(ctx, name):
    """scan(L) -> selection(L.b < 40) -> probe(R.c = L.a) [-> unnest] -> top, on the device."""
    import hj3d
    t = EX[name]
    L, R = rel_u32(t["L"]), rel_u32(t["R"])
    _, sel, cnt = ctx.select(hj3d.Rel(dev(L), 0), PRED)
    assert cnt == t["counts"]["probe_Sel"]
    kind = hj3d.HJ3D_CHAIN if name == "algebra_test3" else hj3d.HJ3D_NESTED
    tab = hj3d.Table(ctx, kind, NB)
    tab.build(hj3d.Rel(dev(R), 0))
    res = ctx.probe(tab, sel, unnest=name == "algebra_test2")
    c = t["counts"]
    if name == "algebra_test3":
        assert res.n_out == c["probe_Top"] == c["probe_Probe"]
    else:
        assert res.n_matched == c["probe_Probe"] and res.n_out == c["probe_Top"]
    exp = pair_checksums(expected_pairs(t))
    got = {"n": res.n_out, "sum_a": res.sum_a, "sum_b": res.sum_b, "sum_h": res.sum_h, "xor_h": res.xor_h}
    assert got == exp
    tab.close()


@pytest.mark.gpu
def test_gpu_selection_then_join_seeded(ctx):
    """Selected probe side of a uniform key/FK join vs the oracle's probe of the same selection
    (row ids of the selected tuples are their scan positions, as the reference's pointers are)."""
    import hj3d
    Rk, Sa, _ = O.gen_exp1(1 << 14, 1 << 18, False, 1.0, 0)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(1 << 18, dtype=np.uint32), Sa)
    S[:, 2] = np.random.default_rng(3).integers(0, 100, size=len(S)).astype(np.uint32)
    preds = [(2, "<", 37)]
    sel_h = O.select(S, 1, preds)
    exp = O.chain_plan(R, 0, sel_h, 0, len(R), True, prow=1)
    _, sel, cnt = ctx.select(hj3d.Rel(dev(S), 1), preds)
    assert cnt == len(sel_h)
    tab = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, len(R))
    tab.build(hj3d.Rel(dev(R), 0))
    res = ctx.probe(tab, sel, unique=True)
    assert (res.n_out, res.n_cmps) == (exp.c_top, exp.c_cmp)
    for k in ("sum_a", "sum_b", "sum_h", "xor_h"):
        assert getattr(res, k) == exp.out[k], k
    tab.close()


BIN = os.path.join(os.path.dirname(HERE), "3d-hashjoin_amd", "bin", "dropin_selection")


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BIN), reason="drop-in selection program not built (make -C 3d-hashjoin_amd)")
def test_gpu_dropin_selection_pushdown_matches_reference_example():
    """tests/cpp/dropin_selection.cc: the example's plans through the drop-in operators, selection
    on the host and pushed down to hj3d_select; every operator count equals the reference's and
    the printed chaining output equals the reference's output, in the reference's order."""
    import re
    import subprocess
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    got = {}
    for ln in lines:
        m = re.match(r"(\w+) (\w+) (.*)", ln)
        if m and "=" in m.group(3):
            got[(m.group(1), m.group(2))] = dict(kv.split("=") for kv in m.group(3).split())
    exp = {"chain": EX["algebra_test3"]["counts"], "nested": EX["algebra_test1"]["counts"],
           "unnest": EX["algebra_test2"]["counts"]}
    modes = {"chain": ("host", "device", "device_dyn", "device_print"), "nested": ("host", "device"),
             "unnest": ("host", "device")}
    for plan, ms in modes.items():
        for mode in ms:
            g, c = got[(plan, mode)], exp[plan]
            assert int(g["Top"]) == c["probe_Top"], (plan, mode)
            assert int(g["Probe"]) == c["probe_Probe"], (plan, mode)
            assert int(g["Sel"]) == c["probe_Sel"], (plan, mode)
            assert int(g["Scan"]) == c["probe_Scan"], (plan, mode)
            assert int(g["Build"]) == c["build_Build"], (plan, mode)
    printed = [[int(v) for v in ln.strip("()").split(",")] for ln in lines if ln.startswith("(")]
    assert printed == EX["algebra_test3"]["output"]


FUSED_CASES = [
    ("lt_signed", [(2, "<", 37)]),
    ("le_unsigned", [(2, "<=", 0, None, False)]),
    ("gt", [(2, ">", 90)]),
    ("ge", [(2, ">=", 50)]),
    ("eq", [(2, "==", 7)]),
    ("ne", [(2, "!=", 7)]),
    ("range", [(2, "range", 20, 30)]),
    ("empty_range", [(2, "range", 30, 30)]),
    ("on_key_word", [(1, "<", 1000)]),
    ("two_preds_unfused", [(2, ">=", 10), (2, "<", 60)]),
]


@pytest.mark.gpu
@pytest.mark.parametrize("unique", [True, False], ids=["unique", "nonunique"])
@pytest.mark.parametrize("name,preds", FUSED_CASES, ids=[c[0] for c in FUSED_CASES])
def test_gpu_probe_sel_bit_exact(ctx, name, preds, unique):
    """hj3d_probe_sel (selection fused into the probe partitioner for one predicate, select-first
    otherwise) vs the oracle's probe of oracle.select's output: counters and output checksums."""
    import hj3d
    import torch
    nR, nS = 1 << 14, 1 << 18
    Rk, Sa, _ = O.gen_exp1(nR, nS, False, 1.0, 0)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    S[:, 2] = np.random.default_rng(5).integers(-5, 100, size=nS).astype(np.int32).view(np.uint32)
    sel_h = O.select(S, 1, preds)
    exp = O.chain_plan(R, 0, sel_h, 0, nR, unique, prow=1)
    ctx.radix_min(1 << 12)  # the partitioned (fusing) path at this size
    tab = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nR)
    tab.build(hj3d.Rel(dev(R), 0))
    out = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    for unfused in (False, True):
        ctx.sel_unfused(unfused)
        res = ctx.probe_sel(tab, hj3d.Rel(dev(S), 1), preds, unique=unique, out=out)
        assert res.n_probe == len(sel_h), unfused
        assert (res.n_out, res.n_cmps) == (exp.c_top, exp.c_cmp), unfused
        for k in ("sum_a", "sum_b", "sum_h", "xor_h"):
            assert getattr(res, k) == exp.out[k], (unfused, k)
        pairs = out[: res.n_probe if unique else res.n_out].cpu().numpy().view(np.uint32)
        if unique:
            pairs = pairs[pairs[:, 1] != 0xFFFFFFFF]
        got = pairs[:, [0, 1]]
        assert len(got) == exp.c_top
        assert sorted(map(tuple, got.tolist())) == sorted(
            (int(a), int(b)) for a, b in zip(sel_h[:, 1], np.argsort(Rk)[sel_h[:, 0]]))
    ctx.sel_unfused(False)
    ctx.radix_min(1 << 20)
    tab.close()


@pytest.mark.gpu
@pytest.mark.parametrize("unnest", [True, False], ids=["unnest", "nested_tuples"])
def test_gpu_probe_sel_nested(ctx, unnest):
    """A selected probe into a nested table (Nrs shape: 3D table on Zipf S.a, probe R), fused into
    the nested probe's partitioner and select-first, vs the oracle's plan on oracle.select's output."""
    import hj3d
    import torch
    nR, nS = 1 << 14, 1 << 17
    Rk, Sa, _ = O.gen_exp1(nR, nS, True, 0.8, 0)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    R[:, 2] = np.arange(nR, dtype=np.uint32) % 10
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    dv = O.num_distinct(Sa)
    preds = [(2, "<", 3)]
    sel_h = O.select(R, 0, preds)
    exp = O.nested_plan(S, 1, sel_h, 0, dv, unnest, prow=1)
    ctx.radix_min(1 << 10)  # the partitioned (fusing) nested probe at this size
    tab = hj3d.Table(ctx, hj3d.HJ3D_NESTED, dv)
    tab.build(hj3d.Rel(dev(S), 1))
    out = torch.empty((nS + nR, 2), dtype=torch.int32, device="cuda")
    for unfused in (False, True):
        ctx.sel_unfused(unfused)
        for o in (None, out):
            res = ctx.probe_sel(tab, hj3d.Rel(dev(R), 0), preds, unnest=unnest, out=o)
            assert res.n_probe == len(sel_h), (unfused, o is None)
            assert (res.n_matched, res.n_out, res.n_cmps) == (exp.c_probe, exp.c_top, exp.c_cmp), (unfused, o is None)
            for k in ("sum_a", "sum_b", "sum_h", "xor_h"):
                assert getattr(res, k) == exp.out[k], (unfused, o is None, k)
    ctx.sel_unfused(False)
    ctx.radix_min(1 << 20)
    tab.close()


def _fmix32(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [2, 8])
def test_gpu_partition_with_selection(ctx, parts):
    """hj3d_partition_sel (selection below the multi-GPU exchange): per destination, the passing
    tuples' (key, row) pairs in scan order, destination = owner of murmur32(key) % NB (§8e)."""
    import hj3d
    import torch
    n, nb = 300_001, 100_003
    rng = np.random.default_rng(11)
    t = np.stack([rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
                  rng.integers(0, nb, n).astype(np.uint32),
                  rng.integers(0, 100, n).astype(np.uint32)], axis=1)
    preds = [(2, ">=", 25), (2, "<", 75)]
    sel = O.select(t, 1, preds)
    owner = ((_fmix32(sel[:, 0]) % np.uint64(nb)) * np.uint64(parts) // np.uint64(nb)).astype(np.int64)
    out = torch.empty((n, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(parts, dtype=torch.int64, device="cuda")
    ctx.partition(hj3d.Rel(dev(t), 1), nb, parts, out, cnt, preds=preds)
    got_cnt = cnt.cpu().tolist()
    assert got_cnt == [int((owner == d).sum()) for d in range(parts)]
    got = out[: sum(got_cnt)].cpu().numpy().view(np.uint32)
    off = 0
    for d in range(parts):
        exp = sel[owner == d]
        assert (got[off: off + len(exp)] == exp).all(), d
        off += len(exp)
