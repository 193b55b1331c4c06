"""Full-size (BASELINE config B: |R| = 1e7, |S| = 1e8) parity through size-independent
properties, on relations generated on the device (hj3d_gen_keys / hj3d_gen_fk).

For a key/FK join every S tuple has exactly one partner, the R row whose key equals S.a.
hj3d_expected_fk_join computes that pair set WITHOUT a hash table (inverse permutation of
R.k), so the join's cardinality and its order-independent pair checksums are checked
bit-exactly at full size. Comparison counts are checked against the oracle at 1e6 / 1e7
on the same generator."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

SEED_R, SEED_S = 0x5eed0001, 0x5eed0002


def make_rel(ctx, nR, nS, fk_max=None):
    import torch
    R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
    S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
    ctx.gen_keys(R, 0, 0, nR, SEED_R)          # R.k = permutation of [0, |R|)
    ctx.gen_keys(S, 0, 0, 0, 0)                # S.k = row id
    ctx.gen_fk(S, 1, 0, fk_max or nR, SEED_S)  # S.a ~ U[0, |R|)
    return R, S


def test_config_b_csr_full_size(ctx):
    import torch
    import hj3d
    nR, nS = 10_000_000, 100_000_000
    R, S = make_rel(ctx, nR, nS)
    exp = ctx.expected_fk_join(hj3d.Rel(R, 0), hj3d.Rel(S, 1), nR)
    assert exp["n"] == nS
    out = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    got = hj3d.exp1_plan(ctx, "Csr", R, S, nR, out=out)
    assert got["c_top"] == nS and got["c_probe"] == nS
    assert {k: got["out"][k] for k in ("n", "sum_a", "sum_b", "sum_h", "xor_h")} == exp
    assert got["stats"]["entries"] == nR and got["stats"]["distinct"] == nR
    assert got["stats"]["cc0_sum"] == nR
    # the materialised pairs (one slot per S tuple, partition order): sampled slots hold
    # (s, partner of s) with S[s].a == R[partner].k
    idx = torch.randint(0, nS, (4096,), device="cuda")
    smp = out[idx].long()
    assert (smp[:, 1] >= 0).all()
    assert torch.equal(S[smp[:, 0], 1], R[smp[:, 1], 0])
    rows = out[:, 0].sort().values
    assert torch.equal(rows, torch.arange(nS, device="cuda", dtype=torch.int32))
    # aggregate-only probe gives identical counters
    agg = hj3d.exp1_plan(ctx, "Csr", R, S, nR, stats=False)
    assert agg["out"] == got["out"] and agg["c_cmp"] == got["c_cmp"]


def test_config_b_nested_full_size(ctx):
    """Nrs (3D table on the non-unique S.a, 1e8 inserts) and Nsr at full size."""
    import hj3d
    nR, nS = 10_000_000, 100_000_000
    R, S = make_rel(ctx, nR, nS)
    exp_sr = ctx.expected_fk_join(hj3d.Rel(R, 0), hj3d.Rel(S, 1), nR)
    exp_rs = ctx.expected_fk_join(hj3d.Rel(R, 0), hj3d.Rel(S, 1), nR, swap=True)
    got = hj3d.exp1_plan(ctx, "Nsr", R, S, nR, stats=False)
    assert got["c_top"] == nS
    assert {k: got["out"][k] for k in ("n", "sum_a", "sum_b", "sum_h", "xor_h")} == exp_sr
    # #dv(S.a) from the nested table itself (one main record per distinct key)
    t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nR)
    t.build(hj3d.Rel(S, 1))
    dv = t.stats()["distinct"]
    assert 0.99 * nR * (1 - np.exp(-10)) < dv <= nR
    got = hj3d.exp1_plan(ctx, "Nrs", R, S, dv)
    assert got["c_unnest"] == nS and got["c_probe"] == dv
    assert {k: got["out"][k] for k in ("n", "sum_a", "sum_b", "sum_h", "xor_h")} == exp_rs
    assert got["stats"]["entries"] == nS and got["stats"]["distinct"] == dv


@pytest.mark.parametrize("nR,nS", [(1_000_000, 10_000_000)])
def test_device_generator_cmps_vs_oracle(ctx, nR, nS):
    """Config A sizes (1e6 / 1e7) on the device generator: the C oracle (reference semantics)
    reproduces every counter of the GPU plans, comparison counts included."""
    import hj3d
    R, S = make_rel(ctx, nR, nS)
    Rh = R.cpu().numpy().view(np.uint32)
    Sh = S.cpu().numpy().view(np.uint32)
    dv = O.num_distinct(Sh[:, 1])
    for plan, fn in (("Csr", lambda: O.chain_plan(Rh, 0, Sh, 1, nR, True)),
                     ("Crs", lambda: O.chain_plan(Sh, 1, Rh, 0, dv, False)),
                     ("Nrs", lambda: O.nested_plan(Sh, 1, Rh, 0, dv, True))):
        e = fn()
        nb = nR if plan == "Csr" else dv
        got = hj3d.exp1_plan(ctx, plan, R, S, nb)
        assert (got["c_probe"], got["c_cmp"], got["c_top"]) == (e.c_probe, e.c_cmp, e.c_top), plan
        assert got["out"] == e.out, plan
        assert got["stats"]["cc0_max"] == e.stats["cc0_max"] and got["stats"]["empty"] == e.stats["empty"]


# ---- config C: nested table on a non-unique build side with Zipf(0.8) duplicates ----

def make_zipf(ctx, nR, nS, theta=0.8):
    import torch
    R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
    S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
    ctx.gen_keys(R, 0, 0, nR, SEED_R)
    ctx.gen_keys(S, 0, 0, 0, 0)
    ctx.gen_zipf(S, 1, 0, nR, theta, SEED_S)
    return R, S


def test_device_zipf_matches_pmf(ctx):
    """The device sampler's value frequencies follow P(v) ~ (v+1)^-theta (5-sigma bounds)."""
    import torch
    nR, nS, theta = 1_000_000, 10_000_000, 0.8
    _, S = make_zipf(ctx, nR, nS, theta)
    a = S[:, 1]
    assert int(a.min()) >= 0 and int(a.max()) < nR
    cnt = torch.bincount(a.long(), minlength=nR)[:16].cpu().numpy().astype(np.float64)
    w = np.arange(1, nR + 1, dtype=np.float64) ** -theta
    p = w[:16] / w.sum()
    sd = np.sqrt(nS * p * (1 - p))
    assert (np.abs(cnt - nS * p) < 5 * sd + 1).all(), (cnt, nS * p)


@pytest.mark.parametrize("theta", [0.8, 1.0])
def test_config_c_zipf_plans_vs_oracle(ctx, theta):
    """Config C plans (Nrs, NrsNU, Nsr, Crs) on device-generated Zipf FKs at 1e6 / 1e7: every
    counter equal to the oracle's on the same (downloaded) relations."""
    import hj3d
    nR, nS = 1_000_000, 10_000_000
    R, S = make_zipf(ctx, nR, nS, theta)
    Rh = R.cpu().numpy().view(np.uint32)
    Sh = S.cpu().numpy().view(np.uint32)
    dv = O.num_distinct(Sh[:, 1])
    cases = {
        "Nrs": (dv, lambda: O.nested_plan(Sh, 1, Rh, 0, dv, True)),
        "NrsNU": (dv, lambda: O.nested_plan(Sh, 1, Rh, 0, dv, False)),
        "Nsr": (nR, lambda: O.nested_plan(Rh, 0, Sh, 1, nR, True)),
        "Crs": (dv, lambda: O.chain_plan(Sh, 1, Rh, 0, dv, False)),
    }
    for plan, (nb, fn) in cases.items():
        e = fn()
        got = hj3d.exp1_plan(ctx, plan, R, S, nb)
        assert (got["c_probe"], got["c_cmp"], got["c_unnest"], got["c_top"]) == \
            (e.c_probe, e.c_cmp, e.c_unnest, e.c_top), plan
        assert got["out"] == e.out, plan
        for k in ("empty", "distinct", "cc0_max", "cc0_sum", "cc1_cnt"):
            assert got["stats"][k] == e.stats[k], (plan, k)


def test_config_c_full_size(ctx):
    """Config C at full size (|R| = 1e7, |S| = 1e8, Zipf 0.8): Nrs (3D table on S.a, probe R,
    unnest) and NrsNU produce exactly the key/FK pair set; the hot key's ~1% of S is one
    sub-list expanded by whole workgroups."""
    import hj3d
    nR, nS = 10_000_000, 100_000_000
    R, S = make_zipf(ctx, nR, nS, 0.8)
    exp_rs = ctx.expected_fk_join(hj3d.Rel(R, 0), hj3d.Rel(S, 1), nR, swap=True)
    exp_sr = ctx.expected_fk_join(hj3d.Rel(R, 0), hj3d.Rel(S, 1), nR)
    assert exp_rs["n"] == nS
    t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nR)
    t.build(hj3d.Rel(S, 1))
    st = t.stats()
    dv = st["distinct"]
    assert st["entries"] == nS and dv < nR
    got = hj3d.exp1_plan(ctx, "Nrs", R, S, dv)
    assert got["c_probe"] == dv and got["c_unnest"] == nS and got["c_top"] == nS
    assert {k: got["out"][k] for k in ("n", "sum_a", "sum_b", "sum_h", "xor_h")} == exp_rs
    nu = hj3d.exp1_plan(ctx, "NrsNU", R, S, dv, stats=False)
    assert nu["c_probe"] == dv and nu["c_top"] == dv and nu["c_cmp"] == got["c_cmp"]
    sr = hj3d.exp1_plan(ctx, "Nsr", R, S, nR, stats=False)
    assert {k: sr["out"][k] for k in ("n", "sum_a", "sum_b", "sum_h", "xor_h")} == exp_sr


def test_large_table_beyond_partition_fanout(ctx):
    """|R| = 4e7 buckets: more than 2048 LDS-sized slices, so the build takes the direct path and
    the probe widens its slices beyond LDS (the L2-slice kernel); results stay exact."""
    import torch
    import hj3d
    nR, nS = 40_000_000, 50_000_000
    R, S = make_rel(ctx, nR, nS)
    exp = ctx.expected_fk_join(hj3d.Rel(R, 0), hj3d.Rel(S, 1), nR)
    out = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    got = hj3d.exp1_plan(ctx, "Csr", R, S, nR, out=out)
    assert got["c_top"] == nS
    assert {k: got["out"][k] for k in ("n", "sum_a", "sum_b", "sum_h", "xor_h")} == exp
    assert got["stats"]["entries"] == nR and got["stats"]["distinct"] == nR
    # the direct probe path agrees, comparison counts included
    ctx.force_direct(True)
    try:
        d = hj3d.exp1_plan(ctx, "Csr", R, S, nR, stats=False)
    finally:
        ctx.force_direct(False)
    assert d["out"] == got["out"] and d["c_cmp"] == got["c_cmp"]


@pytest.mark.parametrize("path", ["radix", "direct"])
def test_probe_in_chunks_accumulates(ctx, path):
    """One probe strand issued as 4 chunk probes with HJ3D_PROBE_ACCUMULATE (the multi-GPU
    pipeline does this) gives the counters and output of the single probe."""
    import torch
    import hj3d
    nR, nS = 2_000_000, 10_000_000
    R, S = make_rel(ctx, nR, nS)
    t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nR)
    if path == "direct":
        ctx.force_direct(True)
    try:
        t.build(hj3d.Rel(R, 0))
        one = ctx.probe(t, hj3d.Rel(S, 1), unique=True)
        out = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
        b = [0, 1_000_000, 4_000_000, 4_500_000, nS]
        for c in range(4):
            lo, hi = b[c], b[c + 1]
            ctx.probe(t, hj3d.Rel(S[lo:hi], 1, row_base=lo), unique=True, out=out[lo:hi], fetch=False,
                      accumulate=c > 0)
        got = ctx.probe_result()
    finally:
        ctx.force_direct(False)
    assert not got.overflow
    assert (got.n_probe, got.n_matched, got.n_out, got.n_cmps) == (one.n_probe, one.n_matched, one.n_out, one.n_cmps)
    assert (got.sum_a, got.sum_b, got.sum_h, got.xor_h) == (one.sum_a, one.sum_b, one.sum_h, one.xor_h)
    rows = out[:, 0].sort().values
    assert torch.equal(rows, torch.arange(nS, device="cuda", dtype=torch.int32))


@pytest.mark.parametrize("build_side", ["S", "R"])
def test_nested_partitioned_probe_vs_direct(ctx, build_side):
    """The partitioned nested probe (LDS slices of directory + main records) against the direct
    nested probe, in all four modes (nested tuples: aggregate / dense output; unnested:
    aggregate / materialised), on Zipf(1.0) duplicates: counters, checksums and the
    materialised output multiset are identical. build_side S: 3D table on the non-unique S.a,
    probe R (Nrs); R: table on the unique R.k, probe S (Nsr)."""
    import torch
    import hj3d
    nR, nS = 2_000_000, 20_000_000
    R, S = make_zipf(ctx, nR, nS, 1.0)
    if build_side == "S":
        t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nR)
        t.build(hj3d.Rel(S, 1))
        nb = t.stats()["distinct"]
        t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
        t.build(hj3d.Rel(S, 1))
        probe = hj3d.Rel(R, 0)
        n_out = nS
    else:
        t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nR)
        t.build(hj3d.Rel(R, 0))
        probe = hj3d.Rel(S, 1)
        n_out = nS
    assert probe.c.n >= 1 << 20  # the partitioned path (HJ3D_OPT_RADIX_MIN default)

    def run(unnest, emit):
        out = torch.full((n_out if unnest else probe.c.n, 2), -1, dtype=torch.int32, device="cuda") if emit else None
        res = ctx.probe(t, probe, unnest=unnest, out=out)
        got = None
        if emit:
            o = out[: res.n_out] if unnest else out
            key = (o[:, 0].long() << 32) | (o[:, 1].long() & 0xFFFFFFFF)
            got = key.sort().values
        return res, got

    for unnest in (False, True):
        for emit in (False, True):
            a, oa = run(unnest, emit)
            ctx.force_direct(True)
            try:
                b, ob = run(unnest, emit)
            finally:
                ctx.force_direct(False)
            assert a == b, (unnest, emit)
            if emit:
                assert torch.equal(oa, ob), (unnest, emit)


def test_explicit_row_ids_partitioned(ctx):
    """Probe sides whose row ids are a column (row_word, as the multi-GPU exchange delivers
    them) rather than implicit: the partitioners' explicit-row forms give the counters and
    checksums of the implicit form. S.k holds the row id (S.k = i), so both forms name the
    same rows; chaining (Csr, unique) and nested (Nsr, unnested materialised) probes."""
    import torch
    import hj3d
    nR, nS = 2_000_000, 12_000_000
    R, S = make_rel(ctx, nR, nS)
    assert torch.equal(S[:1000, 0], torch.arange(1000, dtype=torch.int32, device="cuda"))
    t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nR)
    t.build(hj3d.Rel(R, 0))
    imp = ctx.probe(t, hj3d.Rel(S, 1), unique=True)
    exp_ = ctx.probe(t, hj3d.Rel(S, 1, row_word=0), unique=True)
    assert imp == exp_ and imp.n_out == nS
    tn = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nR)
    tn.build(hj3d.Rel(R, 0))
    out_a = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    out_b = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    a = ctx.probe(tn, hj3d.Rel(S, 1), unnest=True, out=out_a)
    b = ctx.probe(tn, hj3d.Rel(S, 1, row_word=0), unnest=True, out=out_b)
    assert a == b and a.n_out == nS
    ka = ((out_a[:, 0].long() << 32) | (out_a[:, 1].long() & 0xFFFFFFFF)).sort().values
    kb = ((out_b[:, 0].long() << 32) | (out_b[:, 1].long() & 0xFFFFFFFF)).sort().values
    assert torch.equal(ka, kb)
