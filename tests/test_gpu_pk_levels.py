"""GPU parity of the packed unique probe's geometries (chain_pk.hip): the two-level partition
(k_pk_part into coarse ranges of C slices, then k_pk_split by slice) that tables of more than 1024
LDS slices take (config D: 1e8 buckets on one GPU, 1.25e7-5e7 per rank at 8/4/2 GPUs), the
partitioner's mid-stream carry flush together with region overflows, and bucket-range shards
(bucket_lo != 0, explicit row ids) on every geometry.

Small tables are put on the two-level path with HJ3D_OPT_PK_SLICE (slice width bound); the
counters, statistics and output checksums must equal the reference binary's fixtures exactly
(integer work: bit-exact bar), and the materialised pairs are checked pair by pair.
"""
import numpy as np
import pytest

import oracle as O
from conftest import load_golden

pytestmark = pytest.mark.gpu

EXP1 = dict(load_golden("exp1_*.json", headline=False))


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


def rel_of(name):
    g = EXP1[name]
    _, nR, nS, skew, theta, t, b = g["generator_args"][:7]
    Rk, Sa, _ = O.gen_exp1(nR, nS, bool(skew), theta, t)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    return g, R, S, b


def host_checksums(pairs):
    a = pairs[:, 0].astype(np.uint64)
    b = pairs[:, 1].astype(np.uint64)
    z = (a << np.uint64(32)) | b
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    z = z ^ (z >> np.uint64(31))
    with np.errstate(over="ignore"):
        return {"n": len(pairs), "sum_a": int(a.sum(dtype=np.uint64)), "sum_b": int(b.sum(dtype=np.uint64)),
                "sum_c": 0, "sum_h": int(z.sum(dtype=np.uint64)), "xor_h": int(np.bitwise_xor.reduce(z)) if len(z) else 0}


@pytest.fixture
def pk(ctx):
    """Packed probe on every probe size; options restored afterwards."""
    ctx.radix_min(0)
    yield ctx
    ctx.pk_slice_max(0)
    ctx.pk_stage(0)
    ctx.pk_build(False)
    ctx.radix_min(1 << 20)


def check_csr(ctx, name, emit=True):
    import torch
    import hj3d
    g, R, S, b = rel_of(name)
    nb = hj3d.num_buckets_exp1("Csr", len(R), g["numDvSa"], b)
    ref = g["plans"]["Csr"]
    out = torch.full((len(S), 2), -1, dtype=torch.int32, device="cuda") if emit else None
    got = hj3d.exp1_plan(ctx, "Csr", dev(R), dev(S), nb, out=out)
    assert (got["c_probe"], got["c_cmp"], got["c_top"]) == (ref["c_probe"], ref["c_cmp"], ref["c_top"]), name
    assert got["out"] == ref["out"], name
    if emit:
        host = out.cpu().numpy().view(np.uint32)
        assert host_checksums(host[host[:, 1] != 0xFFFFFFFF]) == ref["out"], name
        # every probe row once, each paired with the R row whose key it references
        rows = np.sort(host[:, 0])
        assert np.array_equal(rows, np.arange(len(S), dtype=np.uint32)), name
        assert np.array_equal(S[host[:, 0], 1], R[host[:, 1], 0]), name


# slice bounds at 2^20 buckets (P rounded up to whole waves of 256 workgroups): 1024 slices (one level,
# one slice per partitioning thread), 2048 (one level, two per thread, 64-B segments), and two levels
# with C = 4, 16 and 32 slices per coarse range
@pytest.mark.parametrize("w", [1024, 512, 256, 64, 32])
def test_two_level_uniform_equals_reference(pk, w):
    pk.pk_slice_max(w)
    check_csr(pk, "exp1_R1048576_S8388608_uni")


@pytest.mark.parametrize("w", [128, 100, 16])
def test_two_level_zipf_region_overflow_equals_reference(pk, w):
    """Zipf(1) probe keys: a hot slice overflows its regions at both levels (k_pk_part's and
    k_pk_split's; w = 100: one level of 1536 slices, two per partitioning thread), the overflow list
    is probed against the table in HBM."""
    pk.pk_slice_max(w)
    check_csr(pk, "exp1_R131072_S1048576_zipf1")


@pytest.mark.parametrize("two_level", [False, "two_per_thread", True])
def test_carry_flush_with_region_overflow(pk, two_level):
    """after a mid-stream carry flush the partitioner's region cursor is not segment
    aligned, so a whole segment can straddle the region's end; it must go to the overflow list
    whole and the region's count stop at its start. Forced here: flush after every tile
    (HJ3D_OPT_PK_STAGE = 1), ~1024 slices, Zipf(1) keys that overflow the hot slice's regions."""
    pk.pk_stage(1)
    pk.pk_slice_max(100 if two_level == "two_per_thread" else 16 if two_level else 128)
    check_csr(pk, "exp1_R131072_S1048576_zipf1")
    check_csr(pk, "exp1_R1048576_S8388608_uni")


@pytest.mark.parametrize("w", [0, 64])
def test_bucket_range_shards_on_packed_paths(pk, w):
    """Owner ranges of the multi-GPU split emulated on one device (hj3d.exp1_plan_sharded): tables
    over [lo, hi) with lo != 0, probed with explicit-row pairs through the packed probe (single or
    two-level), add up to the reference's counters, statistics and output checksums."""
    import torch
    import hj3d
    pk.pk_slice_max(w)
    for name in ("exp1_R1048576_S8388608_uni", "exp1_R131072_S1048576_zipf1"):
        g, R, S, b = rel_of(name)
        nb = hj3d.num_buckets_exp1("Csr", len(R), g["numDvSa"], b)
        ref = g["plans"]["Csr"]
        out = torch.full((len(S), 2), -1, dtype=torch.int32, device="cuda")
        for parts in (3, 8):
            got = hj3d.exp1_plan_sharded(pk, "Csr", dev(R), dev(S), nb, parts, out=out)
            assert (got["c_probe"], got["c_cmp"], got["c_top"]) == (ref["c_probe"], ref["c_cmp"], ref["c_top"]), (name, parts)
            assert got["out"] == ref["out"], (name, parts)
            assert {k: got["stats"][k] for k in ref["stats"] if k in got["stats"]} == \
                {k: ref["stats"][k] for k in ref["stats"] if k in got["stats"]}, (name, parts)
            host = out.cpu().numpy().view(np.uint32)
            assert host_checksums(host) == ref["out"], (name, parts)


def test_pk_plan_geometry(ctx):
    """The slice plan the bench's configs land on (host-side arithmetic, checked on the device's CU
    count): config B and every config-D rank size fit one LDS slice per probe workgroup with whole
    waves of workgroups; up to 2048 slices one level (two slices per partitioning thread above 1024:
    config D's rank at 4 GPUs), above that two levels with C slices per coarse range."""
    import hj3d
    for nbl, n_build, levels in ((10_000_000, 10_000_000, 1), (12_500_000, 12_500_000, 1),
                                 (25_000_000, 25_000_000, 1), (50_000_000, 50_000_000, 2),
                                 (100_000_000, 100_000_000, 2)):
        pl = ctx.pk_plan(nbl, n_build)
        assert pl["P"] * pl["W"] >= nbl and (pl["P"] - 1) * pl["W"] < nbl
        assert (pl["C"] > 1) == (levels == 2), (nbl, pl)
        assert pl["P1"] <= (2048 if levels == 1 else 1024) and pl["P1"] * pl["W1"] >= nbl
        # the slice image at fill n_build / nbl: W directory words + 2 words per entry (+ 6 sigma)
        fill = n_build / nbl
        assert pl["W"] * (1 + 2 * fill) + 12 * (pl["W"] * fill) ** 0.5 <= 39552, (nbl, pl)


STAT_KEYS = ("nb", "empty", "entries", "distinct", "cc0_min", "cc0_max", "cc0_sum", "cc0_cnt",
             "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")


@pytest.mark.parametrize("name", ["exp1_R1048576_S8388608_uni", "exp1_R131072_S1048576_zipf1",
                                  "exp1_R65537_S1000000_zipf08"])
def test_slice_build_equals_reference(pk, name):
    """The two-level slice build (pk_build, the chaining build of tables beyond 2048 x 16384
    buckets, i.e. config D's 1e8) forced on fixture tables: statistics and the counters and output
    checksums of Csr / CsrUU / Crs equal the reference binary's. Crs builds on the skewed S.a: hot
    keys overflow the partition regions there and the direct build takes over."""
    import hj3d
    pk.pk_build(True)
    try:
        g, R, S, b = rel_of(name)
        dR, dS = dev(R), dev(S)
        for plan in ("Csr", "CsrUU", "Crs"):
            nb = hj3d.num_buckets_exp1(plan, len(R), g["numDvSa"], b)
            got = hj3d.exp1_plan(pk, plan, dR, dS, nb)
            ref = g["plans"][plan]
            for k in ("c_build", "c_probe", "c_cmp", "c_top"):
                assert got[k] == ref[k], (name, plan, k, got[k], ref[k])
            assert {k: got["stats"][k] for k in STAT_KEYS} == {k: ref["stats"][k] for k in STAT_KEYS}, (name, plan)
            assert got["out"] == ref["out"], (name, plan)
    finally:
        pk.pk_build(False)


@pytest.mark.parametrize("fill", [1.0, 1.3])
def test_slice_build_large_slices_vs_oracle(pk, fill):
    """Slices whose fine regions exceed the register-held form (more than 704 pairs, frequent at
    fill 1.3 with 8192-bucket slices) take the in-kernel HBM path of k_pk_build; random non-unique
    keys; statistics and both probe forms equal the oracle's."""
    import hj3d
    rng = np.random.default_rng(int(fill * 10))
    nb = 1 << 20
    n = int(nb * fill)
    Bk = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    Bk[rng.random(n) < 0.05] = 12345  # one key with ~5 % of the rows (a long bucket, arrival order)
    Pk = np.concatenate([Bk[rng.integers(0, n, 600_000)], rng.integers(0, 1 << 32, 200_000, dtype=np.uint64).astype(np.uint32)])
    B = O.tuples3(Bk, np.zeros(n, np.uint32))
    Pt = O.tuples3(np.arange(len(Pk), dtype=np.uint32), Pk)
    pk.pk_build(True)
    try:
        t = hj3d.Table(pk, hj3d.HJ3D_CHAIN, nb)
        t.build(hj3d.Rel(dev(B), 0))
        st = t.stats()
        for unique in (True, False):
            e = O.chain_plan(B, 0, Pt, 1, nb, unique)
            r = pk.probe(t, hj3d.Rel(dev(Pt), 1), unique=unique)
            assert (r.n_out, r.n_cmps) == (e.c_probe, e.c_cmp), unique
            assert {"n": r.n_out, "sum_a": r.sum_a, "sum_b": r.sum_b, "sum_c": 0, "sum_h": r.sum_h,
                    "xor_h": r.xor_h} == e.out, unique
        assert {k: st[k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}
    finally:
        pk.pk_build(False)
