"""GPU parity: libhj3d.so on the MI355X against the reference's golden fixtures and the oracle.

Inputs are produced by the oracle's bit-exact generator restatement (itself pinned to the
reference by test_oracle_golden.py) and uploaded; every counter the reference reports
(c_htProbe, c_htProbeCmp, c_unnest, c_top), every HtStatistics field and the order-independent
output checksums must match EXACTLY (integer work: bit-exact bar).
"""
import numpy as np
import pytest

import oracle as O
from conftest import load_golden

pytestmark = pytest.mark.gpu

EXP1 = load_golden("exp1_*.json", headline=False)  # the headline sizes: test_gpu_headline.py
EXP4 = load_golden("exp4_*.json", headline=False)
STAT_KEYS = ("nb", "empty", "entries", "distinct", "cc0_min", "cc0_max", "cc0_sum", "cc0_cnt",
             "cc1_min", "cc1_max", "cc1_sum", "cc1_cnt")
PLANS = ("Csr", "CsrUU", "Crs", "Nsr", "Nrs", "NrsNU")


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


def exp1_rel(g):
    _, nR, nS, skew, theta, t, b = g["generator_args"][:7]
    Rk, Sa, _ = O.gen_exp1(nR, nS, bool(skew), theta, t)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    return R, S, b


def host_checksums(pairs: np.ndarray) -> dict:
    """Order-independent checksums of emitted (a, b) pairs, computed on the host."""
    a = pairs[:, 0].astype(np.uint64)
    b = pairs[:, 1].astype(np.uint64)
    z = (a << np.uint64(32)) | b
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    z = z ^ (z >> np.uint64(31))
    with np.errstate(over="ignore"):
        return {"n": len(pairs), "sum_a": int(a.sum(dtype=np.uint64)), "sum_b": int(b.sum(dtype=np.uint64)),
                "sum_c": 0, "sum_h": int(z.sum(dtype=np.uint64)), "xor_h": int(np.bitwise_xor.reduce(z)) if len(z) else 0}


@pytest.mark.parametrize("name,g", EXP1, ids=[n for n, _ in EXP1])
def test_exp1_plans_bit_exact(ctx, name, g):
    import hj3d
    R, S, b = exp1_rel(g)
    dR, dS = dev(R), dev(S)
    for plan in PLANS:
        nb = hj3d.num_buckets_exp1(plan, len(R), g["numDvSa"], b)
        ref = g["plans"][plan]
        got = hj3d.exp1_plan(ctx, plan, dR, dS, nb)
        assert got["nb"] == ref["nb"], plan
        for k in ("c_probe", "c_cmp", "c_top"):
            assert got[k] == ref[k], (plan, k, got[k], ref[k])
        assert got["c_unnest"] == ref.get("c_unnest", 0), plan
        assert {k: got["stats"][k] for k in STAT_KEYS} == {k: ref["stats"][k] for k in STAT_KEYS}, plan
        assert got["out"] == ref["out"], plan


@pytest.mark.parametrize("name,g", [x for x in EXP1 if x[1]["nS"] <= 1_100_000], ids=lambda v: v if isinstance(v, str) else "")
def test_exp1_materialised_output(ctx, name, g):
    """HJ3D_PROBE_EMIT: the pairs written to HBM are exactly the reference's output tuples."""
    import torch
    import hj3d
    R, S, b = exp1_rel(g)
    dR, dS = dev(R), dev(S)
    for plan in PLANS:
        nb = hj3d.num_buckets_exp1(plan, len(R), g["numDvSa"], b)
        ref = g["plans"][plan]
        cap = max(ref["out"]["n"], len(S), len(R), 1)
        out = torch.zeros((cap, 2), dtype=torch.int32, device="cuda")
        got = hj3d.exp1_plan(ctx, plan, dR, dS, nb, out=out, stats=False)
        assert not got["overflow"]
        host = out.cpu().numpy().view(np.uint32)
        kind, _, _, _, unique, unnest = hj3d.EXP1_PLANS[plan]
        dense = (kind == hj3d.HJ3D_CHAIN and unique) or (kind == hj3d.HJ3D_NESTED and not unnest)
        if dense:  # one slot per probe tuple, unmatched slots carry 0xFFFFFFFF
            nprobe = len(S) if hj3d.EXP1_PLANS[plan][1] == "R" else len(R)
            host = host[:nprobe]
            assert (np.sort(host[:, 0]) == np.arange(nprobe, dtype=np.uint32)).all()
            host = host[host[:, 1] != 0xFFFFFFFF]
        else:
            host = host[: ref["out"]["n"]]
        assert host_checksums(host) == ref["out"], plan
        assert got["out"]["n"] == ref["out"]["n"]


@pytest.mark.parametrize("name,g", [x for x in EXP1 if x[1]["nR"] >= 64], ids=lambda v: v if isinstance(v, str) else "")
@pytest.mark.parametrize("path", ["radix", "direct"])
def test_exp1_both_chaining_paths(ctx, name, g, path):
    """The radix-partitioned (LDS-slice) and the direct chaining kernels give identical results."""
    import torch
    import hj3d
    R, S, b = exp1_rel(g)
    dR, dS = dev(R), dev(S)
    if path == "radix":
        ctx.radix_min(0)
    else:
        ctx.force_direct(True)
    try:
        for plan in ("Csr", "CsrUU", "Crs", "Nsr", "Nrs", "NrsNU"):
            nb = hj3d.num_buckets_exp1(plan, len(R), g["numDvSa"], b)
            ref = g["plans"][plan]
            got = hj3d.exp1_plan(ctx, plan, dR, dS, nb)
            assert (got["c_probe"], got["c_cmp"], got["c_top"]) == (ref["c_probe"], ref["c_cmp"], ref["c_top"]), plan
            assert {k: got["stats"][k] for k in STAT_KEYS} == {k: ref["stats"][k] for k in STAT_KEYS}, plan
            assert got["out"] == ref["out"], plan
            cap = max(ref["out"]["n"], len(S), len(R), 1)
            out = torch.zeros((cap, 2), dtype=torch.int32, device="cuda")
            got = hj3d.exp1_plan(ctx, plan, dR, dS, nb, out=out, stats=False)
            host = out.cpu().numpy().view(np.uint32)
            dense = plan in ("Csr", "NrsNU")  # one slot per probe tuple
            host = host[host[:, 1] != 0xFFFFFFFF][: ref["out"]["n"]] if dense else host[: ref["out"]["n"]]
            assert host_checksums(host) == ref["out"], plan
    finally:
        ctx.radix_min(1 << 20)
        ctx.force_direct(False)


@pytest.mark.parametrize("nb", [64, 2000, 50000])
@pytest.mark.parametrize("path", ["radix", "direct"])
def test_nested_many_keys_per_bucket(ctx, nb, path):
    """Nested build with many distinct keys per bucket: ~1560 (the aggregation build gives up on
    key ranges too dense for its LDS table and the sort-based build takes over), ~50 (ranges retried
    in halves) and ~2 per bucket; every counter and the output equal the oracle's."""
    import hj3d
    rng = np.random.default_rng(nb)
    nR, nS = 100_000, 400_000
    Rk = rng.permutation(nR).astype(np.uint32)
    Sa = rng.integers(0, nR, nS, dtype=np.uint32)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    if path == "radix":
        ctx.radix_min(0)
    else:
        ctx.force_direct(True)
    try:
        for plan, e in (("Nsr", O.nested_plan(R, 0, S, 1, nb, True)), ("Nrs", O.nested_plan(S, 1, R, 0, nb, True))):
            got = hj3d.exp1_plan(ctx, plan, dev(R), dev(S), nb)
            assert (got["c_probe"], got["c_cmp"], got["c_unnest"], got["c_top"]) == \
                (e.c_probe, e.c_cmp, e.c_unnest, e.c_top), plan
            assert got["out"] == e.out, plan
            assert {k: got["stats"][k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}, plan
    finally:
        ctx.radix_min(1 << 20)
        ctx.force_direct(False)


def test_scan_status_regrowth_ignores_stale_memory():
    """exclusive_scan_u32's look-back status words are cleared whenever their buffer is
    reallocated, also when the allocator hands back the freed block's address. Device memory
    is first filled with words that read as 'published' for the first 64 scan epochs and
    released to HIP; a fresh context then runs sort-built nested tables of growing size (each
    regrows the status buffer and the sort scratch), whose distinct-key counts must equal numpy's.
    Before the fix a reallocation at the old address skipped the clear (a rare wrong main count)."""
    import torch
    import hj3d
    k = torch.arange(1 << 24, dtype=torch.int64, device="cuda")
    poison = (((k % 64) + 1) << 34) | (1 << 32) | 7  # epoch 1..64, flag 'aggregate', value 7
    del k, poison
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    c = hj3d.Context()
    c.force_direct(True)
    c.nested_sort(True)
    try:
        rng = np.random.default_rng(5)
        for n in (20_000, 90_000, 400_000, 1_700_000, 4_000_000):
            a = rng.integers(0, n // 10, n, dtype=np.uint32)
            S = O.tuples3(np.arange(n, dtype=np.uint32), a)
            dS = dev(S)
            t = hj3d.Table(c, hj3d.HJ3D_NESTED, max(n // 7, 1))
            t.build(hj3d.Rel(dS, 1, 0))
            st = t.stats()
            t.close()
            assert st["distinct"] == len(np.unique(a)), n
            assert st["entries"] == n, n
    finally:
        c.close()


@pytest.mark.parametrize("zipf", [False, True], ids=["uniform", "zipf"])
@pytest.mark.parametrize("nb", [2000, 7000, 20000, 100000, 250000])
def test_nested_agg_build_vs_oracle(ctx, nb, zipf):
    """The partition + LDS aggregation nested build (nested_agg.hip) at ~50, 14, 5, 1 and 0.4
    distinct keys per bucket (at 50 it gives up and the sort build replaces the table after the
    fact; at 14 it splits every partition into several rounds), uniform and Zipf(1.0)
    duplicates (hot keys aggregated per wave): counters, output checksums and statistics equal
    the oracle's, and equal the LSD key-sort build's and those of the aggregation build on the
    packed partitioner's slices (HJ3D_OPT_NESTED_PK: the form of tables above 2048 partitions)."""
    import hj3d
    rng = np.random.default_rng(nb + zipf)
    nR, nS = 100_000, 400_000
    Rk = rng.permutation(nR).astype(np.uint32)
    Sa = (np.minimum(rng.zipf(1.3, nS) - 1, nR - 1) if zipf else rng.integers(0, nR, nS)).astype(np.uint32)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    ctx.radix_min(0)
    try:
        for plan, e in (("Nsr", O.nested_plan(R, 0, S, 1, nb, True)), ("Nrs", O.nested_plan(S, 1, R, 0, nb, True))):
            for mode in ("agg", "slices", "sort"):
                ctx.nested_sort(mode == "sort")
                ctx.nested_pk(mode == "slices")
                t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
                got = hj3d.exp1_plan(ctx, plan, dev(R), dev(S), nb, table=t)
                path = t.build_path()
                t.close()
                assert (got["c_probe"], got["c_cmp"], got["c_unnest"], got["c_top"]) == \
                    (e.c_probe, e.c_cmp, e.c_unnest, e.c_top), (plan, mode, path)
                assert got["out"] == e.out, (plan, mode, path)
                assert {k: got["stats"][k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}, (plan, mode)
                # the packed-slice form really ran where nothing sends it to the sort build (~50
                # keys per bucket give up; Zipf S.a overflows the slices' regions)
                if mode == "slices" and nb >= 20000 and not (zipf and plan == "Nrs"):
                    assert path.startswith("nested_agg_slices"), (plan, path)
    finally:
        ctx.radix_min(1 << 20)
        ctx.nested_sort(False)
        ctx.nested_pk(False)


def test_nested_slices_lookback_timeout_falls_back(ctx):
    """The slice-path aggregation build's failure path (HJ3D_OPT_DIAG_LOOKBACK: partition 0 never
    publishes its count, so every successor's look-back runs out after 1 ms and sets the give-up
    flag): the sort build replaces the table and the join equals the oracle's; the look-back words
    are left in step, so the next build on the same context takes the slice path again and is exact."""
    import hj3d
    rng = np.random.default_rng(17)
    nR, nS, nb = 100_000, 400_000, 20_000  # 20 partitions of ~20K pairs: the streaming form (not registers)
    R = O.tuples3(rng.permutation(nR).astype(np.uint32), np.zeros(nR, np.uint32))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), rng.integers(0, nR, nS).astype(np.uint32))
    e = O.nested_plan(S, 1, R, 0, nb, True)
    dR, dS = dev(R), dev(S)
    ctx.radix_min(0)
    ctx.nested_pk(True)
    try:
        for diag, want in ((100_000, "nested_sort"), (0, "nested_agg_slices"), (100_000, "nested_sort"),
                           (0, "nested_agg_slices")):
            ctx.diag_lookback(diag)
            t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
            got = hj3d.exp1_plan(ctx, "Nrs", dR, dS, nb, table=t)
            path = t.build_path()
            t.close()
            assert path == want, (diag, path)
            assert (got["c_probe"], got["c_cmp"], got["c_unnest"], got["c_top"]) == \
                (e.c_probe, e.c_cmp, e.c_unnest, e.c_top), (diag, path)
            assert got["out"] == e.out, (diag, path)
            assert {k: got["stats"][k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}, (diag, path)
    finally:
        ctx.diag_lookback(0)
        ctx.radix_min(1 << 20)
        ctx.nested_pk(False)


@pytest.mark.parametrize("path", ["default", "partitioned"])
@pytest.mark.parametrize("name,g", EXP4, ids=[n for n, _ in EXP4])
def test_exp4_plans_bit_exact(ctx, name, g, path):
    """Experiment 4 against the reference's fixtures; `partitioned` lowers HJ3D_OPT_RADIX_MIN so
    even these small probe sides take the partitioned Ndu kernels (LDS slices of both tables)."""
    import hj3d
    log2R, a, A, b, B = g["generator_args"][1:6]
    Sa, Ta = O.gen_exp4(log2R, a, A, b, B)
    n, cardR = len(Sa), 1 << log2R
    R = dev(O.tuples2(np.arange(cardR, dtype=np.uint32), np.zeros(cardR, np.uint32)))
    S = dev(O.tuples2(np.arange(n, dtype=np.uint32), Sa))
    T = dev(O.tuples2(np.arange(n, dtype=np.uint32), Ta))
    if path == "partitioned":
        ctx.radix_min(1 << 6)
    try:
        _exp4_check(ctx, g, R, S, T)
    finally:
        ctx.radix_min(1 << 20)


@pytest.mark.parametrize("parts", [2, 3, 8])
@pytest.mark.parametrize("name,g", EXP4, ids=[n for n, _ in EXP4])
def test_exp4_owner_split_equals_reference(ctx, name, g, parts):
    """Experiment 4 co-partitioned by bucket range of the FK hash (R, S and T) and run
    owner after owner on this GPU (hj3d.exp4_plan_sharded: per owner one hj3d_build_many of its S and
    T pairs, explicit global rows, and hj3d_probe2 with its R pairs): the summed counters and
    checksums equal the reference binary's fixture, Ndu and Chj. The multi-GPU strand's per-rank
    compute without the exchange (unmeasured on hardware at N > 1)."""
    import hj3d
    log2R, a, A, b, B = g["generator_args"][1:6]
    Sa, Ta = O.gen_exp4(log2R, a, A, b, B)
    n, cardR = len(Sa), 1 << log2R
    R = dev(O.tuples2(np.arange(cardR, dtype=np.uint32), np.zeros(cardR, np.uint32)))
    S = dev(O.tuples2(np.arange(n, dtype=np.uint32), Sa))
    T = dev(O.tuples2(np.arange(n, dtype=np.uint32), Ta))
    for plan in ("Ndu", "Chj"):
        got = hj3d.exp4_plan_sharded(ctx, plan, R, S, T, g["nb"], parts)
        _exp4_compare(plan, got, g["plans"][plan])


def _exp4_compare(plan, got, ref):
    for k in ("c_probe_RS", "c_probe_RS_cmp", "c_probe_RT", "c_probe_RT_cmp", "c_top"):
        assert got[k.lower()] == ref[k], (plan, k, got[k.lower()], ref[k])
    if plan == "Ndu":
        assert got["c_unnest_1"] == ref["c_unnest_1"] and got["c_unnest_2"] == ref["c_unnest_2"]
    assert {k: got[k] for k in ("sum_a", "sum_b", "sum_c", "sum_h", "xor_h")} == \
           {k: ref["out"][k] for k in ("sum_a", "sum_b", "sum_c", "sum_h", "xor_h")}, plan


def _exp4_check(ctx, g, R, S, T):
    """Both plans, with the two builds as one hj3d_build_many call (one launch sequence for the two
    nested tables) and as two hj3d_build calls."""
    import hj3d
    for plan, fused in (("Ndu", True), ("Ndu", False), ("Chj", True)):
        got = hj3d.exp4_plan(ctx, plan, R, S, T, g["nb"], fused=fused)
        ref = g["plans"][plan]
        for k in ("c_probe_RS", "c_probe_RS_cmp", "c_probe_RT", "c_probe_RT_cmp", "c_top"):
            assert got[k.lower()] == ref[k], (plan, k, got[k.lower()], ref[k])
        if plan == "Ndu":
            assert got["c_unnest_1"] == ref["c_unnest_1"] and got["c_unnest_2"] == ref["c_unnest_2"]
        assert {k: got[k] for k in ("sum_a", "sum_b", "sum_c", "sum_h", "xor_h")} == \
               {k: ref["out"][k] for k in ("sum_a", "sum_b", "sum_c", "sum_h", "xor_h")}, plan


def _oracle_plans(R, S, nbR, nbS):
    return {
        "Csr": O.chain_plan(R, 0, S, 1, nbR, True), "CsrUU": O.chain_plan(R, 0, S, 1, nbR, False),
        "Crs": O.chain_plan(S, 1, R, 0, nbS, False), "Nsr": O.nested_plan(R, 0, S, 1, nbR, True),
        "Nrs": O.nested_plan(S, 1, R, 0, nbS, True), "NrsNU": O.nested_plan(S, 1, R, 0, nbS, False),
    }


def _compare(ctx, R, S, nbR, nbS):
    import hj3d
    exp = _oracle_plans(R, S, nbR, nbS)
    dR, dS = dev(R), dev(S)
    for plan in PLANS:
        e = exp[plan]
        nb = nbR if hj3d.EXP1_PLANS[plan][1] == "R" else nbS
        got = hj3d.exp1_plan(ctx, plan, dR, dS, nb)
        assert (got["c_probe"], got["c_cmp"], got["c_top"], got["c_unnest"]) == \
               (e.c_probe, e.c_cmp, e.c_top, e.c_unnest), plan
        assert {k: got["stats"][k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}, plan
        assert got["out"] == e.out, plan


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_relations_vs_oracle(ctx, seed):
    """Non-key build sides, dangling FKs, duplicate R keys, tiny and odd bucket counts."""
    rng = np.random.default_rng(seed)
    nR, nS = int(rng.integers(1, 5000)), int(rng.integers(1, 20000))
    Rk = rng.integers(0, nR * 2, nR).astype(np.uint32)  # duplicates + keys without partners
    Sa = rng.integers(0, nR * 2, nS).astype(np.uint32)
    R = O.tuples3(Rk, np.zeros(nR, np.uint32))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    for nbR, nbS in ((max(nR // 3, 1), 7), (1, 1), (nR + 13, O.num_distinct(Sa))):
        _compare(ctx, R, S, nbR, nbS)


def test_empty_relations(ctx):
    R = O.tuples3(np.array([5, 9], np.uint32), np.zeros(2, np.uint32))
    S0 = O.tuples3(np.zeros(0, np.uint32), np.zeros(0, np.uint32))
    _compare(ctx, R, S0, 2, 1)   # empty probe side / empty build side
    _compare(ctx, S0, R, 1, 2)


def test_skewed_hot_key_heavy_unnest(ctx):
    """One key owns most of S: the nested build groups ~200k duplicates and the unnest of the hot
    key goes through the workgroup-wide (heavy) expansion path; counters must not change."""
    rng = np.random.default_rng(7)
    nR, nS = 1000, 300_000
    Rk = rng.permutation(nR).astype(np.uint32)
    Sa = rng.integers(0, nR, nS).astype(np.uint32)
    Sa[rng.random(nS) < 0.7] = 17
    R = O.tuples3(Rk, np.zeros(nR, np.uint32))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    _compare(ctx, R, S, nR, O.num_distinct(Sa))


@pytest.mark.parametrize("single", [False, True], ids=["stable", "single_pass"])
def test_bucket_shards_sum_to_single_table(ctx, single):
    """Multi-GPU building block: tables that own disjoint bucket ranges, probed by the tuples of
    their range (hj3d_partition; single_pass: the probe side from hj3d_partition_strided, no order
    inside a range), add up to the single-table reference counters exactly."""
    import torch
    import hj3d
    g = dict(load_golden("exp1_R1024_S4096_zipf.json"))["exp1_R1024_S4096_zipf"]
    R, S, b = exp1_rel(g)
    dR, dS = dev(R), dev(S)
    for plan in ("Csr", "Crs", "Nrs", "Nsr"):
        kind, bside, bkey, pkey, unique, unnest = hj3d.EXP1_PLANS[plan]
        nb = hj3d.num_buckets_exp1(plan, len(R), g["numDvSa"], b)
        build = hj3d.Rel(dR if bside == "R" else dS, key_word=bkey)
        probe = hj3d.Rel(dS if bside == "R" else dR, key_word=pkey)
        parts = 3
        bp = torch.zeros((build.n, 2), dtype=torch.int32, device="cuda")
        stride = probe.n if single else None
        pp = torch.zeros((probe.n * (parts if single else 1), 2), dtype=torch.int32, device="cuda")
        bc = torch.zeros(parts, dtype=torch.int64, device="cuda")
        pc = torch.zeros(parts, dtype=torch.int64, device="cuda")
        ctx.partition(build, nb, parts, bp, bc)
        ctx.partition(probe, nb, parts, pp, pc, stride=stride)
        bcs, pcs = [0] + np.cumsum(bc.cpu().numpy()).tolist(), [0] + np.cumsum(pc.cpu().numpy()).tolist()
        if single:  # range p's probe pairs at [p * stride, p * stride + pc[p])
            pcs = [[p * stride, p * stride + int(pc[p])] for p in range(parts)]
        else:
            pcs = [[pcs[p], pcs[p + 1]] for p in range(parts)]
        tot = {"c_cmp": 0, "n_out": 0, "n_matched": 0, "sum_h": 0, "xor_h": 0, "empty": 0, "cc0_max": 0}
        for p in range(parts):
            lo, hi = hj3d.part_range(nb, parts, p)
            t = hj3d.Table(ctx, kind, nb, lo, hi)
            t.build(hj3d.Rel(bp[bcs[p]:bcs[p + 1]], key_word=0, row_word=1))
            r = ctx.probe(t, hj3d.Rel(pp[pcs[p][0]:pcs[p][1]], key_word=0, row_word=1), unique=unique, unnest=unnest)
            st = t.stats()
            tot["c_cmp"] += r.n_cmps
            tot["n_out"] += r.n_out
            tot["n_matched"] += r.n_matched
            tot["sum_h"] = (tot["sum_h"] + r.sum_h) % (1 << 64)
            tot["xor_h"] ^= r.xor_h
            tot["empty"] += st["empty"]
            tot["cc0_max"] = max(tot["cc0_max"], st["cc0_max"])
        ref = g["plans"][plan]
        assert tot["c_cmp"] == ref["c_cmp"], plan
        assert tot["n_out"] == ref["out"]["n"], plan
        assert (tot["sum_h"], tot["xor_h"]) == (ref["out"]["sum_h"], ref["out"]["xor_h"]), plan
        assert tot["empty"] == ref["stats"]["empty"] and tot["cc0_max"] == ref["stats"]["cc0_max"], plan


@pytest.mark.parametrize("name,g", [x for x in EXP1 if x[1]["nS"] <= 1_100_000], ids=lambda v: v if isinstance(v, str) else "")
def test_num_distinct_bitmap_matches_reference(ctx, name, g):
    """#dv(S.a) from the device pre-pass (hj3d_key_bitmap + hj3d_bitmap_or_popcount) equals the
    reference's numDvSa (unordered_set, main_experiment1.cc:453-454) recorded in the fixture; the
    same count from two half-bitmaps OR'ed (the multi-GPU form, rows = 2) and the outside count."""
    import torch
    import hj3d
    _, S, _ = exp1_rel(g)
    nR = g["nR"]
    relS = hj3d.Rel(dev(S), key_word=1)
    assert ctx.num_distinct(relS, nR) == g["numDvSa"]
    n = S.shape[0]
    words = (nR + 31) // 32
    bm = torch.zeros((2, words), dtype=torch.int32, device="cuda")
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.key_bitmap(hj3d.Rel(dev(S[: n // 2]), key_word=1), nR, bm[0], out)
    ctx.key_bitmap(hj3d.Rel(dev(S[n // 2:]), key_word=1), nR, bm[1], out)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.bitmap_or_popcount(bm, cnt)
    assert int(cnt.item()) == g["numDvSa"] and int(out.item()) == 0
    # a domain that excludes the largest keys counts them as outside
    k = int(S[:, 1].max())
    if k == 0:
        return
    bm2 = torch.zeros((1, (k + 31) // 32), dtype=torch.int32, device="cuda")
    ctx.key_bitmap(relS, k, bm2[0], out)
    assert int(out.item()) == int((S[:, 1] >= k).sum())


@pytest.mark.parametrize("theta", [0.6, 1.0])
def test_chaining_build_skewed_partition(ctx, theta):
    """A chaining table at fill ~1 over Zipf keys: the staged persistent build (k_rp_build3) holds a
    partition of up to 12288 pairs in registers; the hot keys' partition exceeds that and takes the
    HBM scatter fallback inside the same kernel. Statistics, comparison counts and the output of
    the unique and non-unique probes equal the oracle's (rows sorted inside buckets of <= 32)."""
    rng = np.random.default_rng(int(theta * 10))
    nB, nP = 2_000_000, 2_000_000
    Bk = (np.minimum(rng.zipf(1.0 + theta, nB), 5_000_000) - 1).astype(np.uint32)
    Pk = rng.integers(0, 4_000_000, nP).astype(np.uint32)
    B = O.tuples3(Bk, np.zeros(nB, np.uint32))
    P = O.tuples3(np.arange(nP, dtype=np.uint32), Pk)
    import hj3d
    for unique in (True, False):
        e = O.chain_plan(B, 0, P, 1, nB, unique)
        t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nB)
        t.build(hj3d.Rel(dev(B), 0))
        r = ctx.probe(t, hj3d.Rel(dev(P), 1), unique=unique)
        assert (r.n_out, r.n_cmps) == (e.c_probe, e.c_cmp), unique
        assert {"n": r.n_out, "sum_a": r.sum_a, "sum_b": r.sum_b, "sum_c": 0, "sum_h": r.sum_h, "xor_h": r.xor_h} == e.out
        st = t.stats()
        assert {k: st[k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}


@pytest.mark.parametrize("items", [5, 6, 7, 8])
def test_packed_probe_items_per_lane(ctx, items):
    """The packed unique probe gives the reference's counters and output pairs for every chunk
    width of its region walk (HJ3D_OPT_PROBE_ITEMS; config B's default is 7)."""
    import torch
    import hj3d
    cases = [x for x in EXP1 if x[1]["nR"] >= 64 and x[1]["nS"] <= 9_000_000]
    ctx.radix_min(0)
    ctx.probe_items(items)
    try:
        for name, g in cases:
            R, S, b = exp1_rel(g)
            dR, dS = dev(R), dev(S)
            nb = hj3d.num_buckets_exp1("Csr", len(R), g["numDvSa"], b)
            ref = g["plans"]["Csr"]
            out = torch.zeros((max(len(S), 1), 2), dtype=torch.int32, device="cuda")
            got = hj3d.exp1_plan(ctx, "Csr", dR, dS, nb, out=out, stats=False)
            assert (got["c_probe"], got["c_cmp"], got["c_top"]) == (ref["c_probe"], ref["c_cmp"], ref["c_top"]), name
            host = out.cpu().numpy().view(np.uint32)
            host = host[host[:, 1] != 0xFFFFFFFF]
            assert host_checksums(host) == ref["out"], name
    finally:
        ctx.probe_items(0)
        ctx.radix_min(1 << 20)


@pytest.mark.parametrize("sync", [False, True], ids=["lazy", "sync"])
@pytest.mark.parametrize("dense", [0, 1])
def test_build_many_one_table_gives_up(ctx, dense, sync):
    """hj3d_build_many over two nested tables of one geometry where table `dense` holds ~50 keys
    per bucket (the LDS aggregation build gives up; the sort build replaces that table) and the
    other ~2 (aggregation build kept). Both tables' statistics and probe counters equal the
    oracle's. Lazy: the replacement runs at the table's next use, is timed as HJ3D_T_BUILD (not as
    probe work), and build_path(finish=False) reports the started path with "?". Sync
    (HJ3D_OPT_SYNC_BUILD): the tables are finished inside the call, so the build relations are
    overwritten and released before the first use."""
    import torch
    import hj3d
    rng = np.random.default_rng(17 + dense)
    nb, n = 2000, 400_000
    dom = (100_000, 4_000) if dense == 0 else (4_000, 100_000)
    rels = [O.tuples3(np.arange(n, dtype=np.uint32), rng.integers(0, d, n, dtype=np.uint32)) for d in dom]
    P = O.tuples3(np.arange(120_000, dtype=np.uint32) % 110_000, np.zeros(120_000, dtype=np.uint32))
    exp = [O.nested_plan(r, 1, P, 0, nb, True) for r in rels]
    ctx.radix_min(0)
    ctx.sync_build(sync)
    ctx.timing(True)
    try:
        ts = [hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb) for _ in range(2)]
        dr = [dev(r) for r in rels]
        ctx.build_many(ts, [hj3d.Rel(d, 1) for d in dr])
        if sync:
            assert not ts[dense].build_path(finish=False).endswith("?")
            for d in dr:
                d.fill_(-1)
            del dr
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        else:
            assert ts[dense].build_path(finish=False) == "nested_agg?"
        ctx.sync()
        ctx.timer_reset()
        dP = dev(P)
        for k in range(2):
            got = ctx.probe(ts[k], hj3d.Rel(dP, 0), unnest=True)
            e = exp[k]
            assert (got.n_matched, got.n_cmps, got.n_out) == (e.c_probe, e.c_cmp, e.c_unnest), k
            assert {f: getattr(got, f) for f in ("sum_a", "sum_b", "sum_h", "xor_h")} == \
                {f: e.out[f] for f in ("sum_a", "sum_b", "sum_h", "xor_h")}, k
            assert {f: ts[k].stats()[f] for f in STAT_KEYS} == {f: e.stats[f] for f in STAT_KEYS}, k
        build_ms, build_cnt = ctx.timer(hj3d.T_BUILD)
        assert build_cnt == (0 if sync else 1)  # the fallback build, counted as build work
        assert ts[dense].build_path() == "nested_sort"
        assert ts[1 - dense].build_path() == "nested_agg"
        for t in ts:
            t.close()
    finally:
        ctx.timing(False)
        ctx.sync_build(False)
        ctx.radix_min(1 << 20)


@pytest.mark.parametrize("theta,n,dom", [(1.0, 4_000_000, 200_000), (1.3, 3_000_000, 50_000), (0.8, 6_000_000, 600_000)])
def test_nested_build_hot_keys(ctx, theta, n, dom):
    """Zipf-skewed build keys whose hottest keys hold most of their partitions' rows: the heavy
    partitions find their hot key from a sample and take the register path for its rows (counted
    per lane in pass A, placed by wave prefix and ballot count in pass B); the other keys keep the
    LDS table. Counters, output checksums and statistics equal the oracle's (Nrs: nested table on
    S.a, probe R, unnest; HtNested1::insert, ht_nested.hh:287-311)."""
    import hj3d
    rng = np.random.default_rng(int(theta * 10))
    Sa = (np.minimum(rng.zipf(1.0 + theta if theta > 1.0 else 2.0, n) if theta > 1.0 else
          _zipf_keys(rng, n, dom, theta), dom) - (1 if theta > 1.0 else 0)).astype(np.uint32)
    S = O.tuples3(np.arange(n, dtype=np.uint32), Sa)
    R = O.tuples3(np.arange(dom, dtype=np.uint32), np.zeros(dom, np.uint32))
    nb = O.num_distinct(Sa)
    e = O.nested_plan(S, 1, R, 0, nb, True)
    got = hj3d.exp1_plan(ctx, "Nrs", dev(R), dev(S), nb)
    assert (got["c_probe"], got["c_cmp"], got["c_unnest"], got["c_top"]) == (e.c_probe, e.c_cmp, e.c_unnest, e.c_top)
    assert got["out"] == e.out
    assert {k: got["stats"][k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}


def _zipf_keys(rng, n, dom, theta):
    """n keys in [0, dom) with P(k) ~ 1 / (k + 1)^theta (theta < 1: inverse CDF on the exact weights)."""
    w = 1.0 / np.arange(1, dom + 1, dtype=np.float64) ** theta
    c = np.cumsum(w)
    c /= c[-1]
    return np.searchsorted(c, rng.random(n)).astype(np.uint32)


@pytest.mark.parametrize("explicit,nb,path", [(False, 200_003, "nested_agg"), (True, 400_009, "nested_agg_reg")],
                         ids=["streaming_implicit_rows", "register_form_explicit_rows"])
def test_build_many_hot_key_split(ctx, explicit, nb, path):
    """Two nested tables in one hj3d_build_many whose heavy partitions are dominated by one Zipf key
    each: k_nagg_hot splits the key off before the aggregation (its rows written down from the end of
    the partition's sub range, the other pairs compacted), in both tables (table 1's sub rows are
    numbered from its own first pair) and with explicit row ids; with ~25 K pairs per partition the
    streaming aggregation runs after the split, with ~13 K (less than a chunk of the split on average:
    no split) the register form, which leaves its partitions too large for its registers to the
    streaming form (k_nagg_defer). Counters, output checksums and statistics equal the oracle's per
    table (HtNested1::insert, ht_nested.hh:287-311)."""
    import hj3d
    rng = np.random.default_rng(77 + explicit)
    n, dom = 5_000_000, 600_000
    rels, brow = [], []
    for k in range(2):
        r = np.zeros((n, 3), np.uint32)
        r[:, 1] = (_zipf_keys(rng, n, dom, 0.9 + 0.2 * k) * 7 + k) % dom
        if explicit:
            r[:, 2] = np.sort(rng.choice(2_000_000_000, n, replace=False)).astype(np.uint32)
        rels.append(r)
        brow.append(2 if explicit else None)
    P = O.tuples3(rng.integers(0, dom, 700_000, dtype=np.uint32), np.zeros(700_000, np.uint32))
    exp = [O.nested_plan(rels[k], 1, P, 0, nb, True, brow=brow[k]) for k in range(2)]
    ts = [hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb) for _ in range(2)]
    dr = [dev(r) for r in rels]
    ctx.build_many(ts, [hj3d.Rel(dr[k], 1, row_word=brow[k]) for k in range(2)])
    dP = dev(P)
    for k in range(2):
        assert ts[k].build_path() == path, ts[k].build_path()
        got = ctx.probe(ts[k], hj3d.Rel(dP, 0), unnest=True)
        e = exp[k]
        assert (got.n_matched, got.n_cmps, got.n_out) == (e.c_probe, e.c_cmp, e.c_unnest), k
        assert {f: getattr(got, f) for f in ("sum_a", "sum_b", "sum_h", "xor_h")} == \
            {f: e.out[f] for f in ("sum_a", "sum_b", "sum_h", "xor_h")}, k
        assert {f: ts[k].stats()[f] for f in STAT_KEYS} == {f: e.stats[f] for f in STAT_KEYS}, k
    for t in ts:
        t.close()


@pytest.mark.parametrize("explicit", [1, 0], ids=["r1_explicit", "r0_explicit"])
def test_build_many_mixed_row_modes(ctx, explicit):
    """hj3d_build_many partitions both relations in one pass. With one relation on implicit rows and
    the other on explicit row ids, large enough for the whole-segment scatter (k_rp_wscatter, >= 4
    tiles of 16384 per workgroup), both tables must carry their own rows: counters, output checksums
    and statistics equal the oracle's per table (explicit rows: ascending, with gaps, over a wide range)."""
    import hj3d
    rng = np.random.default_rng(41 + explicit)
    nb, n = 2_000_003, 9_000_000
    rels, brow = [], []
    for k in range(2):
        r = np.zeros((n, 3), np.uint32)
        r[:, 1] = rng.integers(0, 2_500_000, n, dtype=np.uint32)
        if k == explicit:
            # (ascending in scan order, as the ABI requires of explicit build rows: the reference's
            # insertion order)
            r[:, 2] = np.sort(rng.choice(1_000_000_000, n, replace=False)).astype(np.uint32)
        rels.append(r)
        brow.append(2 if k == explicit else None)
    P = O.tuples3(rng.integers(0, 2_500_000, 1_500_000, dtype=np.uint32), np.zeros(1_500_000, np.uint32))
    exp = [O.nested_plan(rels[k], 1, P, 0, nb, True, brow=brow[k]) for k in range(2)]
    ts = [hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb) for _ in range(2)]
    dr = [dev(r) for r in rels]
    ctx.build_many(ts, [hj3d.Rel(dr[k], 1, row_word=brow[k]) for k in range(2)])
    dP = dev(P)
    for k in range(2):
        assert ts[k].build_path() == "nested_agg", ts[k].build_path()
        got = ctx.probe(ts[k], hj3d.Rel(dP, 0), unnest=True)
        e = exp[k]
        assert (got.n_matched, got.n_cmps, got.n_out) == (e.c_probe, e.c_cmp, e.c_unnest), k
        assert {f: getattr(got, f) for f in ("sum_a", "sum_b", "sum_h", "xor_h")} == \
            {f: e.out[f] for f in ("sum_a", "sum_b", "sum_h", "xor_h")}, k
        assert {f: ts[k].stats()[f] for f in STAT_KEYS} == {f: e.stats[f] for f in STAT_KEYS}, k
    for t in ts:
        t.close()


@pytest.mark.parametrize("keys_per_bucket", [1, 4])
def test_nested_slices_register_form(ctx, keys_per_bucket):
    """The register form of the slice aggregation (k_nagg_reg: a slice's pairs held in registers,
    its sub rows assembled in LDS). At ~1 key per bucket every slice takes it; at ~4 keys per bucket
    the slices hold more distinct keys than its table, so it defers them all to k_nagg's list form.
    Counters, output checksums and statistics equal the oracle's either way."""
    import hj3d
    rng = np.random.default_rng(31 + keys_per_bucket)
    nb, nS = 100_000, 600_000
    Sa = rng.integers(0, nb * keys_per_bucket, nS, dtype=np.uint32)
    Rk = rng.permutation(nb * keys_per_bucket).astype(np.uint32)[:200_000]
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    e = O.nested_plan(S, 1, R, 0, nb, True)
    ctx.radix_min(0)
    ctx.nested_pk(True)
    try:
        t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
        got = hj3d.exp1_plan(ctx, "Nrs", dev(R), dev(S), nb, table=t)
        path = t.build_path()
        st = t.stats()
        t.close()
        assert path == "nested_agg_slices_reg", path
        assert (got["c_probe"], got["c_cmp"], got["c_unnest"], got["c_top"]) == \
            (e.c_probe, e.c_cmp, e.c_unnest, e.c_top)
        assert got["out"] == e.out
        assert {k: st[k] for k in STAT_KEYS} == {k: e.stats[k] for k in STAT_KEYS}
    finally:
        ctx.radix_min(1 << 20)
        ctx.nested_pk(False)


@pytest.mark.parametrize("plan", ["Nrs", "NrsNU", "Nsr"])
def test_nested_probe_two_level_slices(ctx, plan):
    """The partitioned nested probe beyond the one-level partitioner's 2048 LDS slices (config D's
    1e8-bucket table on one GPU) runs on the packed partitioner's two levels (pk_probe_slices:
    k_pk_part + k_pk_split, packed pairs, every slice in LDS). A slice bound of 64 buckets
    (HJ3D_OPT_PK_SLICE) puts a 200K-bucket table there (3125 slices); Zipf duplicates overflow some
    regions, whose pairs the overflow kernel probes. Counters, checksums and the materialised pairs
    equal the oracle's."""
    import torch
    import hj3d
    rng = np.random.default_rng(41)
    nb, nR, nS = 200_000, 300_000, 800_000
    Rk = rng.permutation(nR).astype(np.uint32)
    Sa = np.minimum(rng.zipf(1.5, nS) - 1, nR - 1).astype(np.uint32)
    Sa[: nS // 2] = rng.integers(0, nR, nS // 2, dtype=np.uint32)
    R = O.tuples3(Rk, np.zeros_like(Rk))
    S = O.tuples3(np.arange(nS, dtype=np.uint32), Sa)
    e = _oracle_plans(R, S, nb, nb)[plan]
    ctx.radix_min(0)
    ctx.pk_slice_max(64)
    try:
        got = hj3d.exp1_plan(ctx, plan, dev(R), dev(S), nb)
        assert (got["c_probe"], got["c_cmp"], got["c_unnest"], got["c_top"]) == \
            (e.c_probe, e.c_cmp, e.c_unnest, e.c_top), plan
        assert got["out"] == e.out, plan
        cap = max(e.out["n"], nS, nR, 1)
        out = torch.zeros((cap, 2), dtype=torch.int32, device="cuda")
        got = hj3d.exp1_plan(ctx, plan, dev(R), dev(S), nb, out=out, stats=False)
        host = out.cpu().numpy().view(np.uint32)
        if plan == "NrsNU":  # one slot per probe tuple (R), unmatched slots carry 0xFFFFFFFF
            host = host[:nR]
            host = host[host[:, 1] != 0xFFFFFFFF]
        else:
            host = host[: e.out["n"]]
        assert host_checksums(host) == e.out, plan
    finally:
        ctx.radix_min(1 << 20)
        ctx.pk_slice_max(0)
