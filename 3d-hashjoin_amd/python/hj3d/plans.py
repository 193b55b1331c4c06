"""Experiment plans on the hj3d engine, reported in the reference's CSV vocabulary.

One function per reference plan family; each builds and probes through the C ABI and
returns the counters the reference writes to its measurement CSV:

  Csr / CsrUU  chaining build R, probe S (unique early exit / not)  main_experiment1.cc:623-848
  Crs          chaining build S.a, probe R                          main_experiment1.cc:850-967
  Nsr          nested build R, probe S, unnest                      main_experiment1.cc:1078-1185
  Nrs          nested build S.a, probe R, unnest                    main_experiment1.cc:969-1076
  NrsNU        nested build S.a, probe R, no unnest                 main_experiment1.cc:1187-1285
  Ndu / Chj    experiment 4 deferred unnesting / chaining           main_experiment4.cc:831-1043
"""
from __future__ import annotations

from . import HJ3D_CHAIN, HJ3D_NESTED, Context, Rel, Table

# plan -> (table kind, build relation "R"|"S", build key word, probe key word, unique, unnest)
EXP1_PLANS = {
    "Csr": (HJ3D_CHAIN, "R", 0, 1, True, False),
    "CsrUU": (HJ3D_CHAIN, "R", 0, 1, False, False),
    "Crs": (HJ3D_CHAIN, "S", 1, 0, False, False),
    "Nsr": (HJ3D_NESTED, "R", 0, 1, False, True),
    "Nrs": (HJ3D_NESTED, "S", 1, 0, False, True),
    "NrsNU": (HJ3D_NESTED, "S", 1, 0, False, False),
}


def num_buckets_exp1(plan: str, card_r: int, num_dv_sa: int, b: int = 1) -> int:
    """#buckets as the reference chooses them: max(|R|/b, 1) for builds on R.k,
    max(#dv(S.a)/b, 1) for builds on S.a (main_experiment1.cc:651, 875, 1001, 1111, 1214)."""
    build_side = EXP1_PLANS[plan][1]
    return max((card_r if build_side == "R" else num_dv_sa) // b, 1)


def exp1_plan(ctx: Context, plan: str, R, S, nb: int, out=None, table: Table | None = None,
              stats: bool = True, checksum: bool = True) -> dict:
    """Run one experiment-1 plan on device relations R, S ((n,3) int32 tensors {k,a,b}).

    Returns {nb, c_build, c_probe, c_cmp, c_unnest, c_top, stats, out} with the reference's
    meaning of each counter (see the CSV columns at main_experiment1.cc:1288-1333)."""
    kind, bside, bkey, pkey, unique, unnest = EXP1_PLANS[plan]
    build = Rel(R if bside == "R" else S, key_word=bkey)
    probe = Rel(S if bside == "R" else R, key_word=pkey)
    t = table if table is not None else Table(ctx, kind, nb)
    t.build(build)
    r = ctx.probe(t, probe, unique=unique, unnest=unnest, out=out, checksum=checksum)
    if kind == HJ3D_CHAIN:
        c_probe, c_unnest, c_top = r.n_out, 0, r.n_out
    else:
        c_probe, c_unnest, c_top = r.n_matched, (r.n_out if unnest else 0), (r.n_out if unnest else r.n_matched)
    res = {
        "nb": nb, "c_build": build.n, "c_probe": c_probe, "c_cmp": r.n_cmps, "c_unnest": c_unnest,
        "c_top": c_top, "overflow": r.overflow,
        "out": {"n": r.n_out, "sum_a": r.sum_a, "sum_b": r.sum_b, "sum_c": r.sum_c, "sum_h": r.sum_h,
                "xor_h": r.xor_h},
    }
    if stats:
        res["stats"] = t.stats()
    return res


STAT_ADD = ("nb", "empty", "entries", "distinct", "cc0_sum", "cc0_cnt", "cc1_sum", "cc1_cnt")


def merge_shard_stats(parts: list) -> dict:
    """HtStatistics of a table split into disjoint bucket ranges, from the shards' own: counts add,
    extremes take max / min (a shard without a non-empty bucket has no cc1_min), i.e. the
    single-table statistics (the merge dist.allreduce_stats does across ranks)."""
    out = {k: sum(st[k] for st in parts) for k in STAT_ADD}
    out["cc0_max"] = max(st["cc0_max"] for st in parts)
    out["cc1_max"] = max(st["cc1_max"] for st in parts)
    out["cc0_min"] = min(st["cc0_min"] for st in parts)
    mins = [st["cc1_min"] for st in parts if st["cc1_cnt"]]
    out["cc1_min"] = min(mins) if mins else 0
    return out


def exp1_plan_sharded(ctx: Context, plan: str, R, S, nb: int, parts: int, out=None, stats: bool = True,
                      checksum: bool = True, timing: list | None = None, single_pass: bool = False) -> dict:
    """The multi-GPU split of SURVEY §8(e) emulated on ONE device, owner after owner: both
    relations are partitioned into `parts` bucket ranges by the exchange partitioner
    (hj3d_partition, as every rank does before the all-to-all), then for each owner p a table over
    its range [lo, hi) is built from its build pairs and probed with its probe pairs (explicit global
    row ids, as received). This is each rank's compute at its real geometry (bucket_lo != 0,
    |R| / parts buckets), without the exchange; the counters add up to the single-table run's and
    are returned in exp1_plan's form. timing (a list): one dict of per-owner phase times (ms, the
    library's HIP-event timers) is appended per owner, plus {"owner": "partition", ...} first.
    single_pass: the probe side through the single-pass partitioner (hj3d_partition_strided, no
    order inside an owner) with the library's bounded stride (hj3d_partition_stride: ~|probe| pairs
    of send buffer in all), as bench.py's strand does; a spill (an owner above its stride) falls back
    to the stable partitioner."""
    import torch
    from . import (T_BUILD, T_HIST, T_PARTITION, T_PROBE, T_PROBE_KERNEL, T_SCATTER, MASK64, part_range,
                   partition_stride)
    kind, bside, bkey, pkey, unique, unnest = EXP1_PLANS[plan]
    build = Rel(R if bside == "R" else S, key_word=bkey)
    probe = Rel(S if bside == "R" else R, key_word=pkey)
    dev = R.device
    bp = torch.empty((max(build.n, 1), 2), dtype=torch.int32, device=dev)
    stride = partition_stride(probe.n, parts) if single_pass else None
    pp = torch.empty((max(stride * parts if single_pass else probe.n, 1), 2), dtype=torch.int32, device=dev)
    bc = torch.zeros(parts, dtype=torch.int64, device=dev)
    pc = torch.zeros(parts, dtype=torch.int64, device=dev)
    phases = {"build": T_BUILD, "probe": T_PROBE, "part_kernel": T_SCATTER, "split_kernel": T_HIST,
              "probe_kernel": T_PROBE_KERNEL, "partition": T_PARTITION}

    def timers():
        ctx.sync()
        d = {}
        for k, ph in phases.items():
            ms, cnt = ctx.timer(ph)
            if cnt:
                d[k] = ms
        ctx.timer_reset()
        return d
    if timing is not None:
        ctx.timing(True)
        ctx.timer_reset()
    ctx.partition(build, nb, parts, bp, bc)
    tb = timers() if timing is not None else {}
    ctx.partition(probe, nb, parts, pp, pc, stride=stride)
    if single_pass and max(pc.tolist()) > stride:  # spilled: the stable partitioner instead
        single_pass, stride = False, None
        pp = torch.empty((max(probe.n, 1), 2), dtype=torch.int32, device=dev)
        ctx.partition(probe, nb, parts, pp, pc)
    if timing is not None:
        tp = timers()
        timing.append(dict(owner="partition", partition=tb.get("partition", 0.0) + tp.get("partition", 0.0),
                           partition_build=tb.get("partition"), partition_probe=tp.get("partition")))
    bcs = [0] + torch.cumsum(bc, 0).tolist()
    pcs = [0] + torch.cumsum(pc, 0).tolist()
    pstart = [p * stride for p in range(parts)] if single_pass else pcs[:-1]
    tot = {"c_probe": 0, "c_cmp": 0, "c_unnest": 0, "c_top": 0, "n": 0, "sum_a": 0, "sum_b": 0, "sum_c": 0,
           "sum_h": 0, "xor_h": 0, "overflow": False}
    shard_stats = []
    ooff = 0
    for p in range(parts):
        lo, hi = part_range(nb, parts, p)
        t = Table(ctx, kind, nb, lo, hi)
        nbp, npp = bcs[p + 1] - bcs[p], pcs[p + 1] - pcs[p]
        t.reserve(max(nbp, 1))
        t.build(Rel(bp[bcs[p]:bcs[p + 1]], key_word=0, row_word=1, n=nbp))
        o = out[ooff:] if out is not None else None
        r = ctx.probe(t, Rel(pp[pstart[p]:pstart[p] + npp], key_word=0, row_word=1, n=npp), unique=unique, unnest=unnest,
                      out=o, checksum=checksum)
        if kind == HJ3D_CHAIN:
            c_probe, c_unnest, c_top = r.n_out, 0, r.n_out
            ooff += npp
        else:
            c_probe, c_unnest, c_top = r.n_matched, (r.n_out if unnest else 0), (r.n_out if unnest else r.n_matched)
            ooff += r.n_out
        for k, v in (("c_probe", c_probe), ("c_cmp", r.n_cmps), ("c_unnest", c_unnest), ("c_top", c_top),
                     ("n", r.n_out), ("sum_a", r.sum_a), ("sum_b", r.sum_b), ("sum_c", r.sum_c), ("sum_h", r.sum_h)):
            tot[k] = (tot[k] + v) & MASK64
        tot["xor_h"] ^= r.xor_h
        tot["overflow"] = tot["overflow"] or r.overflow
        if stats:
            shard_stats.append(t.stats())
        if timing is not None:
            timing.append(dict(owner=p, bucket_lo=lo, bucket_hi=hi, build_tuples=nbp, probe_tuples=npp, **timers()))
        t.close()
    res = {"nb": nb, "c_build": build.n, "c_probe": tot["c_probe"], "c_cmp": tot["c_cmp"],
           "c_unnest": tot["c_unnest"], "c_top": tot["c_top"], "overflow": tot["overflow"],
           "out": {k: tot[k] for k in ("n", "sum_a", "sum_b", "sum_c", "sum_h", "xor_h")}}
    if stats:
        res["stats"] = merge_shard_stats(shard_stats)
    return res


def num_distinct_sharded(ctx: Context, rel: Rel, domain: int, parts: int) -> int:
    """The distributed #dv pre-pass of SURVEY §8(e) step 1 (hj3d.dist.num_distinct) emulated on ONE
    device: `parts` ranks each hold a contiguous 1/parts of rel and set the bits of their keys in a
    bitmap over [0, domain) (hj3d_key_bitmap); rank r then receives slice r of every rank's bitmap
    (the all-to-all), ORs the `parts` slices and popcounts them (hj3d_bitmap_or_popcount), and the
    per-rank counts add up. Equals the single-device count; NB = #dv(S.a) of the Nrs / NrsNU plans
    (main_experiment1.cc:453-454)."""
    import torch
    words = (domain + 31) // 32
    words = (words + parts - 1) // parts * parts
    dev = rel.tensor.device
    bm = torch.zeros((parts, words), dtype=torch.int32, device=dev)
    outside = torch.zeros(1, dtype=torch.int64, device=dev)
    for r in range(parts):
        lo, hi = rel.n * r // parts, rel.n * (r + 1) // parts
        ctx.key_bitmap(Rel(rel.tensor[lo:hi], key_word=rel.c.key_off // 4), domain, bm[r], outside)
    per = words // parts
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    for r in range(parts):
        ctx.bitmap_or_popcount(bm[:, r * per:(r + 1) * per].contiguous(), cnt)
    ctx.sync()
    if int(outside.item()):
        raise ValueError(f"{int(outside.item())} keys outside [0, {domain})")
    return int(cnt.item())


def exp1_relations_ref(nR: int, nS: int, skew: bool = False, theta: float = 1.0, t: int = 0, device="cuda"):
    """The reference's experiment-1 relations R {k,0,0}, S {i,a,0} (main_experiment1.cc:415-457,
    495-515) from the bit-exact generator (hj3d_gen_exp1_ref), as (n, 3) int32 device tensors:
    the generated columns are uploaded and scattered into the AoS tuples on the device."""
    import torch
    from . import gen_exp1_ref
    Rk, Sa = gen_exp1_ref(nR, nS, skew, theta, t)
    R = torch.zeros((nR, 3), dtype=torch.int32, device=device)
    S = torch.zeros((nS, 3), dtype=torch.int32, device=device)
    R[:, 0] = torch.from_numpy(Rk.view("int32")).to(device)
    S[:, 0] = torch.arange(nS, dtype=torch.int32, device=device)
    S[:, 1] = torch.from_numpy(Sa.view("int32")).to(device)
    return R, S


def exp4_relations_ref(log2R: int, alpha: int, mult_a: int, beta: int, mult_b: int, device="cuda"):
    """The reference's experiment-4 relations R {k,0}, S {k,a}, T {k,a} (main_experiment4.cc:517-575)
    from the bit-exact generator (hj3d_gen_exp4_ref), as (n, 2) int32 device tensors."""
    import torch
    from . import gen_exp4_ref
    Sa, Ta = gen_exp4_ref(log2R, alpha, mult_a, beta, mult_b)
    n, nR = len(Sa), 1 << log2R
    R = torch.zeros((nR, 2), dtype=torch.int32, device=device)
    R[:, 0] = torch.arange(nR, dtype=torch.int32, device=device)
    S = torch.zeros((n, 2), dtype=torch.int32, device=device)
    T = torch.zeros((n, 2), dtype=torch.int32, device=device)
    S[:, 0] = torch.arange(n, dtype=torch.int32, device=device)
    T[:, 0] = S[:, 0]
    S[:, 1] = torch.from_numpy(Sa.view("int32")).to(device)
    T[:, 1] = torch.from_numpy(Ta.view("int32")).to(device)
    return R, S, T


def exp4_plan(ctx: Context, plan: str, R, S, T, nb: int, fused: bool = True) -> dict:
    """Experiment-4 Ndu (nested, deferred unnesting) or Chj (chaining) on {k,a} relations. fused:
    both tables built by one hj3d_build_many call (one launch sequence for two nested tables),
    else one hj3d_build each (main_experiment4.cc:879-881)."""
    kind = HJ3D_NESTED if plan == "Ndu" else HJ3D_CHAIN
    ts, tt = Table(ctx, kind, nb), Table(ctx, kind, nb)
    rs, rt = Rel(S, key_word=1), Rel(T, key_word=1)
    if fused:
        ctx.build_many([ts, tt], [rs, rt])
    else:
        ts.build(rs)
        tt.build(rt)
    r = ctx.probe2(ts, tt, Rel(R, key_word=0))
    return r


EXP4_SUM = ("c_probe_rs", "c_probe_rs_cmp", "c_probe_rt", "c_probe_rt_cmp", "c_unnest_1", "c_unnest_2", "c_top",
            "sum_a", "sum_b", "sum_c", "sum_h")


def merge_exp4(parts: list) -> dict:
    """Experiment-4 counters of disjoint bucket ranges (probe2 results): every counter and row sum
    adds (each R tuple, and every S / T tuple it can meet, lives in exactly one range), the triple
    hash xor-folds."""
    from . import MASK64
    out = {k: sum(r[k] for r in parts) & MASK64 for k in EXP4_SUM}
    x = 0
    for r in parts:
        x ^= r["xor_h"]
    out["xor_h"] = x
    return out


def exp4_plan_sharded(ctx: Context, plan: str, R, S, T, nb: int, parts: int, timing: list | None = None,
                      checksum: bool = True) -> dict:
    """Experiment 4 split as the multi-GPU strand splits it (Ndu co-partitions R, S and T
    on the one FK hash, one exchange), emulated on ONE device owner after owner: R (on R.k), S and T
    (on S.a, T.a) are partitioned into `parts` bucket ranges by the exchange partitioner
    (hj3d_partition: stable, so received pairs keep global row order, which fixes the chaining form's
    chain order); owner p builds its S and T tables over [lo, hi) from its pairs (explicit global rows,
    one hj3d_build_many for both) and runs the two-table probe strand with its R pairs (hj3d_probe2:
    main_experiment4.cc:831-941 Ndu, 943-1043 Chj). The owners' counters add up to the single-device
    run's (merge_exp4). timing: per-owner build / probe ms appended (library timers)."""
    import torch
    from . import T_BUILD, T_PARTITION, T_PROBE, part_range
    kind = HJ3D_NESTED if plan == "Ndu" else HJ3D_CHAIN
    dev = R.device
    rels = [Rel(R, key_word=0), Rel(S, key_word=1), Rel(T, key_word=1)]
    bufs = [torch.empty((max(r.n, 1), 2), dtype=torch.int32, device=dev) for r in rels]
    cnts = torch.zeros((3, parts), dtype=torch.int64, device=dev)
    if timing is not None:
        ctx.timing(True)
        ctx.timer_reset()
    for k in range(3):
        ctx.partition(rels[k], nb, parts, bufs[k], cnts[k])
    cs = [[0] + torch.cumsum(cnts[k], 0).tolist() for k in range(3)]

    def timers():
        ctx.sync()
        d = {}
        for name, ph in (("partition", T_PARTITION), ("build", T_BUILD), ("probe", T_PROBE)):
            ms, cnt = ctx.timer(ph)
            if cnt:
                d[name] = ms
        ctx.timer_reset()
        return d
    if timing is not None:
        timing.append(dict(owner="partition", **timers()))
    res = []
    for p in range(parts):
        lo, hi = part_range(nb, parts, p)
        ts, tt = Table(ctx, kind, nb, lo, hi), Table(ctx, kind, nb, lo, hi)
        own = [Rel(bufs[k][cs[k][p]:cs[k][p + 1]], key_word=0, row_word=1, n=cs[k][p + 1] - cs[k][p]) for k in range(3)]
        ts.reserve(max(own[1].n, 1))
        tt.reserve(max(own[2].n, 1))
        ctx.build_many([ts, tt], [own[1], own[2]])
        res.append(ctx.probe2(ts, tt, own[0], checksum=checksum))
        if timing is not None:
            timing.append(dict(owner=p, bucket_lo=lo, bucket_hi=hi, probe_tuples=own[0].n, build_tuples=own[1].n + own[2].n,
                               **timers()))
        ts.close()
        tt.close()
    return merge_exp4(res)
