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


def exp4_plan(ctx: Context, plan: str, R, S, T, nb: int) -> dict:
    """Experiment-4 Ndu (nested, deferred unnesting) or Chj (chaining) on {k,a} relations."""
    kind = HJ3D_NESTED if plan == "Ndu" else HJ3D_CHAIN
    ts, tt = Table(ctx, kind, nb), Table(ctx, kind, nb)
    ts.build(Rel(S, key_word=1))
    tt.build(Rel(T, key_word=1))
    r = ctx.probe2(ts, tt, Rel(R, key_word=0))
    return r
