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


def exp4_plan(ctx: Context, plan: str, R, S, T, nb: int) -> dict:
    """Experiment-4 Ndu (nested, deferred unnesting) or Chj (chaining) on {k,a} relations."""
    kind = HJ3D_NESTED if plan == "Ndu" else HJ3D_CHAIN
    ts, tt = Table(ctx, kind, nb), Table(ctx, kind, nb)
    ts.build(Rel(S, key_word=1))
    tt.build(Rel(T, key_word=1))
    r = ctx.probe2(ts, tt, Rel(R, key_word=0))
    return r
