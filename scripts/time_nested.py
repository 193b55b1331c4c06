#!/usr/bin/env python3
"""Timing of the nested (3D) table build on a device-generated S.a column (config C: Zipf 0.8 over
1e7 keys, 1e8 tuples; --theta 0 for uniform FKs, the Nrs build of config B), NB = #dv(S.a) as the
reference sizes it. For A/B sweeps over variant builds (HJ3D_LIB) and the diagnostic variants
(HJ3D_NAGG_DIAG: tables not checked). Prints one JSON line: mean build ms (the library's phase
timer), the build path and the table's distinct-key count."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--domain", type=float, default=1e7)
    ap.add_argument("--theta", type=float, default=0.8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--mode", default="agg", choices=["agg", "slices", "sort"])
    ap.add_argument("--opt", action="append", default=[],
                    help="raw engine option K=V (hj3d_ctx_set_option), e.g. for a library of an older revision")
    ap.add_argument("--label", default=os.path.basename(os.path.dirname(os.environ.get("HJ3D_LIB", "default/x"))))
    a = ap.parse_args()
    import torch
    import hj3d
    n, dom = int(a.n), int(a.domain)
    ctx = hj3d.Context(0)
    S = torch.zeros((n, 3), dtype=torch.int32, device="cuda")
    ctx.gen_keys(S, 0, 0, 0, 0)
    if a.theta > 0:
        ctx.gen_zipf(S, 1, 0, dom, a.theta, 13)
    else:
        ctx.gen_fk(S, 1, 0, dom, 13)
    rel = hj3d.Rel(S, 1)
    nb = ctx.num_distinct(rel, dom)
    ctx.nested_sort(a.mode == "sort")
    ctx.nested_pk(a.mode == "slices")
    for kv in a.opt:
        k, v = kv.split("=")
        ctx.set_option(int(k), int(v))
    t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
    t.reserve(n)
    for _ in range(2):
        t.build(rel)
    path = t.build_path()
    ctx.sync()
    ctx.timing(True)
    ctx.timer_reset()
    for _ in range(a.reps):
        t.build(rel)
    ctx.sync()
    ms, cnt = ctx.timer(hj3d.T_BUILD)
    st = t.stats()
    print(json.dumps({"label": a.label, "n": n, "domain": dom, "theta": a.theta, "nb": nb, "mode": a.mode,
                      "path": path, "build": round(ms / cnt, 4), "distinct": st["distinct"]}), flush=True)


if __name__ == "__main__":
    main()
