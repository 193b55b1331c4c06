"""Selection pushdown at config-B size on one GPU: hj3d_select over S (1e8 x {k, a, b}) with
predicate S.b < x at several selectivities, and the selected probe strand (scan -> selection ->
probe -> count, Csr table on R = 1e7 keys) select-first and fused (hj3d_probe_sel: the predicate
evaluated in the probe partitioner) against the unselected probe. Prints one JSON line.
Algorithmic bytes of the selection: 12 B/tuple read + 8 B per passing tuple written.
usage: python scripts/time_select.py [--reps N]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))
import torch  # noqa: E402
import hj3d  # noqa: E402

reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 10
nR, nS = 10_000_000, 100_000_000
ctx = hj3d.Context(0)
R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
ctx.gen_keys(R, 0, 0, nR, 11)
ctx.gen_keys(S, 0, 0, 0, 0)
ctx.gen_fk(S, 1, 0, nR, 7)
ctx.gen_fk(S, 2, 0, 100, 5)  # S.b ~ U[0, 100): selectivity x / 100
tab = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nR)
tab.reserve(nR)
tab.build(hj3d.Rel(R, 0))
pairs = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
out = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
srel = hj3d.Rel(S, 1)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {"n": nS, "reps": reps, "runs": []}
base_probe = timed(lambda: ctx.probe(tab, srel, unique=True, out=out, fetch=False, checksum=False))
full = ctx.probe(tab, srel, unique=True, out=out)
res["probe_unselected_ms"] = base_probe
for x in (10, 50, 100):
    preds = [(2, "<", x)]
    ms = timed(lambda: ctx.select(srel, preds, pairs, cnt, fetch=False))
    _, sel, n_sel = ctx.select(srel, preds, pairs, cnt)
    pm = timed(lambda: ctx.probe(tab, sel, unique=True, out=out, fetch=False, checksum=False))
    r = ctx.probe(tab, sel, unique=True, out=out)
    fused_ms = timed(lambda: ctx.probe_sel(tab, srel, preds, unique=True, out=out, fetch=False, checksum=False))
    rf = ctx.probe_sel(tab, srel, preds, unique=True, out=out)
    assert (rf.n_probe, rf.n_out, rf.n_cmps) == (n_sel, r.n_out, r.n_cmps)
    alg = 12 * nS + 8 * n_sel
    res["runs"].append({"pred": f"S.b < {x}", "selected": n_sel, "select_ms": ms,
                        "select_GBs": alg / ms / 1e6, "select_frac_of_8TBs": alg / ms / 1e6 / 8000.0,
                        "probe_selected_ms": pm, "strand_ms": ms + pm,
                        "strand_probe_tuples_per_s": nS / ((ms + pm) * 1e-3), "matches": r.n_out,
                        "fused_strand_ms": fused_ms, "fused_scan_tuples_per_s": nS / (fused_ms * 1e-3)})
    assert r.n_out == n_sel, "key/FK join: every selected S tuple has one partner"
print(json.dumps(res))
