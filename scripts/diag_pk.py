#!/usr/bin/env python3
"""Diagnostic: packed probe geometries at large probe sizes, checked by the key/FK identity
(every S tuple matches exactly once; sampled pairs join)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))
import torch
import hj3d

ctx = hj3d.Context(0)
ctx.timing(True)


def run(nR, nS, w=0, stage=0, label="", emit=True, ck=False, ref=False):
    if ref:
        R, S = hj3d.exp1_relations_ref(nR, nS)
    else:
        R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
        S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
        ctx.gen_keys(R, 0, 0, nR, 11)
        ctx.gen_keys(S, 0, 0, 0, 0)
        ctx.gen_fk(S, 1, 0, nR, 12)
    t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nR)
    t.build(hj3d.Rel(R, 0))
    ctx.pk_slice_max(w)
    ctx.pk_stage(stage)
    out = torch.full((nS, 2), -1, dtype=torch.int32, device="cuda")
    for step in range(2):
        ctx.timer_reset()
        r = ctx.probe(t, hj3d.Rel(S, 1), unique=True, out=out if emit else None, checksum=ck)
        ctx.sync()
        tm = {k: ctx.timer(ph) for k, ph in (("part", hj3d.T_SCATTER), ("split", hj3d.T_HIST), ("probe", hj3d.T_PROBE_KERNEL))}
    unmatched = int((out[:, 1] == -1).sum()) if emit else -1
    idx = torch.randint(0, nS, (1 << 16,), device="cuda")
    smp = out[idx].long()
    ok = bool(torch.equal(S[smp[:, 0], 1], R[smp[:, 1], 0])) if unmatched == 0 else False
    print("  res", r.n_out, r.n_matched, r.n_cmps, r.sum_h, r.xor_h)
    print(f"{label} nR={nR} nS={nS} w={w} stage={stage} plan={ctx.pk_plan(nR, nR)} n_out={r.n_out} "
          f"matched={r.n_matched} unmatched_slots={unmatched} pairs_ok={ok} "
          f"ms={ {k: round(v[0] / max(v[1], 1), 3) for k, v in tm.items()} }", flush=True)
    ctx.pk_slice_max(0)
    ctx.pk_stage(0)
    del R, S, out, t
    torch.cuda.empty_cache()


which = sys.argv[1] if len(sys.argv) > 1 else "all"
if which == "mode0":
    run(100_000_000, 1_000_000_000, label="D mode0 ck", emit=False, ck=True)
    run(100_000_000, 1_000_000_000, label="D ref emit ck", emit=True, ck=True, ref=True)
    run(100_000_000, 1_000_000_000, label="D ref mode0 ck", emit=False, ck=True, ref=True)
    sys.exit(0)
run(10_000_000, 100_000_000, label="B")
run(12_500_000, 125_000_000, label="D/8")
run(25_000_000, 250_000_000, label="D/4")
run(10_000_000, 100_000_000, w=2048, label="B two-level C=5")
run(10_000_000, 300_000_000, w=2048, label="B two-level multi-tile")
run(10_000_000, 300_000_000, w=0, label="B single-level 3x")
run(100_000_000, 200_000_000, label="D table, 2e8 probes")
run(100_000_000, 1_000_000_000, label="D")
