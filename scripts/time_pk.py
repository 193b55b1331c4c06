#!/usr/bin/env python3
"""Kernel timing of the packed unique probe (and the chaining build) on device-generated key/FK
relations of a given size, with the library's per-kernel HIP-event timers: for A/B sweeps over
variant builds (HJ3D_LIB) and diagnostic variants (HJ3D_PK_DIAG: results not checked).
Prints one JSON line: mean ms of build, k_pk_part, k_pk_split, k_pk_probe, probe phase."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nR", type=float, default=1e7)
    ap.add_argument("--nS", type=float, default=1e8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-emit", action="store_true")
    ap.add_argument("--layout", default="tuples", choices=["tuples", "pairs", "tuples_rows"],
                    help="probe side: 12-B tuples with implicit rows (config B), received {key, row} pairs "
                         "(8 B, explicit rows: a rank of the multi-GPU strand), or 12-B tuples with an explicit row word")
    ap.add_argument("--chunks", type=int, default=1, help="probe S as this many contiguous chunks (accumulated)")
    ap.add_argument("--label", default=os.path.basename(os.path.dirname(os.environ.get("HJ3D_LIB", "default/x"))))
    a = ap.parse_args()
    import torch
    import hj3d
    nR, nS = int(a.nR), int(a.nS)
    ctx = hj3d.Context(0)
    R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
    S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
    ctx.gen_keys(R, 0, 0, nR, 11)
    ctx.gen_keys(S, 0, 0, 0, 0)
    ctx.gen_fk(S, 1, 0, nR, 12)
    out = None if a.no_emit else torch.empty((nS, 2), dtype=torch.int32, device="cuda")
    t = hj3d.Table(ctx, hj3d.HJ3D_CHAIN, nR)
    t.reserve(nR)
    relR, relS = hj3d.Rel(R, 0), hj3d.Rel(S, 1)
    if a.layout == "pairs":
        P2 = torch.empty((nS, 2), dtype=torch.int32, device="cuda")
        P2[:, 0] = S[:, 1]
        P2[:, 1] = S[:, 0]
        del S
        relS = hj3d.Rel(P2, key_word=0, row_word=1)
    elif a.layout == "tuples_rows":
        relS = hj3d.Rel(S, key_word=1, row_word=0)
    def probe_all():
        if a.chunks <= 1:
            ctx.probe(t, relS, unique=True, out=out, fetch=False)
            return
        assert a.layout == "tuples"
        for c in range(a.chunks):
            lo, hi = nS * c // a.chunks, nS * (c + 1) // a.chunks
            rc = hj3d.Rel(S[lo:hi], 1, row_base=lo)
            ctx.probe(t, rc, unique=True, out=None if out is None else out[lo:hi], fetch=False, accumulate=c > 0)

    for _ in range(3):
        t.build(relR)
        probe_all()
    ctx.sync()
    ctx.timing(True)
    ctx.timer_reset()
    for _ in range(a.reps):
        t.build(relR)
        probe_all()
    ctx.sync()
    res = {"label": a.label, "layout": a.layout, "nR": nR, "nS": nS, "emit": out is not None,
           "chunks": a.chunks}
    for k, ph in (("build", hj3d.T_BUILD), ("probe", hj3d.T_PROBE), ("k_pk_part", hj3d.T_SCATTER),
                  ("k_pk_split", hj3d.T_HIST), ("k_pk_probe", hj3d.T_PROBE_KERNEL)):
        ms, cnt = ctx.timer(ph)
        if cnt:
            res[k] = round(ms / a.reps, 4)  # per step (all chunks)
    r = ctx.probe_result()
    res["n_out"] = r.n_out
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
