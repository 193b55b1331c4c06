"""Write experiment-1 relations to hj3d relation files (hj3d.relfile), once, for later runs.

  --gen reference : the reference's own sequential generator (oracle restatement, bit-exact with
                    main_experiment1.cc:415-457; minutes at 1e9 tuples, done once)
  --gen device    : the parallel device generators (hj3d_gen_keys / hj3d_gen_fk / hj3d_gen_zipf;
                    seconds, not the reference's values)

usage: python scripts/make_relations.py OUTDIR --nR 10000000 --nS 100000000 [--zipf 0.8] [--gen device]
Writes OUTDIR/R.rel ({k, a, b}, key word 0) and OUTDIR/S.rel ({k, a, b}, key word 1)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))
from hj3d import relfile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--nR", type=int, default=10_000_000)
    ap.add_argument("--nS", type=int, default=100_000_000)
    ap.add_argument("--zipf", type=float, default=None, help="S.a ~ Zipf(theta) instead of uniform")
    ap.add_argument("--gen", choices=("reference", "device"), default="reference")
    a = ap.parse_args()
    os.makedirs(a.outdir, exist_ok=True)
    meta = {"exp": 1, "nR": a.nR, "nS": a.nS, "zipf": a.zipf, "gen": a.gen}
    if a.gen == "reference":
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # the bit-exact restatement of the reference generator
        Rk, Sa, _ = O.gen_exp1(a.nR, a.nS, a.zipf is not None, a.zipf or 0.0, 0)
        R = O.tuples3(Rk, np.zeros_like(Rk))
        S = O.tuples3(np.arange(a.nS, dtype=np.uint32), Sa)
    else:
        import torch
        import hj3d
        ctx = hj3d.Context(0)
        Rt = torch.zeros((a.nR, 3), dtype=torch.int32, device="cuda")
        St = torch.zeros((a.nS, 3), dtype=torch.int32, device="cuda")
        ctx.gen_keys(Rt, 0, 0, a.nR, 11)
        ctx.gen_keys(St, 0, 0, 0, 0)
        if a.zipf is None:
            ctx.gen_fk(St, 1, 0, a.nR, 7)
        else:
            ctx.gen_zipf(St, 1, 0, a.nR, a.zipf, 7)
        ctx.sync()
        R, S = Rt.cpu().numpy().view(np.uint32), St.cpu().numpy().view(np.uint32)
    for name, rel, kw in (("R", R, 0), ("S", S, 1)):
        h = relfile.save(os.path.join(a.outdir, f"{name}.rel"), rel, kw, meta)
        print(name, h["n"], "rows, checksum", h["checksum"])


if __name__ == "__main__":
    main()
