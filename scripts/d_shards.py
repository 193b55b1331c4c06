#!/usr/bin/env python3
"""Config D's 8-GPU split emulated on ONE GPU: per-rank compute at the real geometry, timed.

The reference relations (|R| = 1e8, |S| = 1e9, hj3d_gen_exp1_ref) are split into `--parts` owner
bucket ranges by the exchange partitioner (hj3d_partition), then each owner in turn builds its
table over [lo, hi) from its build pairs and probes it with its probe pairs (explicit global
rows), as every rank does after the all-to-all (hj3d.exp1_plan_sharded). The counters summed over
the owners are checked against the reference binary's fixture. Prints one JSON line: per owner the
build / probe phase times and the probe kernels' times with their roofline fractions (algorithmic
bytes as bench.py counts them for a received-pair probe side: k_pk_part 8 + 8 B per pair,
k_pk_probe 8 + 8 B per pair + the table slices once), and the exchange partitioner's time.
Per-rank compute, exchange not included: NOT a scaling number.

Usage: python scripts/d_shards.py [--parts 8] [--plan Csr|Nsr|Nrs|NrsNU] [--reps 3] [--nR 1e8 --nS 1e9]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))
PEAK = 8000.0  # GB/s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--plan", default="Csr", choices=["Csr", "Nsr", "Nrs", "NrsNU"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--nR", type=float, default=1e8)
    ap.add_argument("--nS", type=float, default=1e9)
    ap.add_argument("--xpart", default="single", choices=["single", "stable"],
                    help="probe side: single-pass (hj3d_partition_strided) or stable two-pass exchange partitioner")
    a = ap.parse_args()
    import torch
    import hj3d
    nR, nS = int(a.nR), int(a.nS)
    t0 = time.perf_counter()
    # the reference's relations, generated once per box into the relation cache (bench.py's
    # reference_columns_cached: $HJ3D_REL_CACHE or $TMPDIR/hj3d_relcache) and mapped by later runs
    sys.path.insert(0, ROOT)
    from bench import reference_columns_cached
    Rk, Sa = reference_columns_cached(nR, nS, True, lambda: None)
    R = torch.zeros((nR, 3), dtype=torch.int32, device="cuda")
    S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
    import numpy as np
    R[:, 0] = torch.from_numpy(np.ascontiguousarray(Rk).view("int32")).to("cuda")
    S[:, 0] = torch.arange(nS, dtype=torch.int32, device="cuda")
    S[:, 1] = torch.from_numpy(np.ascontiguousarray(Sa).view("int32")).to("cuda")
    del Rk, Sa
    gen_s = time.perf_counter() - t0
    ctx = hj3d.Context(0)
    # NB of the plans built on S.a: #dv(S.a) by the distributed pre-pass (per-rank bitmaps, OR-merge)
    dv = (hj3d.num_distinct_sharded(ctx, hj3d.Rel(S, key_word=1), nR, a.parts)
          if hj3d.EXP1_PLANS[a.plan][1] == "S" else 0)
    nb = hj3d.num_buckets_exp1(a.plan, nR, dv, 1)
    out = torch.empty((nS, 2), dtype=torch.int32, device="cuda") if a.plan in ("Csr", "Nrs") else None
    sp = a.xpart == "single"
    hj3d.exp1_plan_sharded(ctx, a.plan, R, S, nb, a.parts, out=out, stats=False, checksum=False,
                           single_pass=sp)  # warm-up
    runs = []
    for _ in range(a.reps):
        tm = []
        hj3d.exp1_plan_sharded(ctx, a.plan, R, S, nb, a.parts, out=out, stats=False, checksum=False, timing=tm,
                               single_pass=sp)
        runs.append(tm)
    got = hj3d.exp1_plan_sharded(ctx, a.plan, R, S, nb, a.parts, out=out, single_pass=sp)  # verification run
    fx_path = os.path.join(ROOT, "tests", "golden", f"exp1_R{nR}_S{nS}_uni.json")
    verify = None
    if os.path.exists(fx_path):
        ref = json.load(open(fx_path))["plans"].get(a.plan)
        if ref:
            verify = (got["c_cmp"] == ref["c_cmp"] and got["out"] == ref["out"] and got["c_top"] == ref["c_top"] and
                      all(got["stats"][k] == ref["stats"][k] for k in ref["stats"] if k in got["stats"]))

    def avg(owner, key):
        v = [r[i][key] for r in runs for i in range(len(r)) if r[i]["owner"] == owner and key in r[i]]
        return sum(v) / len(v) if v else None
    owners = []
    for p in range(a.parts):
        first = runs[0][p + 1]
        npp, nbp = first["probe_tuples"], first["build_tuples"]
        d = {"owner": p, "bucket_lo": first["bucket_lo"], "bucket_hi": first["bucket_hi"],
             "build_tuples": nbp, "probe_tuples": npp}
        for k in ("build", "probe", "part_kernel", "split_kernel", "probe_kernel"):
            d[k + "_ms"] = avg(p, k)
        if a.plan == "Csr":
            nbl = first["bucket_hi"] - first["bucket_lo"]
            d["slices"] = ctx.pk_plan(nbl, nbp)
            alg = {"part_kernel": npp * 16, "split_kernel": npp * 16, "probe_kernel": npp * 16 + nbp * 8 + nbl * 4}
            for k, b in alg.items():
                ms = d[k + "_ms"]
                if ms:
                    d[k + "_frac"] = b / (ms * 1e-3) / 1e9 / PEAK
            d["probe_phase_frac"] = (npp * (16 + 8)) / (d["probe_ms"] * 1e-3) / 1e9 / PEAK
        owners.append(d)
    part_ms = avg("partition", "partition")
    pb_ms, pp_ms = avg("partition", "partition_build"), avg("partition", "partition_probe")
    # the plan's sides (Csr / Nsr build on R and probe S; Crs / Nrs / NrsNU build on S.a and probe R)
    # and the partitioners' algorithmic bytes per tuple: the stable two-pass hj3d_partition reads the
    # 12-B tuple twice and writes the 8-B pair (32 B), the single-pass strided one reads once (20 B)
    n_build, n_probe = (nR, nS) if hj3d.EXP1_PLANS[a.plan][1] == "R" else (nS, nR)
    bpt_build, bpt_probe = 32, (20 if sp else 32)
    line = {
        "what": f"config D {a.parts}-owner split emulated on one GPU, plan {a.plan}: per-rank compute at the "
                f"{a.parts}-GPU geometry, owners run one after another; exchange (xGMI) NOT included; not a "
                "scaling number",
        "nR": nR, "nS": nS, "num_buckets": nb, "num_dv_Sa": dv or None, "reps": a.reps, "input_generation_s": gen_s,
        "exchange_partition_ms_both_relations": part_ms,
        "build_side_tuples": n_build, "probe_side_tuples": n_probe,
        "exchange_partition_bytes_per_tuple": {"build": bpt_build, "probe": bpt_probe},
        "exchange_partition_frac": ((n_build * bpt_build + n_probe * bpt_probe) / (part_ms * 1e-3) / 1e9 / PEAK
                                    if part_ms else None),
        "exchange_partitioner_probe_side": ("single-pass hj3d_partition_strided" if sp else
                                            "stable two-pass hj3d_partition"),
        "exchange_partition_build_ms": pb_ms,
        "exchange_partition_probe_ms": pp_ms,
        "exchange_partition_build_frac": (n_build * bpt_build) / (pb_ms * 1e-3) / 1e9 / PEAK if pb_ms else None,
        "exchange_partition_probe_frac": (n_probe * bpt_probe) / (pp_ms * 1e-3) / 1e9 / PEAK if pp_ms else None,
        "owners": owners,
        "max_owner_probe_ms": max(o["probe_ms"] for o in owners),
        "max_owner_build_ms": max(o["build_ms"] for o in owners),
        "counters": {"c_cmp": got["c_cmp"], "c_top": got["c_top"]},
        "verified_against_reference_fixture": verify,
    }
    print(json.dumps(line))
    if verify is False:
        sys.exit("verification failed")


if __name__ == "__main__":
    main()
