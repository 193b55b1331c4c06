#!/usr/bin/env python3
"""Per-partition phase clocks of the nested aggregation kernel (k_nagg), from a library built with
-DHJ3D_NAGG_CLK=1 (HJ3D_LIB=.../variants/clk/libhj3d.so): where a workgroup's time goes (table
clear, pass A, main records, pass B) and how the partitions' start times spread over the launch.

--workload E: config E's two tables in one build_many (1024 partitions of 3072 buckets);
--workload C: one table over 1e8 Zipf-0.8 keys (config C's build); --workload D: 1e9 uniform keys over
1e8 (config D's Nrs build, on the packed slices: 65,104 partitions). Prints one JSON object: the
median / p90 microseconds of every phase over the partitions, the launch span, and the workgroups'
start-time deciles."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="E", choices=["C", "D", "E"])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import hj3d

    dev = torch.device("cuda", 0)
    ctx = hj3d.Context(0)
    if a.workload == "E":
        log2R = 22
        nR = 1 << log2R
        R, S, T = hj3d.exp4_relations_ref(log2R, 3, 4, 2, 2, device=dev)
        nb = (nR >> 3) + (nR >> 2)
        ts, tt = hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb), hj3d.Table(ctx, hj3d.HJ3D_NESTED, nb)
        ts.reserve(S.shape[0])
        tt.reserve(T.shape[0])
        relS, relT = hj3d.Rel(S, key_word=1), hj3d.Rel(T, key_word=1)

        def build():
            ctx.build_many([ts, tt], [relS, relT])
            return ts
    elif a.workload == "D":  # config D's Nrs build shape: 1e9 uniform FKs over 1e8 keys (device generator)
        S = torch.zeros((1_000_000_000, 3), dtype=torch.int32, device=dev)
        ctx.gen_keys(S, 0, 0, 0, 0)
        ctx.gen_fk(S, 1, 0, 100_000_000, 13)
        relS = hj3d.Rel(S, key_word=1)
        dv = ctx.num_distinct(relS, 100_000_000)
        t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, dv)
        t.reserve(S.shape[0])

        def build():
            t.build(relS)
            return t
    else:
        R, S = hj3d.exp1_relations_ref(10_000_000, 100_000_000, True, 0.8, 0, device=dev)
        relS = hj3d.Rel(S, key_word=1)
        dv = ctx.num_distinct(relS, 10_000_000)
        t = hj3d.Table(ctx, hj3d.HJ3D_NESTED, dv)
        t.reserve(S.shape[0])

        def build():
            t.build(relS)
            return t
    for _ in range(a.reps):
        tb = build()
    torch.cuda.synchronize()
    path = tb.build_path()
    parts = 16384
    buf = (C.c_uint64 * (parts * 8))()
    st = hj3d.lib().hj3d_diag_nagg_clk(buf, parts)
    if st != 0:
        raise SystemExit(f"hj3d_diag_nagg_clk: status {st} (library without HJ3D_NAGG_CLK?)")
    x = np.frombuffer(buf, dtype=np.uint64).reshape(parts, 8).astype(np.int64)
    x = x[x[:, 0] > 0]
    t0 = x[:, 0].min()
    us = lambda v: v * 0.01  # 100 MHz ticks -> microseconds
    out = {"workload": a.workload, "path": path, "partitions": int(len(x)), "span_us": round(us(x[:, 5].max() - t0), 1)}
    names = ["clear", "pass_A", "mains", "pass_B", "tail"]
    for k, nm in enumerate(names):
        d = us(x[:, k + 1] - x[:, k])
        out[nm] = {"median": round(float(np.median(d)), 2), "p90": round(float(np.percentile(d, 90)), 2),
                   "max": round(float(d.max()), 2)}
    tot = us(x[:, 5] - x[:, 0])
    out["workgroup_total"] = {"median": round(float(np.median(tot)), 2), "p90": round(float(np.percentile(tot, 90)), 2),
                              "max": round(float(tot.max()), 2)}
    starts = us(x[:, 0] - t0)
    out["start_deciles_us"] = [round(float(np.percentile(starts, q)), 1) for q in range(0, 101, 10)]
    ends = us(np.maximum(x[:, 5], x[:, 7]) - t0)
    out["end_deciles_us"] = [round(float(np.percentile(ends, q)), 1) for q in range(0, 101, 10)]
    # the longest workgroups (heavy partitions): start, total and pass times (last round), us
    top = np.argsort(-tot)[:8]
    out["longest"] = [{"start": round(float(starts[i]), 1), "total": round(float(tot[i]), 1),
                       "pass_A": round(float(us(x[i, 2] - x[i, 1])), 1), "pass_B": round(float(us(x[i, 4] - x[i, 3])), 1)}
                      for i in top]
    # point 7: the end of pass B's sweep (before the image write-out), or with the look-back finish the
    # finish's end
    if ((x[:, 7] >= x[:, 3]) & (x[:, 7] <= x[:, 4])).all():
        for nm, d in (("pass_B_sweep", us(x[:, 7] - x[:, 3])), ("pass_B_writeout", us(x[:, 4] - x[:, 7]))):
            out[nm] = {"median": round(float(np.median(d)), 2), "p90": round(float(np.percentile(d, 90)), 2),
                       "max": round(float(d.max()), 2)}
        # the first-started half against the rest
        first = x[:, 0] <= np.percentile(x[:, 0], 40)
        out["pass_B_sweep_first_vs_rest"] = [round(float(np.median(us(x[first, 7] - x[first, 3]))), 2),
                                              round(float(np.median(us(x[~first, 7] - x[~first, 3]))), 2)]
        out["pass_B_writeout_first_vs_rest"] = [round(float(np.median(us(x[first, 4] - x[first, 7]))), 2),
                                                 round(float(np.median(us(x[~first, 4] - x[~first, 7]))), 2)]
        out["pass_A_first_vs_rest"] = [round(float(np.median(us(x[first, 2] - x[first, 1]))), 2),
                                       round(float(np.median(us(x[~first, 2] - x[~first, 1]))), 2)]
    if (x[:, 7] > x[:, 5]).all():
        fin = us(x[:, 7] - x[:, 5])
        out["finish"] = {"median": round(float(np.median(fin)), 2), "p90": round(float(np.percentile(fin, 90)), 2),
                         "max": round(float(fin.max()), 2)}
    # workgroups running at once on one CU (point 6: XCC_ID << 32 | HW_ID; CU_ID bits 8-11, SH 12,
    # SE 13-15): the largest overlap of [start, exit] intervals per CU, and the CUs seen
    hw = x[:, 6].astype(np.uint64)
    cu = ((hw >> np.uint64(32)) & np.uint64(0xF)) * np.uint64(1 << 8) + ((hw >> np.uint64(8)) & np.uint64(0xFF))
    occ = {}
    for c in np.unique(cu):
        idx = np.where(cu == c)[0]
        ev = sorted([(x[i, 0], 1) for i in idx] + [(max(x[i, 5], x[i, 7]), -1) for i in idx], key=lambda t: (t[0], t[1]))
        cur = best = 0
        for _, d in ev:
            cur += d
            best = max(best, cur)
        occ[best] = occ.get(best, 0) + 1
    out["cus_seen"] = int(len(np.unique(cu)))
    out["max_concurrent_per_cu_hist"] = {str(k): v for k, v in sorted(occ.items())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
