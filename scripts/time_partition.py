#!/usr/bin/env python3
"""Times the probe side's exchange partitioner (hj3d_partition_strided, k_xpart) on its own, for
same-box A/B of variant builds (HJ3D_LIB, scripts/build_variants.sh + scripts/gpu_ab.sh style).

Input: |S| tuples {k, a, 0} on the device, S.a uniform over [0, |R|) (hj3d_gen_fk), partitioned
into `--parts` bucket ranges of |R| buckets with the library's bounded stride. Prints one JSON line:
the mean kernel time over `--reps` calls (the library's T_PARTITION HIP-event timer), the rate
against 20 B per tuple (12-B tuple read + 8-B pair written) and whether the counts add up.

usage: python scripts/time_partition.py [--nS 1e9] [--nR 1e8] [--parts 8] [--reps 10] [--label x]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-hashjoin_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nS", type=float, default=1e9)
    ap.add_argument("--nR", type=float, default=1e8)
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--label", default=os.path.basename(os.path.dirname(os.environ.get("HJ3D_LIB", "default/x"))))
    a = ap.parse_args()
    import torch
    import hj3d
    nS, nR = int(a.nS), int(a.nR)
    ctx = hj3d.Context(0)
    S = torch.zeros((nS, 3), dtype=torch.int32, device="cuda")
    ctx.gen_keys(S, 0, 0, 0, 0)
    ctx.gen_fk(S, 1, 0, nR, 0x5eed0002)
    rel = hj3d.Rel(S, key_word=1)
    stride = hj3d.partition_stride(nS, a.parts)
    out = torch.empty((a.parts * stride, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(a.parts, dtype=torch.int64, device="cuda")
    ctx.partition(rel, nR, a.parts, out, cnt, stride=stride)  # warm-up
    ctx.sync()
    ctx.timing(True)
    ctx.timer_reset()
    for _ in range(a.reps):
        ctx.partition(rel, nR, a.parts, out, cnt, stride=stride)
    ms, n = ctx.timer(hj3d.T_PARTITION)
    c = cnt.tolist()
    avg = ms / n
    print(json.dumps({"label": a.label, "nS": nS, "parts": a.parts, "stride": stride, "ms": avg,
                      "GBs_alg": nS * 20 / (avg * 1e-3) / 1e9, "frac_8TBs": nS * 20 / (avg * 1e-3) / 8e12,
                      "counts_ok": sum(c) == nS and max(c) <= stride}), flush=True)


if __name__ == "__main__":
    main()
