#!/usr/bin/env python3
"""HBM bytes per probe tuple of the config-D 8-owner split (scripts/d_shards.py) from two rocprofv3
PMC passes (FETCH_SIZE, WRITE_SIZE) over one d_shards.py run.

Reads gpurun_out/pmc_<TAG>/p*/run_counter_collection.csv, sums every dispatch's bytes per kernel
(FETCH_SIZE x2 and KiB -> bytes, the gfx950 corrections of MI355X_MICROARCH.md, as
scripts/pmc_summary.py applies them), divides by the number of strand executions in the run
(--runs: d_shards.py's warm-up + reps + verification run) and by |S|, and writes JSON with the
bytes per probe tuple of each kernel and of the probe strand (exchange partitioner of the probe
side, the owners' k_pk_part on received pairs, k_pk_probe).

usage: python scripts/pmc_bytes.py TAG --runs 3 [--nS 1e9] [--out profiles/TAG_D_shards_pmc.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE_STRAND = ("k_xpart", "k_pk_part", "k_pk_split", "k_pk_probe", "k_probe_ovf")


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--nS", type=float, default=1e9)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"pmc_{a.tag}")
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.Counter()
    for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if k is None:
                    continue
                c = r["Counter_Name"]
                v = float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
                tot[k][c] += v
                if c == "FETCH_SIZE":
                    launches[k] += 1
    nS = a.nS * a.runs
    kern = {}
    for k, d in sorted(tot.items()):
        f, w = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
        kern[k] = {"launches": launches[k], "fetch_bytes_per_probe_tuple": f / nS,
                   "write_bytes_per_probe_tuple": w / nS, "bytes_per_probe_tuple": (f + w) / nS}
    strand = sum(kern[k]["bytes_per_probe_tuple"] for k in PROBE_STRAND if k in kern)
    out = {"tag": a.tag, "runs": a.runs, "nS": a.nS,
           "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace -- python3 scripts/d_shards.py --reps 1",
           "corrections": "FETCH_SIZE, WRITE_SIZE in KiB; FETCH_SIZE x2 (gfx950 streaming-read undercount)",
           "probe_strand_kernels": [k for k in PROBE_STRAND if k in kern],
           "probe_strand_bytes_per_probe_tuple": strand,
           "note": "one GPU, owners one after another: no receive write (the exchange is not run); "
                   "algorithmic 12 + 8 (exchange partition) + 8 + 8 (k_pk_part) + 8 + 8 (probe) = 52 B, "
                   "+ 8 B received write on N GPUs",
           "kernels": kern}
    dst = a.out or os.path.join(ROOT, "profiles", f"{a.tag}_D_shards_pmc.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, d in kern.items():
        print(f"{k:18s} launches={d['launches']:>5d} B/probe tuple={d['bytes_per_probe_tuple']:.2f}")
    print(f"probe strand: {strand:.2f} B per probe tuple; wrote {dst}")


if __name__ == "__main__":
    main()
