#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot kernels from a scripts/gpu_pmc.sh run.

Reads gpurun_out/pmc_<TAG>/p*/run_counter_collection.csv (one counter group per rocprofv3
pass) and writes a JSON summary (default profiles/<TAG>_pmc.json) that bench.py picks up as
`roofline.traffic`.

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): rocprofv3 reports FETCH_SIZE / WRITE_SIZE in
KiB; on gfx950 FETCH_SIZE counts half the bytes of a coalesced streaming read, so it is doubled.
WRITE_SIZE is taken as reported (exact for 16-B/lane streaming stores; our 8-B/lane stores are
uncalibrated, noted in the output). For each kernel only the launches of the largest grid are
kept (the probe side S, not the build side R) and the median over those launches is reported.
Of several template instantiations of one kernel the one LAUNCHED MOST OFTEN is reported under the
plain name: that is the one the timed steps run (a checksum-folding verification launch runs
once); the others stay under `instantiations`.

usage: python scripts/pmc_summary.py TAG [--nR 10000000 --nS 100000000 --emit 1]
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# longer names first: a name is matched as a substring of the mangled kernel name
KERNELS = ("k_pk_probe", "k_pk_part", "k_pk_build", "k_rp_probe_seg", "k_rp_part1", "k_probe_ovf", "k_rp_probe",
           "k_rp_scatter", "k_rp_hist", "k_rp_build3", "k_rp_build2", "k_rp_build", "k_sort_small_buckets",
           "k_scan_tiles",
           # nested (config C) and experiment-4 (config E) kernels
           "k_nagg_mains", "k_nagg_order", "k_nagg_rebase", "k_nagg_counts", "k_nagg_ps_shift", "k_nagg_pk_ovf",
           "k_nagg", "k_rn_probe_seg", "k_expand_light",
           "k_expand_heavy_flat", "k_heavy_offsets", "k_ndu_seg", "k_ndu_heavy", "k_ndu", "k_rs_scatter", "k_rs_hist",
           "k_pk_split", "k_xpart", "k_dv_part", "k_dv_bits", "k_dv_merge")


def short(name):
    for k in KERNELS:
        if k in name:
            # template instantiations of one kernel are kept apart (e.g. the LDS-slice and the
            # L2-slice k_rp_probe_seg); the heaviest is reported under the plain name below
            i = name.find(k) + len(k)
            return k + (name[i:name.find(">", i) + 1] if i < len(name) and name[i] == "<" else "")
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--nR", type=int, default=10_000_000)
    ap.add_argument("--nS", type=int, default=100_000_000)
    ap.add_argument("--emit", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--workload", default="B", help="bench.py --workload of the profiled run (B, C, E)")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"pmc_{a.tag}")
    # (kernel, counter) -> list of (grid, value) over dispatches
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if k is None:
                    continue
                vals[(k, r["Counter_Name"])].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    per = {}
    for (k, c), lst in vals.items():
        gmax = max(g for g, _ in lst)
        sel = [x for g, x in lst if g == gmax]
        d = per.setdefault(k, {"grid_size": gmax, "launches": 0})
        d[c] = statistics.median(sel)
        d["launches"] = max(d["launches"], len(sel))
    # one entry per kernel name: the instantiation launched most often (the timed one)
    kern, inst = {}, collections.defaultdict(dict)
    for k, d in per.items():
        base = k.split("<")[0]
        inst[base][k] = {"launches": d["launches"], "grid_size": d["grid_size"]}
        if base not in kern or d["launches"] > kern[base]["launches"]:
            kern[base] = dict(d, instantiation=k)
    for base, d in kern.items():
        if len(inst[base]) > 1:
            d["instantiations"] = inst[base]
    for k, d in kern.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["fetch_bytes"] = d["FETCH_SIZE"] * 1024 * 2
            d["write_bytes"] = d["WRITE_SIZE"] * 1024
            d["traffic_bytes_per_launch"] = d["fetch_bytes"] + d["write_bytes"]
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d["TCC_MISS_sum"], 1)
        if "SQ_INSTS_LDS" in d and "SQ_LDS_BANK_CONFLICT" in d:
            d["lds_conflict_cycles_per_inst"] = d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_INSTS_LDS"], 1)
        if "SQ_WAVE_CYCLES" in d:
            wc = max(d["SQ_WAVE_CYCLES"], 1)
            d["wait_frac"] = d.get("SQ_WAIT_ANY", 0) / wc
            d["issue_stall_frac"] = d.get("SQ_WAIT_INST_ANY", 0) / wc
            d["active_frac"] = d.get("SQ_ACTIVE_INST_ANY", 0) / wc
    out = {
        "tag": a.tag, "workload": a.workload, "nR": a.nR, "nS": a.nS, "emit": bool(a.emit),
        "command": "rocprofv3 --pmc <group> --kernel-trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
                   + ("" if a.workload == "B" else f" --workload {a.workload}"),
        "corrections": "FETCH_SIZE, WRITE_SIZE in KiB; FETCH_SIZE x2 (gfx950 streaming-read undercount); "
                       "WRITE_SIZE as reported (8-B/lane stores uncalibrated)",
        "kernels": kern,
    }
    dst = a.out or os.path.join(ROOT, "profiles", f"{a.tag}_pmc.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, d in sorted(kern.items()):
        t = d.get("traffic_bytes_per_launch")
        print(f"{k:22s} grid={d['grid_size']:>9d} traffic={t/1e9 if t else float('nan'):.3f} GB "
              f"l2hit={d.get('l2_hit_rate', float('nan')):.2f} ldsconf={d.get('lds_conflict_cycles_per_inst', float('nan')):.2f}")
    print("wrote", dst)


if __name__ == "__main__":
    main()
