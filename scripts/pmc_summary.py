#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot kernels from a scripts/gpu_pmc.sh run.

Reads gpurun_out/pmc_<TAG>/p*/run_counter_collection.csv (one counter group per rocprofv3
pass) and writes a JSON summary (default profiles/<TAG>_pmc.json) that bench.py picks up as
`roofline.traffic`.

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): rocprofv3 reports FETCH_SIZE / WRITE_SIZE in
KiB; on gfx950 FETCH_SIZE counts half the bytes of a coalesced streaming read, so it is doubled.
Calibrated in round 5 on known byte counts (micro/micro_fetch.hip, profiles/r05_fetch_calibration.json):
every read the L2 sends to the fabric is a 128-B request (TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ) for
16-, 8- and 4-B streaming loads, 4-B loads at a 12-B stride, and SPARSE 4-B gathers alike (one word per
64-B sector moves the whole 128-B line: twice the sector bytes), while FETCH_SIZE counts 64 B per
request. So 2 x FETCH_SIZE is the read traffic for every access pattern here, and sparse gathers
really move 128 B per touched line. When the request-size passes are present the read bytes are
taken from them directly: 128 RDREQ_128B + 64 RDREQ_64B + 32 RDREQ_32B. Writes: streaming 4- and 8-B
stores go out as 64-B requests (WRITE_SIZE exact); partial lines leave as 32-B requests, so the write
bytes are 64 WRREQ_64B + 32 (WRREQ - WRREQ_64B) when those passes are present. For each kernel only the launches of the largest grid are
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
           "k_rp_scatter", "k_rp_hist", "k_rp_fused", "k_rp_wscatter", "k_rp_build3", "k_rp_build2", "k_rp_build", "k_sort_small_buckets",
           "k_scan_tiles",
           # nested (config C) and experiment-4 (config E) kernels
           "k_nagg_mains", "k_nagg_order", "k_nagg_rebase", "k_nagg_counts", "k_nagg_ps_shift", "k_nagg_pk_ovf",
           "k_nagg_hot", "k_nagg_defer", "k_nagg_reg", "k_nagg", "k_rn_probe_seg", "k_expand_light",
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
        if "TCC_EA0_RDREQ_sum" in d:  # read bytes by request size (calibrated, see the docstring)
            n, n32 = d["TCC_EA0_RDREQ_sum"], d.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            n64, n128 = d.get("TCC_EA0_RDREQ_64B_sum", 0.0), d.get("TCC_EA0_RDREQ_128B_sum", 0.0)
            d["read_bytes_req"] = 128 * n128 + 64 * n64 + 32 * n32 + 64 * max(n - n128 - n64 - n32, 0.0)
        if "TCC_EA0_WRREQ_sum" in d:
            n, n64 = d["TCC_EA0_WRREQ_sum"], d.get("TCC_EA0_WRREQ_64B_sum", 0.0)
            d["write_bytes_req"] = 64 * n64 + 32 * (n - n64)
            d["write_partial_frac"] = (n - n64) / n if n else 0.0
        if "read_bytes_req" in d and "write_bytes_req" in d:
            d["traffic_bytes_per_launch"] = d["read_bytes_req"] + d["write_bytes_req"]
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d["TCC_MISS_sum"], 1)
        if "SQ_INSTS_LDS" in d and "SQ_LDS_BANK_CONFLICT" in d:
            d["lds_conflict_cycles_per_inst"] = d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_INSTS_LDS"], 1)
        if "SQ_WAVE_CYCLES" in d:
            wc = max(d["SQ_WAVE_CYCLES"], 1)
            d["wait_frac"] = d.get("SQ_WAIT_ANY", 0) / wc
            d["issue_stall_frac"] = d.get("SQ_WAIT_INST_ANY", 0) / wc
            d["active_frac"] = d.get("SQ_ACTIVE_INST_ANY", 0) / wc
    # which library the counters were taken on (bench.py prefers the summary of the library it runs)
    import hashlib
    import time
    lib_path = os.environ.get("HJ3D_LIB") or os.path.join(ROOT, "3d-hashjoin_amd", "lib", "libhj3d.so")
    try:
        with open(lib_path, "rb") as fh:
            lib_sha16 = hashlib.sha256(fh.read()).hexdigest()[:16]
    except OSError:
        lib_sha16 = None
    out = {
        "tag": a.tag, "workload": a.workload, "nR": a.nR, "nS": a.nS, "emit": bool(a.emit),
        "lib_sha16": lib_sha16, "collected_unix": int(time.time()),
        "command": "rocprofv3 --pmc <group> --kernel-trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
                   + ("" if a.workload == "B" else f" --workload {a.workload}"),
        "corrections": "FETCH_SIZE, WRITE_SIZE in KiB; FETCH_SIZE x2 (every read request is 128 B, counted as "
                       "64: calibrated for streaming loads and sparse gathers, profiles/r05_fetch_calibration.json); "
                       "traffic from the request-size counters where present (128/64/32-B reads, 64/32-B writes)",
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
