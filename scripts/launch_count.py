#!/usr/bin/env python3
"""Launches per step from a rocprofv3 --kernel-trace run of bench.py (config E's verdict item:
"report launches per step").

Reads <dir>/run_kernel_trace.csv (every dispatch, in order) and cuts it into steps at each dispatch
of the build's first kernel (k_rp_hist: the partition pass that opens every nested build). Per step it
counts the dispatches up to the build's last kernel (k_nagg_mains) as the build, and the rest up to
the next step as the probe strand; runtime fills / copies (__amd_rocclr_*) are counted apart. The
median step is reported.

usage: python scripts/launch_count.py gpurun_out/prof/<name> [--first k_rp_hist] [--last k_nagg_mains]
"""
import argparse
import csv
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--first", default="k_rp_hist")
    ap.add_argument("--last", default="k_nagg_mains")
    a = ap.parse_args()
    f = os.path.join(a.dir, "run_kernel_trace.csv")
    with open(f) as fh:
        rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    starts = [i for i, n in enumerate(names) if a.first in n]
    steps = []
    for k, i0 in enumerate(starts):
        i1 = starts[k + 1] if k + 1 < len(starts) else len(names)
        seg = names[i0:i1]
        last = max((j for j, n in enumerate(seg) if a.last in n), default=len(seg) - 1)
        build, probe = seg[:last + 1], seg[last + 1:]
        rt = lambda xs: sum(1 for n in xs if n.startswith("__amd_rocclr"))
        steps.append({"build_kernels": len(build) - rt(build), "build_runtime_ops": rt(build),
                      "probe_kernels": len(probe) - rt(probe), "probe_runtime_ops": rt(probe),
                      "build_names": [n.split("(")[0].split("::")[-1] for n in build]})
    if not steps:
        raise SystemExit("no step found")
    med = {k: statistics.median(s[k] for s in steps) for k in steps[0] if k != "build_names"}
    print(json.dumps({"steps": len(steps), "median": med, "build_names_of_a_step": steps[len(steps) // 2]["build_names"]},
                     indent=1))


if __name__ == "__main__":
    main()
