#!/usr/bin/env python3
"""Per (kernel, grid) durations from a rocprofv3 kernel_trace.csv: where each launch shape spends time."""
import collections
import csv
import re
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    n = re.sub(r"\(.*$", "", n).replace("hj3d::", "").replace("void ", "")
    d[(n[:48], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:48s} blocks={g:>8d} n={len(v):3d} avg={sum(v) / len(v):8.1f}us total={sum(v) / 1e3:7.2f}ms")
