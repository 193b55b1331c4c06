#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv compactly: kernel name (namespaces stripped), calls, avg, share."""
import csv
import re
import sys

for f in sys.argv[1:]:
    print(f)
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
        n = re.sub(r"\(.*$", "", n).replace("hj3d::", "")
        print(f"  {n[:60]:60s} calls={r['Calls']:>5s} avg={float(r['AverageNs']) / 1e3:9.1f}us pct={float(r['Percentage']):5.1f}")
