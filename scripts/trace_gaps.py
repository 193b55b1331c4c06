"""One timed step's kernel timeline from a rocprofv3 kernel trace: start offset, duration and the
idle gap before each kernel (us). Usage: trace_gaps.py run_kernel_trace.csv [first-kernel substring] [count]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2] if len(sys.argv) > 2 else "k_rp_"
count = int(sys.argv[3]) if len(sys.argv) > 3 else 16
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
i0 = idx[-3] if len(idx) >= 3 else idx[0]
t0, prev = int(rows[i0]["Start_Timestamp"]), None
for r in rows[i0:i0 + count]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} gap={gap:6.1f} {r['Kernel_Name'][:80]}")
    prev = e
