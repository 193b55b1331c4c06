#!/usr/bin/env python3
"""Fixture for the selection operators (AlgSelection / AlgDynSelection, algebra.hh:278-358) from
the REAL reference: runs oracle/_ref/main_algebra_example.out (built by `make -C oracle ref` from
/root/reference/main_algebra_example.cc) and records, per plan, the relations it prints, the output
tuples it prints (values only; pointers dropped) and every operator count.

The four plans: test0 scan -> selection(L.b < 40) -> top; test1 + nested join probe on R.c = L.a;
test2 + unnest; test3 chaining join. Writes tests/golden/algebra_example.json (data only).

Usage: python tests/golden/make_algebra_golden.py   (needs /root/reference)
"""
import json
import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(ROOT, "oracle", "_ref", "main_algebra_example.out")


def main():
    out = subprocess.run([BIN], check=True, capture_output=True, text=True).stdout
    tests, cur, section = {}, None, None
    for line in out.splitlines():
        m = re.match(r"### void (algebra_test\d)\(\) ###", line)
        if m:
            cur = tests.setdefault(m.group(1), {"L": [], "R": [], "output": [], "counts": {}})
            section = None
            continue
        if cur is None:
            continue
        if line.startswith("-- Relation "):
            section = line.split()[2]
        elif line.startswith("Output tuples"):
            section = "output"
        elif line.startswith("("):
            vals = [int(v) for v in re.match(r"\(([-\d,]+)\)", line).group(1).split(",")]
            cur["output" if section == "output" else section].append(vals)
        else:
            m = re.match(r"\s*(?:count )?(Top|Sel|Scan|Build|Probe|Unnest):?\s+(\d+)", line)
            if m:
                strand = "build" if "Build Strand" in cur.get("_strand", "") else "probe"
                cur["counts"][f"{strand}_{m.group(1)}"] = int(m.group(2))
            if "Strand" in line:
                cur["_strand"] = line
    for t in tests.values():
        t.pop("_strand", None)
        if not t["R"]:
            del t["R"]
    with open(os.path.join(HERE, "algebra_example.json"), "w") as f:
        json.dump({"source": "oracle/_ref/main_algebra_example.out (reference main_algebra_example.cc)",
                   "tests": tests}, f, indent=1)


if __name__ == "__main__":
    main()
