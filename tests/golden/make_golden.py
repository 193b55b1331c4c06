#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REAL reference.

Runs oracle/_ref/ref_golden.out (built by `make -C oracle ref` from the read-only
sources under /root/reference plus oracle/ref_golden.cc) for every config below
and writes one JSON file per config. Only data (inputs' checksums / small input
columns and the reference's counters, statistics and output checksums) is
committed — never reference source.

Usage: python tests/golden/make_golden.py [name ...]   (needs /root/reference; ~15 min in all,
most of it the two 1e7/1e8 headline configs; names restrict the run)
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_golden.out")

# (name, args); exp1 args = nR nS skew theta t b [dump]; exp4 args = log2R a A b B [dump]
EXP1 = [
    ("exp1_R8_S16_uni", [8, 16, 0, 1.0, 0, 1, "dump"]),            # SURVEY App. A -R 3 -S 4
    ("exp1_R8_S16_zipf", [8, 16, 1, 1.0, 0, 1, "dump"]),
    ("exp1_R1024_S4096_uni", [1024, 4096, 0, 1.0, 0, 1, "dump"]),  # App. A -R 10 -S 12
    ("exp1_R1024_S4096_zipf", [1024, 4096, 1, 1.0, 0, 1, "dump"]),
    ("exp1_R4096_S65536_uni_t2_b2", [4096, 65536, 0, 1.0, 2, 2]),  # App. A -R 12 -S 16 -t 2 -b 2
    ("exp1_R1000_S10000_uni", [1000, 10000, 0, 1.0, 0, 1, "dump"]),  # exact (non power of two) sizes
    ("exp1_R10007_S100003_zipf08_t1_b3", [10007, 100003, 1, 0.8, 1, 3]),
    ("exp1_R65537_S1000000_zipf08", [65537, 1000000, 1, 0.8, 0, 1]),
    ("exp1_R131072_S1048576_zipf1", [131072, 1048576, 1, 1.0, 0, 1]),
    ("exp1_R1_S7_uni", [1, 7, 0, 1.0, 0, 1, "dump"]),                # single key, every probe collides
    ("exp1_R5_S3_uni_b4", [5, 3, 0, 1.0, 0, 4, "dump"]),             # NB = max(5/4, 1) = 1
    ("exp1_R1048576_S8388608_uni", [1048576, 8388608, 0, 1.0, 0, 1]),  # App. A -R 20 -S 23
    # the headline configs at their exact sizes (BASELINE configs B and C; ~7 min each)
    ("exp1_R10000000_S100000000_uni", [10000000, 100000000, 0, 1.0, 0, 1]),
    ("exp1_R10000000_S100000000_zipf08", [10000000, 100000000, 1, 0.8, 0, 1]),
    # BASELINE config A at its exact size (|R| = 1e6, |S| = 1e7)
    ("exp1_R1000000_S10000000_uni", [1000000, 10000000, 0, 1.0, 0, 1]),
    # config D (|R| = 1e8, |S| = 1e9): Csr, the 3D plan Nsr (unique build keys) and the non-unique
    # 3D plans Nrs / NrsNU (build on S.a, NB = #dv(S.a)); ~30 min per pair of plans, ~40 GB of host
    # memory (Crs, the chaining table on S: ~45 GB). Plans already in an existing fixture with the same
    # inputs are kept, not recomputed.
    ("exp1_R100000000_S1000000000_uni", [100000000, 1000000000, 0, 1.0, 0, 1, "nodump", "Csr,Nsr,Nrs,NrsNU,CsrUU,Crs"]),
]
EXP4 = [
    ("exp4_R3_a2_A2_b2_B1", [3, 2, 2, 2, 1, "dump"]),   # App. A print-relations case
    ("exp4_R10_a3_A2_b2_B3", [10, 3, 2, 2, 3, "dump"]),
    ("exp4_R16_a3_A4_b2_B2", [16, 3, 4, 2, 2]),
    ("exp4_R18_a1_A3_b3_B5", [18, 1, 3, 3, 5]),
    ("exp4_R22_a3_A4_b2_B2", [22, 3, 4, 2, 2]),  # config E (SURVEY App. A -R 22 -a 3 -A 4 -b 2 -B 2)
]


def main():
    if not os.path.exists(BIN):
        sys.exit(f"{BIN} missing: run `make -C oracle ref` first (needs /root/reference)")
    only = set(sys.argv[1:])
    for name, args in [(n, ["exp1"] + a) for n, a in EXP1] + [(n, ["exp4"] + a) for n, a in EXP4]:
        if only and name not in only:
            continue
        path = os.path.join(HERE, name + ".json")
        run_args, kept = list(args), {}
        if args[0] == "exp1" and len(args) > 8 and os.path.exists(path):
            # run only the plans the existing fixture lacks; merge after checking the inputs agree
            with open(path) as f:
                old = json.load(f)
            kept = old.get("plans", {})
            missing = [p for p in args[8].split(",") if p not in kept]
            if not missing:
                print("kept", name)
                continue
            run_args[8] = ",".join(missing)
        out = subprocess.run([BIN] + [str(a) for a in run_args], check=True, capture_output=True, text=True).stdout
        d = json.loads(out)
        if kept:
            for key in ("nR", "nS", "numDvSa", "colsum_Rk", "colsum_Sa", "head_Rk", "head_Sa"):
                assert d[key] == old[key], (name, key)
            d["plans"] = {**kept, **d["plans"]}
        d["generator_args"] = args
        with open(path, "w") as f:
            json.dump(d, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
