# PMC passes (one counter group each) over a short config C bench run; prints the k_nagg rows.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SALU" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py --workload C --steps 2 --warmup 1 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 - $OUT/p$i <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r.get("Kernel_Name", "")
    if "k_nagg(" in n or "k_rp_scatter" in n:
        acc[(n.split("(")[0].split("::")[-1], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, sorted(v)[len(v) // 2])
PY
done
