cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for v in base dh dh2 r2; do
  L=""; [ $v != base ] && L="HJ3D_LIB=3d-hashjoin_amd/exp/lib$v.so"
  for w in C Nrs; do
    a="--workload C"; [ $w = Nrs ] && a="--plan Nrs --no-cpu-baseline"
    timeout -k 10 300 env $L rocprofv3 --kernel-trace --stats -d gpurun_out/prof/x4_${v}_$w -o run --output-format csv -- python3 bench.py $a --steps 3 --warmup 1 > gpurun_out/x4_${v}_$w.log 2>&1
    echo "$v $w rc=$? $(grep -o '"build_ms": [0-9.]*' gpurun_out/x4_${v}_$w.log) $(grep -o '"verified_bit_exact": [a-z]*' gpurun_out/x4_${v}_$w.log)"
    python3 scripts/kstats.py $(find gpurun_out/prof/x4_${v}_$w -name "*kernel_stats.csv") | grep -E "k_nagg "
  done
done
