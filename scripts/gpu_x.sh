cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for v in base ns; do
  L=""; [ $v = ns ] && L="HJ3D_LIB=3d-hashjoin_amd/exp/libns.so"
  timeout -k 10 300 env $L rocprofv3 --kernel-trace --stats -d gpurun_out/prof/x_$v -o run --output-format csv -- python3 bench.py --workload C --steps 3 --warmup 1 > gpurun_out/exp/x_$v.log 2>&1
  echo "$v rc=$?"
  python3 scripts/kstats.py $(find gpurun_out/prof/x_$v -name "*kernel_stats.csv") | grep -E "k_nagg |k_rp_scatter|k_rp_hist"
done
