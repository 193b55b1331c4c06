cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider -k "nested_agg or exp1_plans" 2>&1 | tail -2
for w in "--workload C" "--plan Nrs --no-cpu-baseline"; do
  tag=$(echo $w | tr -d ' -')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/x_$tag -o run --output-format csv -- python3 bench.py $w --steps 3 --warmup 1 > gpurun_out/x_$tag.log 2>&1
  echo "$tag rc=$?"
  python3 scripts/kstats.py $(find gpurun_out/prof/x_$tag -name "*kernel_stats.csv") > gpurun_out/x_$tag.k; grep -E "k_nagg |k_rp_scatter|k_rp_hist" gpurun_out/x_$tag.k
  grep -o '"build_ms": [0-9.]*' gpurun_out/x_$tag.log
done
