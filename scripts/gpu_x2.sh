cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/x_nrs -o run --output-format csv -- python3 bench.py --plan Nrs --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/x_nrs.log 2>&1
echo "rc=$?"
python3 scripts/kstats.py $(find gpurun_out/prof/x_nrs -name "*kernel_stats.csv") | head -12
tail -1 gpurun_out/x_nrs.log | cut -c1-300
