# rocprofv3 kernel stats of short bench runs (one per ARGS entry, separated by ';'), named TAG_<i>.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-kp}
i=0
IFS=';' read -ra RUNS <<< "$ARGS"
for a in "${RUNS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_$i -o run --output-format csv -- \
    python3 bench.py $a --no-cpu-baseline --no-mintime > gpurun_out/${TAG}_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_$i.log; exit 1; }
  echo "== $i: $a"
  python3 scripts/kstats.py gpurun_out/prof/${TAG}_$i/run_kernel_stats.csv | head -${TOP:-14}
done
