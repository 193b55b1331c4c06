# Same-box A/B of bench lines: for each workload in WORKLOADS (default "B E") and each variant in
# VARIANTS ("default", a variant library name under 3d-hashjoin_amd/variants/, or "flag:<bench args>"),
# ROUNDS rounds; one JSON line per run with the build and probe phase times. Optional TESTS: pytest node ids
# run first with every variant library (parity before timing).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-ab}
for v in $VARIANTS; do
  case $v in default|flag:*) continue;; esac
  if [ -n "$TESTS" ]; then
    HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so timeout -k 10 600 python -u -m pytest $TESTS -x -q \
      --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
    echo "tests $v: $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
  fi
done
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    extra=""
    unset HJ3D_LIB
    case $v in
      default) ;;
      flag:*) extra="${v#flag:}"; extra="${extra//,/ }";;
      *) export HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so;;
    esac
    for w in ${WORKLOADS:-B E}; do
      timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-mintime $extra $BENCH_ARGS > gpurun_out/${TAG}_run.log 2>&1 || { tail -5 gpurun_out/${TAG}_run.log; exit 1; }
      python3 -c "
import json
for l in open('gpurun_out/${TAG}_run.log'):
    if l.startswith('{') and 'metric' in l: d=json.loads(l)
print(json.dumps({'w':'$w','v':'$v','round':$round,'build_ms':round(d['build_ms'],4),'probe_ms':round(d['probe_ms'],4),'verified':d.get('verified_bit_exact')}))"
    done
  done
done | tee gpurun_out/${TAG}_ab.jsonl
