# Same-box A/B of bench.py --workload ${WORKLOAD:-C} (probe + unnest phase) between the working tree library and variants (VARIANTS).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
for round in 1 2; do
  for v in default $VARIANTS; do
    if [ $v = default ]; then unset HJ3D_LIB; else export HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so; fi
    timeout -k 10 300 python bench.py --workload ${WORKLOAD:-C} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-mintime $BENCH_ARGS > gpurun_out/abC_$v.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/abC_$v.log'):
    if l.startswith('{') and 'metric' in l: d=json.loads(l)
print(json.dumps({'label':'$v','probe_ms':d['probe_ms'],'build_ms':d['build_ms'],'verified':d.get('verified_bit_exact')}))"
  done
done
