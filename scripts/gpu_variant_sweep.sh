# Build-parameter sweep: workload $WL (default C) with the default library and variant builds under
# 3d-hashjoin_amd/variants/<name>/libhj3d.so (HJ3D_LIB selects the library the host loads);
# VARIANTS names them (default: every variant but the commdiag diagnostic build).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/sweep
VARIANTS=${VARIANTS:-$(ls 3d-hashjoin_amd/variants | grep -v '^commdiag$')}
for v in default $VARIANTS; do
  if [ $v = default ]; then unset HJ3D_LIB; else export HJ3D_LIB=$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$v/libhj3d.so; fi
  timeout -k 10 200 python bench.py --workload ${WL:-C} --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-mintime $BENCH_ARGS > gpurun_out/sweep/$v.log 2>&1 || { tail -5 gpurun_out/sweep/$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sweep/$v.log').read().strip().splitlines()[-1]); print('$v build_ms', round(d['build_ms'],3), 'probe_ms', round(d['probe_ms'],3), {k: round(x['avg_ms'],3) for k, x in d['roofline'].get('kernels', {}).items()}, 'exact', d['verified_bit_exact'])"
done
