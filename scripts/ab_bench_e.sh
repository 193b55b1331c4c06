cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "lookback or nested_agg_build or hot_key or exp4" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lb1_tests.log 2>&1 || { tail -30 gpurun_out/lb1_tests.log; exit 1; }
tail -2 gpurun_out/lb1_tests.log
lib_for() { [ "$1" = default ] && echo "" || echo "$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$1/libhj3d.so"; }
for r in 1 2 3; do
  for v in prev default; do
    HJ3D_LIB=$(lib_for $v) timeout -k 10 200 python bench.py --workload E --steps 20 --warmup 3 --no-cpu-baseline --no-mintime > gpurun_out/lb1_E_$v.log 2>&1 || { tail -5 gpurun_out/lb1_E_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/lb1_E_$v.log').read().strip().splitlines()[-1]); print(json.dumps({'label':'$v','round':$r,'build_ms':d['build_ms'],'probe_ms':d['probe_ms'],'ok':d['verified_bit_exact']}))"
  done
done | tee gpurun_out/lb1_E_ab.jsonl
