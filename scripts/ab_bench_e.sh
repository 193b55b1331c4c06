# Same-box A/B of config E's (WORKLOAD: or C's) bench line (build_ms / probe_ms) over variant libraries:
#   VARIANTS  "default" and/or names under 3d-hashjoin_amd/variants/ (HJ3D_LIB); TAG names the files;
#   ROUNDS    alternating rounds (default 3); KEXPR: the nested / exp4 parity tests run first with
#             every variant.
# One JSON line per run in gpurun_out/${TAG}_${WORKLOAD:-E}_ab.jsonl.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-eab}
VARIANTS=${VARIANTS:-"prev default"}
lib_for() { [ "$1" = default ] && echo "" || echo "$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$1/libhj3d.so"; }
for v in $VARIANTS; do
  HJ3D_LIB=$(lib_for $v) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    -k "${KEXPR:-lookback or nested_agg_build or hot_key or exp4}" -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_tests_$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/${TAG}_tests_$v.log)"
done
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    HJ3D_LIB=$(lib_for $v) timeout -k 10 200 python bench.py --workload ${WORKLOAD:-E} --steps 20 --warmup 3 --no-cpu-baseline --no-mintime > gpurun_out/${TAG}_${WORKLOAD:-E}_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_${WORKLOAD:-E}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_${WORKLOAD:-E}_$v.log').read().strip().splitlines()[-1]); print(json.dumps({'label':'$v','round':$r,'build_ms':d['build_ms'],'probe_ms':d['probe_ms'],'ok':d['verified_bit_exact']}))"
  done
done | tee gpurun_out/${TAG}_${WORKLOAD:-E}_ab.jsonl
