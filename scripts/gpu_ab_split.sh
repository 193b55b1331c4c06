# Same-box A/B of the packed partitioner's second level (k_pk_split) over variant libraries
# (VARIANTS, "default" = the tree's build): parity tests first, then config D's probe (time_pk.py,
# 1e8 / 1e9, C = 8), a 2-owner rank's received pairs (5e7 / 5e8, C = 4) and config D's Nrs build
# shape (time_nested.py, C = 64). One JSON line per run in gpurun_out/${TAG}_split_ab.jsonl.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-split}
lib_for() { [ "$1" = default ] && echo "" || echo "$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$1/libhj3d.so"; }
# (parity with every variant; KEXPR: the -k expression, TESTS: the files)
for v in $VARIANTS; do
  HJ3D_LIB=$(lib_for $v) timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_pk_levels.py tests/test_gpu_parity.py} \
    -k "${KEXPR:-pk or slice or nested_agg_build or lookback}" -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_tests_$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/${TAG}_tests_$v.log)"
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    HJ3D_LIB=$(lib_for $v) timeout -k 10 300 python scripts/time_pk.py --nR 1e8 --nS 1e9 --reps 5 --label $v > gpurun_out/${TAG}_run.log 2>&1 || { tail -5 gpurun_out/${TAG}_run.log; exit 1; }
    tail -1 gpurun_out/${TAG}_run.log
    HJ3D_LIB=$(lib_for $v) timeout -k 10 300 python scripts/time_pk.py --nR 5e7 --nS 5e8 --layout pairs --reps 5 --label $v > gpurun_out/${TAG}_run.log 2>&1 || { tail -5 gpurun_out/${TAG}_run.log; exit 1; }
    tail -1 gpurun_out/${TAG}_run.log
    HJ3D_LIB=$(lib_for $v) timeout -k 10 300 python scripts/time_nested.py --label $v --n 1e9 --domain 1e8 --theta 0 --reps 4 > gpurun_out/${TAG}_run.log 2>&1 || { tail -5 gpurun_out/${TAG}_run.log; exit 1; }
    tail -1 gpurun_out/${TAG}_run.log
  done
done | tee gpurun_out/${TAG}_split_ab.jsonl
