# Same-box A/B of the nested (3D) build (scripts/time_nested.py) over variant libraries:
#   VARIANTS  "default" and/or names under 3d-hashjoin_amd/variants/ (HJ3D_LIB)
#   SHAPES    space-separated time_nested.py argument sets, ',' for ' ' (default: config C's Zipf 0.8
#             1e8 / 1e7, uniform 1e8 / 1e7, config D's Nrs shape 1e9 / 1e8)
#   TESTS     optional pytest node ids run first with every variant (parity before timing), KEXPR an
#             optional -k expression for them
#   ROUNDS    rounds over the variants (default 2)
# One JSON line per run in gpurun_out/${TAG}_nested_ab.jsonl.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-ab}
SHAPES=${SHAPES:-"--theta,0.8 --theta,0 --n,1e9,--domain,1e8,--theta,0,--reps,4"}
lib_for() { [ "$1" = default ] && echo "" || echo "$GRAFT_REPO_ROOT/3d-hashjoin_amd/variants/$1/libhj3d.so"; }
if [ -n "$TESTS" ]; then
  for v in $VARIANTS; do
    HJ3D_LIB=$(lib_for $v) timeout -k 10 600 python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
    echo "tests $v: $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
  done
fi
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    for sh in $SHAPES; do
      HJ3D_LIB=$(lib_for $v) timeout -k 10 300 python scripts/time_nested.py --label $v ${sh//,/ } \
        > gpurun_out/${TAG}_run.log 2>&1 || { tail -5 gpurun_out/${TAG}_run.log; exit 1; }
      tail -1 gpurun_out/${TAG}_run.log
    done
  done
done | tee gpurun_out/${TAG}_nested_ab.jsonl
