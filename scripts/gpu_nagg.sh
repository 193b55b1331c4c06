# Nested build A/B (LDS aggregation vs key sort) on config C and the Nrs plan, after the GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_nagg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_nagg.log
[ $rc -le 1 ] || exit $rc
for nb in agg sort; do
  timeout -k 10 300 python bench.py --workload C --steps 5 --warmup 1 --nested-build $nb > gpurun_out/c_$nb.log 2>&1; echo "C $nb rc=$?"; tail -1 gpurun_out/c_$nb.log | cut -c1-1000
done
