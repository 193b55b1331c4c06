# The driver's GPU tier, run by hand: pytest -m gpu (one process, per-test time limit), then
# smoke(). Output under gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL=${1:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
exit $rc
