# One iteration: GPU parity tests, then the profiled bench (kernel trace + stats).
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:-iter}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_${TAG}.log
[ $rc -le 1 ] || exit $rc
bash scripts/gpu_prof.sh ${TAG}
