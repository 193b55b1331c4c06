# PMC passes with caller-chosen counter groups over a short bench run (one group per pass).
# usage: bash scripts/gpu_pmc_groups.sh TAG "CNT_A CNT_B" "CNT_C" ... [-- bench args]
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "$1" = "--" ] && shift
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
