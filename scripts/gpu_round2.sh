# Round record, part 2: configs C and E (bench lines + kernel stats) and the PMC passes of the
# default config-B bench (HBM traffic per launch for roofline.traffic).
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:-r01}
bash scripts/gpu_configs.sh $TAG || exit 1
bash scripts/gpu_pmc.sh $TAG
