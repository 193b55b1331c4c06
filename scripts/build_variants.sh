# Variant builds of libhj3d.so for A/B sweeps (scripts/gpu_variant_sweep.sh runs them):
#   bash scripts/build_variants.sh name1 "-DFLAG=1 ..." name2 "..."
# Each lands in 3d-hashjoin_amd/variants/<name>/libhj3d.so (objects under build_<name>/).
set -e
cd "$(dirname "$0")/../3d-hashjoin_amd"
rm -rf variants
while [ $# -ge 2 ]; do
  make -s -j8 OBJ=build_$1 LIB=variants/$1/libhj3d.so EXTRA="$2" variants/$1/libhj3d.so &
  shift 2
done
wait
ls variants
