# A round record (split in three calls so that each fits gpurun's limit): PART=a the GPU tier
# (pytest -m gpu, smoke), the default bench line (as the driver runs it) + its rocprofv3 kernel stats,
# PMC passes on the same code; PART=b configs C, E, D lines with kernel stats; PART=c the 8-owner
# split of config D (scripts/d_shards.py) with its kernel stats and its HBM bytes per probe tuple
# (FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_bytes.py). PART unset: all. Output under gpurun_out/
# (copied to profiles/ by hand).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r03}
PART=${PART:-abc}
mkdir -p gpurun_out/prof
step() { echo "[$(date +%T)] $*"; }
if [[ $PART == *a* ]]; then
  step tests
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
  step bench B
  timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
  step rocprof B
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
  step pmc B
  bash scripts/gpu_pmc.sh ${TAG} || exit 1
fi
if [[ $PART == *b* ]]; then
  for w in C E D; do
    step bench $w
    timeout -k 10 600 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/${TAG}_$w.log 2>&1 || { tail -20 gpurun_out/${TAG}_$w.log; exit 1; }
    tail -1 gpurun_out/${TAG}_$w.log | cut -c1-300
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-mintime > gpurun_out/${TAG}_${w}_prof.log 2>&1 || exit 1
  done
fi
if [[ $PART == *c* ]]; then
  step d_shards
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_Dshards -o run --output-format csv -- python3 scripts/d_shards.py > gpurun_out/${TAG}_D_shards.json 2> gpurun_out/${TAG}_D_shards.err || { tail -5 gpurun_out/${TAG}_D_shards.err; exit 1; }
  tail -c 600 gpurun_out/${TAG}_D_shards.json
  step pmc d_shards
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_Dsh/p$i -o run -- python3 scripts/d_shards.py --reps 1 > gpurun_out/pmc_${TAG}_Dsh_p$i.log 2>&1 || exit 1
  done
  python scripts/pmc_bytes.py ${TAG}_Dsh --runs 3 --out gpurun_out/${TAG}_D_shards_pmc.json
fi
step done
