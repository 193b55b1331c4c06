# A round's GPU record, in parts (each call of gpurun fits its limit): TAG names the files
# (profiles/<TAG>_*), PART picks the parts (letters, default "tb"):
#   t  the GPU tier (pytest -m gpu) and smoke
#   b  the default bench line (as the driver runs it), its rocprofv3 kernel stats, PMC passes on it
#   c  configs C and E: bench line, rocprofv3 kernel stats, PMC passes (HBM traffic per phase)
#   d  config D on one GPU (Csr and the non-unique 3D plan Nrs): bench line + kernel stats
#   s  the 8-, 4- and 2-owner splits of config D (scripts/d_shards.py, Csr) with kernel stats, the HBM
#      bytes per probe tuple of the 8-owner split (FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_bytes.py),
#      and the 8-owner split of the non-unique 3D plan Nrs
#   r  the RCCL message-size sweep (scripts/rccl_limits.sh; needs the commdiag variant library)
# Output under gpurun_out/ (copied to profiles/ by hand). Every GPU step has its own time limit;
# the first failing step ends the call.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r04}
PART=${PART:-tb}
mkdir -p gpurun_out/prof
step() { echo "[$(date +%T)] $*"; }
prof() {  # name, bench args...: rocprofv3 kernel stats of a short bench run
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/$name -o run --output-format csv -- \
    python3 bench.py "$@" --no-cpu-baseline --no-mintime > gpurun_out/${name}_prof.log 2>&1 || { tail -20 gpurun_out/${name}_prof.log; exit 1; }
}
if [[ -n $TESTS ]]; then  # a subset of the GPU tier first (pytest node ids / -k expression in TESTS)
  step tests $TESTS
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest_subset.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_subset.log; exit 1; }
  tail -3 gpurun_out/${TAG}_pytest_subset.log
fi
if [[ $PART == *t* ]]; then
  step tests
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
fi
# (PMC passes first: their summary goes into the box's profiles/ too, so the bench line that follows
# cites the PMC file of the same library as roofline.pmc_source, pmc_same_library true)
if [[ $PART == *b* ]]; then
  step rocprof B
  prof ${TAG} --steps 5 --warmup 2
  step pmc B
  bash scripts/gpu_pmc.sh ${TAG} || exit 1
  python scripts/pmc_summary.py ${TAG} --out gpurun_out/${TAG}_pmc.json && cp gpurun_out/${TAG}_pmc.json profiles/ || exit 1
  step bench B
  timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
fi
if [[ $PART == *c* ]]; then
  for w in C E; do
    prof ${TAG}_$w --workload $w --steps 3 --warmup 1
    step pmc $w
    BENCH_ARGS="--workload $w" bash scripts/gpu_pmc.sh ${TAG}_$w || exit 1
    python scripts/pmc_summary.py ${TAG}_$w --workload $w --out gpurun_out/${TAG}_${w}_pmc.json &&
      cp gpurun_out/${TAG}_${w}_pmc.json profiles/ || exit 1
    step bench $w
    timeout -k 10 600 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/${TAG}_$w.log 2>&1 || { tail -20 gpurun_out/${TAG}_$w.log; exit 1; }
    tail -1 gpurun_out/${TAG}_$w.log | cut -c1-300
  done
fi
if [[ $PART == *d* ]]; then
  for plan in Csr Nrs; do
    step bench D $plan
    timeout -k 10 900 python bench.py --workload D --plan $plan --steps 5 --warmup 1 > gpurun_out/${TAG}_D_$plan.log 2>&1 || { tail -20 gpurun_out/${TAG}_D_$plan.log; exit 1; }
    tail -1 gpurun_out/${TAG}_D_$plan.log | cut -c1-300
    prof ${TAG}_D_$plan --workload D --plan $plan --steps 3 --warmup 1
  done
fi
if [[ $PART == *s* ]]; then
  for o in 8 4 2; do
    step d_shards $o owners
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_Dshards$o -o run --output-format csv -- python3 scripts/d_shards.py --parts $o > gpurun_out/${TAG}_D_shards$o.json 2> gpurun_out/${TAG}_D_shards$o.err || { tail -5 gpurun_out/${TAG}_D_shards$o.err; exit 1; }
    tail -c 600 gpurun_out/${TAG}_D_shards$o.json
  done
  step d_shards 8 owners Nrs
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_Dshards8_Nrs -o run --output-format csv -- python3 scripts/d_shards.py --parts 8 --plan Nrs --reps 2 > gpurun_out/${TAG}_D_shards8_Nrs.json 2> gpurun_out/${TAG}_D_shards8_Nrs.err || { tail -5 gpurun_out/${TAG}_D_shards8_Nrs.err; exit 1; }
  tail -c 600 gpurun_out/${TAG}_D_shards8_Nrs.json
  step pmc d_shards
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_Dsh/p$i -o run -- python3 scripts/d_shards.py --reps 1 > gpurun_out/pmc_${TAG}_Dsh_p$i.log 2>&1 || exit 1
  done
  python scripts/pmc_bytes.py ${TAG}_Dsh --runs 3 --out gpurun_out/${TAG}_D_shards_pmc.json
fi
if [[ $PART == *r* ]]; then
  step rccl sweep
  bash scripts/rccl_limits.sh > gpurun_out/${TAG}_rccl_limits.jsonl 2>&1 || { tail -5 gpurun_out/${TAG}_rccl_limits.jsonl; exit 1; }
  cat gpurun_out/${TAG}_rccl_limits.jsonl
fi
step done
