# Fused build partition: parity tests, then a same-box A/B of the default line (config B) and config E,
# fused (default) against the two-launch form (--rp-unfused), two rounds each.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-fz}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_part.py "tests/test_gpu_headline.py::test_headline_exp4_equal_reference" \
  "tests/test_gpu_headline.py::test_headline_exp1_all_plans_equal_reference" -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
for round in 1 2; do
  for v in fused unfused; do
    extra=""; [ $v = unfused ] && extra="--rp-unfused"
    for w in B E; do
      timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-mintime $extra > gpurun_out/${TAG}_${w}_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_${w}_$v.log; exit 1; }
      python3 -c "
import json
for l in open('gpurun_out/${TAG}_${w}_$v.log'):
    if l.startswith('{') and 'metric' in l: d=json.loads(l)
print(json.dumps({'w':'$w','v':'$v','round':$round,'build_ms':round(d['build_ms'],4),'probe_ms':round(d['probe_ms'],4),'verified':d.get('verified_bit_exact')}))"
    done
  done
done | tee gpurun_out/${TAG}_ab.jsonl
