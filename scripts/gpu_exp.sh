# A/B experiments on the default bench line: one bench run per variant (env settings in $@,
# each "NAME:ENV=VAL,ENV2=VAL"); prints the probe-phase and per-kernel times of each.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/exp
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  [ "$envs" = "$spec" ] && envs=""
  timeout -k 10 240 env ${envs//,/ } python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/exp/$name.log 2>&1
  rc=$?
  python3 - "$name" "$rc" <<'PY'
import json, sys
name, rc = sys.argv[1], sys.argv[2]
line = None
for l in open(f"gpurun_out/exp/{name}.log"):
    if l.startswith("{"):
        line = json.loads(l)
if line is None:
    print(name, "rc", rc, "no JSON"); sys.exit(0)
k = line["roofline"]["kernels"]
print(f"{name:12s} rc={rc} probe_ms={line['probe_ms']:.4f} build_ms={line['build_ms']:.4f} "
      + " ".join(f"{n}={v['avg_ms']:.4f}" for n, v in k.items()) + f" ok={line['verified_bit_exact']}")
PY
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ] && exit $rc
done
exit 0
