# Workload B plans on one GPU (Csr, Nsr, Nrs) and the multi-GPU code path of each rehearsed with
# 2 ranks on cuda:0 (gloo, host-staged exchange; not a scaling number).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for plan in Csr Nsr Nrs; do
  timeout -k 10 300 python bench.py --plan $plan --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/plan_$plan.log 2>&1 || { tail -5 gpurun_out/plan_$plan.log; exit 1; }
  tail -1 gpurun_out/plan_$plan.log | cut -c1-400
done
for plan in Nsr Nrs; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --rehearse --plan $plan --steps 2 --warmup 1 --nR 2000000 --nS 20000000 \
    > gpurun_out/rehearse_$plan.log 2>&1 || { tail -20 gpurun_out/rehearse_$plan.log; exit 1; }
  grep '^{' gpurun_out/rehearse_$plan.log | cut -c1-400
done
