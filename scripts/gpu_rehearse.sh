# Multi-GPU bench path rehearsed on ONE GPU: 2 ranks on cuda:0, gloo exchange via host memory.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
N=${1:-2}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N --rehearse --steps 3 --warmup 1 --nR 2000000 --nS 20000000 \
  > gpurun_out/rehearse_$N.log 2>&1
rc=$?
tail -3 gpurun_out/rehearse_$N.log
exit $rc
