set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r2n_distab2.log
for i in 1 2; do
  for ts in 1 0; do
    echo "== plain ts=$ts" >> gpurun_out/r2n_distab2.log
    RSL_BENCH_TRAJ_STREAM=$ts timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/r2n_distab2.log 2>&1 || exit 1
    echo "== nccl1 ts=$ts" >> gpurun_out/r2n_distab2.log
    RSL_BENCH_TRAJ_STREAM=$ts RSL_BENCH_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 295$i$ts bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/r2n_distab2.log 2>&1 || exit 1
  done
done
