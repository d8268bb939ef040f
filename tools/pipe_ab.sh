# A/B of the pipelined bench (tools/pipe_ab.sh; GPU box)
set -o pipefail
run() { timeout -k 10 200 env "$@" python bench.py --no-cpu-baseline > gpurun_out/p.log 2>&1 || exit 1; echo "$* :: $(grep -o '"value": [0-9.]*' gpurun_out/p.log) $(grep -o '"doa_scan": [0-9.]*' gpurun_out/p.log | tr '\n' ' ')"; }
for ppw in 0 2 4 8; do
  run RSL_BENCH_PIPELINE=0 RSL_DOA_PPW=$ppw
  run RSL_BENCH_PIPELINE=1 RSL_DOA_PPW=$ppw
done
