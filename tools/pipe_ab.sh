# A/B of the pipelined bench (tools/pipe_ab.sh; GPU box)
set -o pipefail
run() { timeout -k 10 200 env "$@" python bench.py --no-cpu-baseline > gpurun_out/p.log 2>&1 || exit 1; echo "$* :: $(grep -o '"value": [0-9.]*' gpurun_out/p.log) $(grep -o '"kernel_ms_per_step": {[^}]*}' gpurun_out/p.log | cut -c1-230)"; }
run RSL_BENCH_PIPELINE=0
run RSL_BENCH_PIPELINE=0 RSL_RF_NP=1
run RSL_BENCH_PIPELINE=1
run RSL_BENCH_PIPELINE=1 RSL_RF_NP=1
run RSL_BENCH_PIPELINE=1 RSL_RF_NP=1 RSL_DOA_BPC=3
run RSL_BENCH_PIPELINE=1 RSL_RF_NP=1 RSL_DOA_BPC=2
