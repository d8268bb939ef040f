# A/B of the pipelined bench (tools/pipe_ab.sh; GPU box)
set -o pipefail
run() { timeout -k 10 200 env "$@" python bench.py --no-cpu-baseline > gpurun_out/p.log 2>&1 || exit 1; echo "$* :: $(grep -o '"value": [0-9.]*' gpurun_out/p.log)"; }
for r in 1 2; do
  run RSL_RF_BPC=0
  run RSL_RF_BPC=2
  run RSL_RF_BPC=1
  run RSL_RF_NP=1
done
