set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 bash tools/chain_counters.sh > gpurun_out/r2l_chainctr.log 2>&1
