#!/bin/bash
# Placement of the offsets / compaction in the pipelined bench (RSL_BENCH_EMIT_BACK 0 / 1 / 2), alternating rounds:
#   tools/emit_ab.sh TAG ROUNDS "0 1"
TAG=${1:-emit}; ROUNDS=${2:-3}; OPTS=${3:-"0 1 2"}
for r in $(seq 1 "$ROUNDS"); do for e in $OPTS; do
  RSL_BENCH_EMIT_BACK=$e timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extra --no-pcie --no-cpu-baseline > gpurun_out/${TAG}_e${e}_$r.json 2>/dev/null || exit 1
done; done
