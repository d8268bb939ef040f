#!/bin/bash
# Chain buffers in flight in the pipelined bench (RSL_BENCH_NBUF 2 / 3), alternating rounds:  tools/nbuf_ab.sh TAG ROUNDS
TAG=${1:-nbuf}; ROUNDS=${2:-4}
for r in $(seq 1 "$ROUNDS"); do for n in 2 3; do
  RSL_BENCH_NBUF=$n timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extra --no-pcie --no-cpu-baseline > gpurun_out/${TAG}_n${n}_$r.json 2>/dev/null || exit 1
done; done
