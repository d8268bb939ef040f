# DoA passes per wave (grid size) re-measured in the pipelined chain: 8 (default) vs 4 vs 16, alternating
set -e
for i in 1 2; do
  for p in 8 4 16; do
    RSL_DOA_PPW=$p timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ppw_${p}_$i.json 2>/dev/null
  done
done
